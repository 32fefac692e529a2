"""Multi-rank path on CPU: world_size-2 gloo, oracle as the per-rank solver (test only)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from _common import normwise


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem():
    from dbslmm_amd import synth
    p = synth.simulate(1200, 96, pop="EUR", chroms=[21, 22], seed=4, miss_rate=0.002, large_every=3)
    return synth.make_problem(p)


def _oracle_solve(sub, sigmas=None):
    """The oracle's direct solve of a sub-problem: (beta_s, beta_l, status), or with sigmas the
    est_distributed solver callback: [(beta_s, beta_l)] per sigma."""
    import oracle as O
    if sigmas is None:
        bs, bl, st, rc = O.est(sub.bed, sub.n_ref, sub.n_obs, sub.sigma_s, sub.s_ptr, sub.s_pos,
                               sub.z_s, sub.l_ptr, sub.l_pos, sub.z_l, method="direct")
        return bs, bl, st
    out = []
    for sg in sigmas:
        bs, bl, _, _ = O.est(sub.bed, sub.n_ref, sub.n_obs, sg, sub.s_ptr, sub.s_pos, sub.z_s,
                             sub.l_ptr, sub.l_pos, sub.z_l, method="direct")
        out.append((bs, bl))
    return out


def _worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    prob = _problem()
    bs, bl = D.est_distributed(prob, solve=_oracle_solve) or (None, None)
    if rank == 0:
        np.save(out_path, np.concatenate([bs, bl]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_blocks_balanced_and_complete():
    """Single-solve shard plan (dbslmm_shard_plan, host only): every non-empty block on exactly one
    rank, empty blocks nowhere, and the time model's predicted device steps within the largest
    block's cost of each other (LPT)."""
    from dbslmm_amd.dist import shard_blocks, shard_units
    rng = np.random.default_rng(0)
    m = rng.integers(0, 600, size=1703)
    for world in (1, 2, 4, 8):
        sh = shard_blocks(m, 10000, world)
        allb = np.sort(np.concatenate(sh))
        assert np.array_equal(allb, np.flatnonzero(m > 0))
        ud, ms = shard_units(m, 10000, world, 1)
        assert np.all(ud[m == 0] == -1)
        _, one = shard_units(m[m == m.max()][:1], 10000, 1, 1)
        assert ms.max() - ms.min() <= one[0] + 1e-9, (world, ms)


def _config4_blocks():
    from dbslmm_amd import synth
    return synth.block_sizes(1000000, pop="EUR", seed=1)


def test_shard_units_split_largest_blocks_copies():
    """h2f (3 copies): the blocks whose chain exceeds the fair share get one copy per device (three
    distinct devices of a 3-device group); every other block keeps its copies together; every unit
    has a device.  A device's split units all share one h2f copy (one job, chains run together):
    at 4 GPUs both large blocks join the one group, at 8 each has a group of its own."""
    from dbslmm_amd.dist import shard_units
    m = _config4_blocks()
    for world, want_split, groups in ((1, 0, 0), (2, 0, 0), (4, 2, 1), (8, 2, 2)):
        ud, ms = shard_units(m, 10000, world, 3)
        assert np.all((ud >= 0) == (m > 0)[:, None])
        split = np.flatnonzero(~np.all(ud == ud[:, :1], axis=1))
        assert split.size == want_split, (world, split)
        for b in split:
            assert len(set(ud[b].tolist())) == 3          # distinct devices
            assert m[b] >= np.sort(m)[-2]                  # the largest blocks
        # on a device, every split unit has the same copy (two copies would be two jobs sharing
        # the device's hardware queues, their chains one after the other)
        for d in range(world):
            copies = {c for b in split for c in range(3) if ud[b, c] == d}
            assert len(copies) <= 1, (world, d, copies)
        assert len({tuple(ud[b].tolist()) for b in split}) == groups
        assert ms.size == world and np.all(ms > 0)


def test_shard_model_predictions_config4():
    """The time model reproduces the measured one-GPU config-4 step (42-44 ms)
    and the round-5 one-GPU rehearsal of two devices (31.8 ms per device), and predicts the 8-GPU
    step below 16 ms once the two largest blocks' h2f copies are split;
    configs 3 / 5 at one GPU: 8.6 / 34 ms measured (the model over-predicts config 3's single
    solve: its chain constants are config 4's)."""
    from dbslmm_amd import synth
    from dbslmm_amd.dist import shard_units
    m4 = _config4_blocks()
    assert 38.0 < shard_units(m4, 10000, 1, 3)[1].max() < 48.0
    assert 28.0 < shard_units(m4, 10000, 2, 3)[1].max() < 36.0
    assert shard_units(m4, 10000, 8, 3)[1].max() < 16.0
    m3 = synth.block_sizes(500000, pop="EUR", seed=1)
    assert 7.0 < shard_units(m3, 5000, 1, 1)[1].max() < 12.5
    m5 = synth.block_sizes(1000000, pop="AFR", seed=1)
    assert 28.0 < shard_units(m5, 10000, 1, 1)[1].max() < 40.0


def test_rank_jobs_cover_every_unit_once():
    from dbslmm_amd.dist import rank_jobs, shard_units
    m = _config4_blocks()
    world = 8
    ud, _ = shard_units(m, 10000, world, 3)
    seen = np.zeros(ud.shape, dtype=int)
    for r in range(world):
        for blocks, copies in rank_jobs(ud, r):
            assert len(copies) in (1, 3)
            for c in copies:
                seen[blocks, c] += 1
    assert np.all(seen[m > 0] == 1) and np.all(seen[m == 0] == 0)


def test_sub_problem_roundtrip():
    from dbslmm_amd.dist import sub_problem
    prob = _problem()
    sub, s_idx, l_idx = sub_problem(prob, np.array([0, 3, 5]))
    assert sub.num_block == 3
    assert np.array_equal(sub.s_pos, prob.s_pos[s_idx])
    assert np.array_equal(sub.z_l, prob.z_l[l_idx])


def test_two_rank_gloo_matches_single_process(tmp_path):
    out = str(tmp_path / "beta.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    prob = _problem()
    bs, bl, _ = _oracle_solve(prob)
    ref = np.concatenate([bs, bl])
    assert got.shape == ref.shape
    assert normwise(got, ref) == 0.0      # same solver, same blocks: bit-identical


def _gpu_worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    sys.path.insert(0, here)
    import torch
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    prob = _problem()
    bs, bl = D.est_distributed(prob, device=0) or (None, None)   # HIP solver on each rank
    if rank == 0:
        np.save(out_path, np.concatenate([bs, bl]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_two_rank_gpu_shards_match_single_gpu(tmp_path):
    from dbslmm_amd import DBSLMMFIT
    out = str(tmp_path / "beta.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    prob = _problem()
    bs, bl, _ = DBSLMMFIT(0).est(prob)
    ref = np.concatenate([bs, bl])
    assert np.all(np.isfinite(got))
    assert normwise(got, ref) < 1e-12
    os_, ol, _ = _oracle_solve(prob)
    assert normwise(got, np.concatenate([os_, ol])) < 1e-10


def test_compact_sub_problem_same_rows():
    """compact=True: the sub-problem's own .bed holds exactly its rows; every SNP's row bytes are
    the full panel's row bytes."""
    from dbslmm_amd.dist import sub_problem
    prob = _problem()
    blocks = np.array([1, 2, 6])
    sub, s_idx, l_idx = sub_problem(prob, blocks, compact=True)
    bps = (prob.n_ref + 3) // 4
    row = lambda bed, r: bed[3 + r * bps: 3 + (r + 1) * bps]
    for i, j in enumerate(s_idx):
        assert np.array_equal(row(sub.bed, sub.s_pos[i]), row(prob.bed, prob.s_pos[j]))
    for i, j in enumerate(l_idx):
        assert np.array_equal(row(sub.bed, sub.l_pos[i]), row(prob.bed, prob.l_pos[j]))
    assert sub.bed.size == 3 + (s_idx.size + l_idx.size) * bps
    a = _oracle_solve(sub)
    b = _oracle_solve(sub_problem(prob, blocks)[0])
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def _split_problem(sizes=(60, 1600, 80, 100, 0, 40, 70)):
    """One dominant block (1600 SNPs) beside small ones: with 3 h2f copies on >= 3 ranks the shard
    plan splits that block's copies over three ranks."""
    from dbslmm_amd import BlockProblem, synth
    sizes = list(sizes)
    total = sum(sizes)
    p = synth.simulate(total + 50, 96, pop="EUR", chroms=[22], seed=6, large_every=0)
    rng = np.random.default_rng(6)
    bid = np.repeat(np.arange(len(sizes)), sizes)
    large = np.zeros(total, dtype=bool)
    large[rng.choice(total, size=5, replace=False)] = True
    z = rng.standard_normal(total)
    z[large] *= 6.0

    def csr(mask):
        idx = np.flatnonzero(mask)
        ptr = np.zeros(len(sizes) + 1, dtype=np.int64)
        np.add.at(ptr, bid[idx] + 1, 1)
        return np.cumsum(ptr), idx.astype(np.int32), z[idx]
    s_ptr, s_pos, z_s = csr(~large)
    l_ptr, l_pos, z_l = csr(large)
    prob = BlockProblem(bed=p.bed, n_ref=96, n_obs=100000, sigma_s=0.5 / total, s_ptr=s_ptr, s_pos=s_pos,
                        z_s=z_s, l_ptr=l_ptr, l_pos=l_pos, z_l=z_l)
    return prob, np.array(sizes)


def _gather_worker(rank, world, port, out_path, k):
    """The bench's per-step path: this rank's units of the shard plan (k h2f copies), oracle solve
    of each job, UnitGather called twice."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    prob, m = _split_problem()
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)[:k]]
    ud, _ = D.shard_units(m, prob.n_ref, world, k)
    bs = np.zeros((k, prob.n_s))
    bl = np.zeros((k, prob.n_l))
    for blocks, copies in D.rank_jobs(ud, rank):
        sub, s_idx, l_idx = D.sub_problem(prob, blocks, compact=True)
        for c, (s, l) in zip(copies, _oracle_solve(sub, [sig[c] for c in copies])):
            bs[c, s_idx] = s
            bl[c, l_idx] = l
    g = D.UnitGather(prob, ud)
    for _ in range(2):
        res = g(bs, bl)
    if rank == 0:
        np.save(out_path, np.stack([np.concatenate(r) for r in res]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,k", [(2, 1), (3, 3)])
def test_unit_gather_per_step(tmp_path, world, k):
    """world 3, k 3: the dominant block's copies are split over the three ranks (asserted); the
    gathered betas equal the single-process oracle solve of every copy bit for bit."""
    from dbslmm_amd.dist import shard_units
    prob, m = _split_problem()
    ud, _ = shard_units(m, prob.n_ref, world, k)
    split = np.flatnonzero(~np.all(ud == ud[:, :1], axis=1))
    assert (split.size > 0) == (k == 3), split
    out = str(tmp_path / "beta.npy")
    mp.spawn(_gather_worker, args=(world, _free_port(), out, k), nprocs=world, join=True)
    got = np.load(out)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)[:k]]
    for c, (bs, bl) in enumerate(_oracle_solve(prob, sig)):
        np.testing.assert_array_equal(got[c], np.concatenate([bs, bl]))


@pytest.mark.gpu
def test_unit_gather_device_scatter_rccl():
    """The nccl (RCCL) path of UnitGather -- received segments scattered on the device, one copy
    into pinned memory -- on a world-1 process group: every unit of every copy lands at its
    original position, twice in a row (the reused buffers)."""
    import torch
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        prob, m = _split_problem()
        ud, _ = D.shard_units(m, prob.n_ref, 1, 3)
        g = D.UnitGather(prob, ud, device="cuda")
        rng = np.random.default_rng(5)
        for _ in range(2):
            bs, bl = rng.standard_normal((3, prob.n_s)), rng.standard_normal((3, prob.n_l))
            res = g(bs, bl)
            for c in range(3):
                np.testing.assert_array_equal(res[c][0], bs[c])
                np.testing.assert_array_equal(res[c][1], bl[c])
    finally:
        dist.destroy_process_group()


REHEARSAL = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r06", "shard")
# config -> (SNPs, n_ref, pop, LMM-only, h2f factors, step tolerance, device spread)
_REH = {4: (1_000_000, 10_000, "EUR", False, (0.8, 1.0, 1.2), 0.10, 0.80),
        5: (1_000_000, 10_000, "AFR", True, (1.0,), 0.10, 0.80),
        3: (500_000, 5_000, "EUR", False, (1.0,), 0.10, 0.80)}


@pytest.mark.parametrize("cfg", [4, 5, 3])
def test_pcg_shard_model_matches_rehearsal(cfg):
    """The PCG-route shard plan (dbslmm_shard_plan_problem, host only) against the committed
    one-GPU rehearsal (profiles/r06/shard/rehearsal_c<cfg>.json, tools/r06_dev.py: each device's
    units plan of the N-device plan timed alone on one MI355X, the median of seven batches): the
    plan's device assignment is the rehearsed one, every block whole on one device, the predicted
    step (slowest device) is within 10 % of the measured one at N = 1, 2, 4, 8 for configs 3, 4
    and 5 (measured: within 8 %), and the model's balance keeps every measured device within 20 %
    of the measured step (measured: within 9.2 %)."""
    import json
    from dbslmm_amd import synth
    from dbslmm_amd.dist import shard_units_problem
    snps, n_ref, pop, lmm, f, tol, spread = _REH[cfg]
    rec = json.load(open(os.path.join(REHEARSAL, f"rehearsal_c{cfg}.json")))
    prob = synth.make_problem(synth.simulate(snps, n_ref, pop=pop, seed=1, engine="none"), lmm_only=lmm)
    sig = [prob.sigma_s * x for x in f]
    for N, devs in rec["results"].items():
        N = int(N)
        ud, ms = shard_units_problem(prob, sig, N)
        assert np.all(ud == ud[:, :1])                              # whole blocks
        for d, dv in enumerate(devs):
            assert np.array_equal(np.flatnonzero(ud[:, 0] == d), dv["block_ids"]), (N, d)
        wall = np.array([dv["wall_ms"] for dv in devs])
        step, pred = wall.max(), ms.max()
        assert abs(pred - step) <= tol * step, (cfg, N, pred, step)
        assert wall.min() >= spread * step, (cfg, N, wall)
