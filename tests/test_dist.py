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


def _oracle_solve(sub):
    import oracle as O
    bs, bl, st, rc = O.est(sub.bed, sub.n_ref, sub.n_obs, sub.sigma_s, sub.s_ptr, sub.s_pos,
                           sub.z_s, sub.l_ptr, sub.l_pos, sub.z_l, method="direct")
    return bs, bl, st


def _worker(rank, world, port, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    prob = _problem()
    bs, bl = D.est_distributed(prob, solve=_oracle_solve)
    if rank == 0:
        np.save(out_path, np.concatenate([bs, bl]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_blocks_lpt_balanced_and_complete():
    from dbslmm_amd.dist import block_cost, shard_blocks
    rng = np.random.default_rng(0)
    m = rng.integers(0, 600, size=1703)
    for world in (1, 2, 4, 8):
        sh = shard_blocks(m, 10000, world)
        allb = np.sort(np.concatenate(sh))
        assert np.array_equal(allb, np.flatnonzero(m > 0))
        loads = [block_cost(m[s], 10000).sum() for s in sh]
        assert max(loads) <= sum(loads) / world + block_cost(np.array([m.max()]), 10000)[0]


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
    bs, bl = D.est_distributed(prob, device=0)       # HIP solver on each rank
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


def _gather_worker(rank, world, port, out_path):
    """The bench's per-step path: compact shard per rank, oracle solve, ShardGather (k = 2 solves
    per step, called twice)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here):
        sys.path.insert(0, p)
    import torch.distributed as dist
    from dbslmm_amd import dist as D
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    prob = _problem()
    m = np.diff(prob.s_ptr) + np.diff(prob.l_ptr)
    sub, s_idx, l_idx = D.sub_problem(prob, D.shard_blocks(m, prob.n_ref, world)[rank], compact=True)
    g = D.ShardGather(prob.n_s, prob.n_l, s_idx, l_idx, k=2)
    bs, bl, _ = _oracle_solve(sub)
    for _ in range(2):
        res = g([(bs, bl), (2 * bs, 2 * bl)])
    if rank == 0:
        np.save(out_path, np.stack([np.concatenate(r) for r in res]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shard_gather_per_step(tmp_path, world):
    out = str(tmp_path / "beta.npy")
    mp.spawn(_gather_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    bs, bl, _ = _oracle_solve(_problem())
    ref = np.concatenate([bs, bl])
    np.testing.assert_array_equal(got[0], ref)
    np.testing.assert_array_equal(got[1], 2 * ref)
