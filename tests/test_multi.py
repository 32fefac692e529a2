"""Multi-GPU through the C-ABI (dbslmm_ctx_create_multi): the LD blocks
of one problem sharded over several devices must give the single-device result BIT FOR BIT --
every block is solved by the same kernels on the same data, only on another device.  On the
one-GPU test box the shards share device 0 (device list [0, 0, 0]): the sharding, the compact
per-device .bed images, the concurrent host threads and the scatter back to the caller's order are
exercised exactly as on a node; only the device ordinal repeats.  Reference: the OpenMP block
parallelism of DBSLMMFIT::est, scr/dbslmmfit.cpp:191-220."""
import os

import numpy as np
import pytest

from _common import GOLD, TD, load_bed, normwise

pytestmark = pytest.mark.gpu

DEVS = [0, 0, 0]


def _problem(seed=4, snps=20000, n_ref=600, lmm_only=False, miss=0.001):
    from dbslmm_amd import synth
    p = synth.simulate(snps, n_ref, seed=seed, chroms=[1, 2, 3], miss_rate=miss)
    prob = synth.make_problem(p, lmm_only=lmm_only)
    return p, prob


@pytest.mark.parametrize("lmm_only", [False, True])
def test_sharded_est_bit_identical(lmm_only):
    from dbslmm_amd import DBSLMMFIT
    _, prob = _problem(lmm_only=lmm_only)
    prob.opts["tiled_min"] = 256          # blocks on all three solve paths
    one = DBSLMMFIT(0).est(prob)
    many = DBSLMMFIT(DEVS).est(prob)
    for x, y in zip(one, many):
        np.testing.assert_array_equal(x, y)
    assert np.all(one[2] != 2)


def test_sharded_plan_run_multi_and_shards():
    from dbslmm_amd import Context, Plan
    _, prob = _problem(seed=5)
    prob.opts["tiled_min"] = 256
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    single = Plan(Context(0), prob)
    ref = single.run_multi(sig)
    ctx = Context(DEVS)
    assert ctx.num_devices == len(DEVS)
    plan = Plan(ctx, prob)
    info = plan.shard_info()
    m = np.diff(prob.s_ptr) + np.diff(prob.l_ptr)
    assert np.all((info == -1) == (m == 0))
    assert set(info[m > 0].tolist()) == set(range(len(DEVS)))      # every device got blocks
    # the library's shard plan (time model, dbslmm_shard_plan) is what the context used
    from dbslmm_amd.dist import shard_units
    ud, _ = shard_units(m, prob.n_ref, len(DEVS), 1)
    np.testing.assert_array_equal(info, ud[:, 0])
    for _ in range(2):                                             # repeated runs stay identical
        got = plan.run_multi(sig)
        for (a, b, c), (x, y, z) in zip(got, ref):
            np.testing.assert_array_equal(a, x)
            np.testing.assert_array_equal(b, y)
            np.testing.assert_array_equal(c, z)
    # plain run + download of the plan's own sigma
    plan.run()
    plan.sync()
    single.run()
    single.sync()
    for x, y in zip(plan.download(), single.download()):
        np.testing.assert_array_equal(x, y)
    wl, w1 = plan.workload(), single.workload()
    assert wl["snps"] == w1["snps"] and wl["blocks"] == w1["blocks"]
    plan.enable_timing(True)
    plan.run()
    plan.sync()
    ms, n = plan.kernel_ms()
    assert n == 1 and ms[1] > 0


@pytest.mark.parametrize("h2f", [False, True])
def test_sharded_variance_matches_single(h2f):
    """h2f: the variance follows an h2f run_multi whose last sigma was solved by Chebyshev
    iteration, so every shard re-runs that sigma (a graph capture) before its variance; the
    shards share device 0, where one shard's capture must not meet another's synchronous
    variance setup."""
    from test_variance import synth_variance_case
    from dbslmm_amd import Context, Plan
    prob, tbed, ind, tsp, tlp = synth_variance_case()
    prob.opts["tiled_min"] = 64
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    out, betas = [], []
    for dev in (0, [0, 0], [0, 0, 0]):
        plan = Plan(Context(dev), prob)
        if h2f:
            betas.append(plan.run_multi(sig))
            assert plan.workload()["cheb_iters"] > 0
        else:
            plan.run()
            plan.sync()
        out.append(plan.variance(tbed, ind, tsp, tlp))
    for o in out[1:]:
        np.testing.assert_array_equal(out[0], o)
    for b in betas[1:]:
        for x, y in zip(betas[0], b):
            for u, v in zip(x, y):
                np.testing.assert_array_equal(u, v)


def test_sharded_bed_maf_and_tools():
    from dbslmm_amd import Context, bed_maf, read_snp_std
    one, many = Context(0), Context(DEVS)
    for path, n_ref, n_snp in ((os.path.join(TD, "ref_chr1.bed"), 400, 723),
                               (os.path.join(GOLD, "synth_small", "ref.bed"), 203, 600)):
        bed = load_bed(path)
        np.testing.assert_array_equal(bed_maf(one, bed, n_ref, n_snp), bed_maf(many, bed, n_ref, n_snp))
        rows = list(range(0, n_snp, 11))
        for a, b in zip(read_snp_std(one, bed, n_ref, rows), read_snp_std(many, bed, n_ref, rows)):
            np.testing.assert_array_equal(a, b)


def test_sharded_more_devices_than_blocks():
    """A shard may end up with no block: it must stay idle and harmless."""
    from dbslmm_amd import BlockProblem, DBSLMMFIT
    d = __import__("_common").td_problem(nsnp=996, tau=0.8)     # one LD block
    prob = BlockProblem(bed=d["bed"], n_ref=d["n_ref"], n_obs=d["n_obs"], sigma_s=d["sigma_s"],
                        s_ptr=d["s_ptr"], s_pos=d["s_pos"], z_s=d["z_s"], l_ptr=d["l_ptr"],
                        l_pos=d["l_pos"], z_l=d["z_l"])
    one = DBSLMMFIT(0).est(prob)
    many = DBSLMMFIT([0, 0]).est(prob)
    for x, y in zip(one, many):
        np.testing.assert_array_equal(x, y)
    assert normwise(np.concatenate(one[:2]), np.concatenate(many[:2])) == 0.0


def test_split_h2f_units_match_single_device():
    """shard_copies = 3 on three devices (all device 0 here): the dominant block's three h2f
    copies become (block, copy) units on distinct devices, each factored directly on a context of
    its own beside that device's whole blocks.  Every other block equals the one-device run bit for
    bit, and so does the split block's base copy (the same factorisation and backward solve); its
    other copies are exact solves where the one-device run iterated (Chebyshev to cheb_tol), so
    they agree with it to cheb_tol and with the oracle's direct solve to 1e-10.  One units plan
    per device index (dbslmm_plan_create_units, the torchrun ranks' path) fills the same arrays bit
    for bit; a run_multi with another number of sigmas solves the split block whole."""
    import oracle as O
    from test_dist import _split_problem
    from dbslmm_amd import Context, Plan
    from dbslmm_amd.dist import shard_units
    prob, m = _split_problem()
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    ud, _ = shard_units(m, prob.n_ref, 3, 3)
    split = np.flatnonzero(~np.all(ud == ud[:, :1], axis=1))
    assert split.tolist() == [1] and sorted(ud[1].tolist()) == [0, 1, 2]
    single = Plan(Context(0), prob).run_multi(sig)
    prob.opts["shard_copies"] = 3
    many = Plan(Context(DEVS), prob)
    got = many.run_multi(sig)
    sl = np.r_[prob.s_ptr[1]:prob.s_ptr[2]]
    ll = np.r_[prob.l_ptr[1]:prob.l_ptr[2]]
    keep_s = np.setdiff1d(np.arange(prob.n_s), sl)
    keep_l = np.setdiff1d(np.arange(prob.n_l), ll)
    for c in range(3):
        np.testing.assert_array_equal(got[c][0][keep_s], single[c][0][keep_s])
        np.testing.assert_array_equal(got[c][1][keep_l], single[c][1][keep_l])
        np.testing.assert_array_equal(got[c][2], single[c][2])
        g = np.concatenate([got[c][0][sl], got[c][1][ll]])
        o = np.concatenate([single[c][0][sl], single[c][1][ll]])
        if c == 1:                                       # the base copy (median sigma)
            np.testing.assert_array_equal(g, o)
        else:
            assert normwise(g, o) < 1e-8, c
        rs, rl, _, _ = O.est(prob.bed, prob.n_ref, prob.n_obs, sig[c], prob.s_ptr, prob.s_pos, prob.z_s,
                             prob.l_ptr, prob.l_pos, prob.z_l, method="direct")
        assert normwise(np.concatenate([got[c][0], got[c][1]]), np.concatenate([rs, rl])) < 1e-10, c
    # the torchrun ranks' path: one units plan per device index, each writing its units only
    bs, bl = np.full((3, prob.n_s), np.nan), np.full((3, prob.n_l), np.nan)
    st = np.full((3, prob.num_block), -7, dtype=np.int32)
    for d in range(3):
        u = Plan.units(Context(0), prob, ud, d)
        u.run_multi(sig, out=(bs, bl, st))
        u.close()
    for c in range(3):
        np.testing.assert_array_equal(bs[c], got[c][0])
        np.testing.assert_array_equal(bl[c], got[c][1])
    # two sigmas (!= shard_copies): the split block is solved whole by its copy-0 device
    two = many.run_multi(sig[:2])
    ref2 = Plan(Context(0), prob).run_multi(sig[:2])
    for (a, b, c_), (x, y, z) in zip(two, ref2):
        np.testing.assert_array_equal(a, x)
        np.testing.assert_array_equal(b, y)
        np.testing.assert_array_equal(c_, z)


def test_two_split_blocks_share_one_job_per_device():
    """Two dominant blocks and three devices (all device 0 here): both blocks' h2f copies are split
    over the same 3-device group, so each device runs ONE job holding copy c of both blocks (their
    chains in the same launches).  The base copy of both equals the one-device run bit for bit,
    the other copies agree with it to cheb_tol and with the oracle's direct solve to 1e-10, every
    other block bit for bit; the units plans of the torchrun ranks fill the same arrays."""
    import oracle as O
    from test_dist import _split_problem
    from dbslmm_amd import Context, Plan
    from dbslmm_amd.dist import rank_jobs, shard_units
    prob, m = _split_problem((60, 1600, 80, 1400, 0, 40, 70))
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    ud, _ = shard_units(m, prob.n_ref, 3, 3)
    split = np.flatnonzero(~np.all(ud == ud[:, :1], axis=1))
    assert split.tolist() == [1, 3] and ud[1].tolist() == ud[3].tolist()
    for d in range(3):   # one job per device for the split units
        assert [j for j in rank_jobs(ud, d) if len(j[1]) == 1][0][0].tolist() == [1, 3]
    single = Plan(Context(0), prob).run_multi(sig)
    prob.opts["shard_copies"] = 3
    many = Plan(Context(DEVS), prob)
    got = many.run_multi(sig)
    sl = np.concatenate([np.r_[prob.s_ptr[b]:prob.s_ptr[b + 1]] for b in split])
    ll = np.concatenate([np.r_[prob.l_ptr[b]:prob.l_ptr[b + 1]] for b in split])
    keep_s = np.setdiff1d(np.arange(prob.n_s), sl)
    keep_l = np.setdiff1d(np.arange(prob.n_l), ll)
    for c in range(3):
        np.testing.assert_array_equal(got[c][0][keep_s], single[c][0][keep_s])
        np.testing.assert_array_equal(got[c][1][keep_l], single[c][1][keep_l])
        np.testing.assert_array_equal(got[c][2], single[c][2])
        g = np.concatenate([got[c][0][sl], got[c][1][ll]])
        o = np.concatenate([single[c][0][sl], single[c][1][ll]])
        if c == 1:
            np.testing.assert_array_equal(g, o)
        else:
            assert normwise(g, o) < 1e-8, c
        rs, rl, _, _ = O.est(prob.bed, prob.n_ref, prob.n_obs, sig[c], prob.s_ptr, prob.s_pos, prob.z_s,
                             prob.l_ptr, prob.l_pos, prob.z_l, method="direct")
        assert normwise(np.concatenate([got[c][0], got[c][1]]), np.concatenate([rs, rl])) < 1e-10, c
    bs, bl = np.full((3, prob.n_s), np.nan), np.full((3, prob.n_l), np.nan)
    st = np.full((3, prob.num_block), -7, dtype=np.int32)
    for d in range(3):
        u = Plan.units(Context(0), prob, ud, d)
        u.run_multi(sig, out=(bs, bl, st))
        u.close()
    for c in range(3):
        np.testing.assert_array_equal(bs[c], got[c][0])
        np.testing.assert_array_equal(bl[c], got[c][1])
