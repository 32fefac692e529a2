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
    # LPT balance: no device holds more than the largest block plus its fair share of the cost
    cost = prob.n_ref * m * (m + 1.0) + m ** 3 / 3.0
    loads = [cost[info == d].sum() for d in range(len(DEVS))]
    assert max(loads) <= cost.sum() / len(DEVS) + cost.max()
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
