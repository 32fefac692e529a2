"""GPU parity of the multi-workgroup ("tiled") Cholesky path against the oracle's direct solve
and against the single-workgroup path (the path is chosen per block by m >= dbslmm_options.tiled_min).

Block sizes put the z row (row m of the bordered matrix) at every position that matters inside
its 64-row tile: m % 64 in {0, 1, 31, 32, 33, 63}, alone in its own tile (m % 64 == 0), plus
blocks with large-effect SNPs and a monomorphic SNP."""
import numpy as np
import pytest

import oracle as O
from _common import normwise

pytestmark = pytest.mark.gpu

BASE_SIZES = [128, 129, 159, 160, 161, 191, 192, 575, 640, 703, 1000]
SIZES = BASE_SIZES + [4100]   # 4100: 512-column super steps (blocks of m >= 4096)


def _problem(seed=11, n_ref=256, with_large=True, mono_block=None, sizes=BASE_SIZES, miss_rate=0.002):
    from dbslmm_amd import BlockProblem, synth
    SIZES = sizes
    total = sum(SIZES)
    p = synth.simulate(total + 50, n_ref, pop="EUR", chroms=[1, 2], seed=seed, miss_rate=miss_rate,
                       large_every=0)
    rng = np.random.default_rng(seed)
    rows = np.arange(total)
    bid = np.repeat(np.arange(len(SIZES)), SIZES)
    large = np.zeros(total, dtype=bool)
    if with_large:
        for b in range(1, len(SIZES), 2):
            idx = np.flatnonzero(bid == b)
            large[rng.choice(idx, size=1 + b % 3, replace=False)] = True
    z = rng.standard_normal(total)
    z[large] = 6.0 * np.sign(z[large])
    bed = p.bed.copy()
    if mono_block is not None:
        j = int(np.flatnonzero(bid == mono_block)[5])
        nb = (n_ref + 3) // 4
        bed[3 + j * nb: 3 + (j + 1) * nb] = 0xFF
    nbk = len(SIZES)

    def csr(mask):
        idx = np.flatnonzero(mask)
        ptr = np.zeros(nbk + 1, dtype=np.int64)
        np.add.at(ptr, bid[idx] + 1, 1)
        return np.cumsum(ptr), rows[idx].astype(np.int32), z[idx]
    s_ptr, s_pos, z_s = csr(~large)
    kw = {}
    if with_large:
        l_ptr, l_pos, z_l = csr(large)
        kw = dict(l_ptr=l_ptr, l_pos=l_pos, z_l=z_l)
    return BlockProblem(bed=bed, n_ref=n_ref, n_obs=100000, sigma_s=0.5 / total, s_ptr=s_ptr,
                        s_pos=s_pos, z_s=z_s, **kw)


def _solve(prob, tiled_min, monkeypatch=None):
    from dbslmm_amd import DBSLMMFIT
    prob.opts["tiled_min"] = int(tiled_min)
    bs, bl, st = DBSLMMFIT(0).est(prob)
    return np.concatenate([bs, bl]), st


def _oracle(prob):
    O.use_blas(True)
    bs, bl, st, _ = O.est(prob.bed, prob.n_ref, prob.n_obs, prob.sigma_s, prob.s_ptr, prob.s_pos,
                          prob.z_s, prob.l_ptr, prob.l_pos, prob.z_l, tau=prob.tau,
                          method="direct", threads=8)
    return np.concatenate([bs, bl]), st


@pytest.mark.parametrize("with_large", [True, False])
def test_tiled_matches_oracle_and_single_workgroup(monkeypatch, with_large):
    prob = _problem(with_large=with_large, sizes=SIZES)
    ref, _ = _oracle(prob)
    tiled, st_t = _solve(prob, 64, monkeypatch)          # every block on the tiled path
    single, st_s = _solve(prob, 10 ** 9, monkeypatch)    # none
    assert np.all(np.isfinite(tiled))
    assert np.all(st_t == 0) and np.all(st_s == 0)
    assert normwise(tiled, ref) < 1e-10
    assert normwise(tiled, single) < 1e-11
    # per block as well (small blocks must not hide behind the big ones' scale)
    off = 0
    for b, m in enumerate(SIZES):
        ms = int(prob.s_ptr[b + 1] - prob.s_ptr[b])
        ml = m - ms
        sl = np.r_[prob.s_ptr[b]:prob.s_ptr[b + 1]]
        assert normwise(tiled[sl], ref[sl]) < 1e-9, (b, m)
        if prob.l_ptr is not None and ml:
            ll = prob.n_s + np.r_[prob.l_ptr[b]:prob.l_ptr[b + 1]]
            assert normwise(tiled[ll], ref[ll]) < 1e-9, (b, m)
        off += m


def test_tiled_monomorphic_block_is_nan(monkeypatch):
    prob = _problem(mono_block=8)
    tiled, st = _solve(prob, 64, monkeypatch)
    sl = np.r_[prob.s_ptr[8]:prob.s_ptr[9]]
    assert st[8] == 3
    assert np.all(np.isnan(tiled[sl]))
    others = np.ones(prob.n_s, dtype=bool)
    others[sl] = False
    assert np.all(np.isfinite(tiled[:prob.n_s][others]))


def test_tiled_plan_rerun_bit_identical(monkeypatch):
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=3, sizes=SIZES)
    prob.opts["tiled_min"] = 128
    plan = Plan(Context(0), prob)
    wl = plan.workload()
    assert wl["blocks_tiled"] == len(SIZES) and wl["tiled_launches"] > 0
    plan.run()
    a = plan.download()
    for _ in range(3):
        plan.run()
    b = plan.download()
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("miss", [0.0, 0.01])
@pytest.mark.parametrize("n_ref", [200, 333])
def test_gram_kernels_bit_identical(monkeypatch, miss, n_ref):
    """The 256x256 (m >= gram_huge_min), 128x128 (m >= gram_big_min) and per-wave
    32x32 Gram kernels compute the same exact integers and the same fp64 epilogue: beta must
    agree bit for bit whichever kernel handles every block."""
    from dbslmm_amd import DBSLMMFIT, synth
    p = synth.simulate(6000, n_ref, pop="EUR", chroms=[1], seed=7, miss_rate=miss, large_every=3)
    prob = synth.make_problem(p)
    out = []
    for big, huge in ((1, 1), (1, 10 ** 9), (10 ** 9, 10 ** 9)):
        prob.opts.update(gram_big_min=big, gram_huge_min=min(huge, 2 ** 31 - 1))
        out.append(DBSLMMFIT(0).est(prob))
    for other in out[1:]:
        for x, y in zip(out[0], other):
            np.testing.assert_array_equal(x, y)
    ref, _ = _oracle(prob)
    assert normwise(np.concatenate(out[0][:2]), ref) < 1e-10


@pytest.mark.parametrize("tiled_min", ["64", "512"])
def test_run_multi_merged_copies_bit_identical(monkeypatch, tiled_min):
    """h2f tuning factors device copies of the Gram in ONE merged tiled sequence (block ids
    b + c * nb): each copy must equal a fresh single-sigma plan bit for bit, with the monomorphic
    block NaN in every copy; a plain run afterwards (copy 0 again) and the variance-holding copy
    (the last sigma) stay consistent."""
    from dbslmm_amd import Context, DBSLMMFIT, Plan
    prob = _problem(seed=5, mono_block=3)
    prob.opts.update(tiled_min=int(tiled_min), h2f_mode=1)   # the merged path (test_h2f_cheb.py: the other)
    plan = Plan(Context(0), prob)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    multi = plan.run_multi(sig)
    fit = DBSLMMFIT(0)
    for f, (bs, bl, st) in zip(sig, multi):
        prob.sigma_s = f
        rs, rl, rst = fit.est(prob)
        np.testing.assert_array_equal(bs, rs)
        np.testing.assert_array_equal(bl, rl)
        np.testing.assert_array_equal(st, rst)
        assert st[3] == 3
    prob.sigma_s = sig[2]
    last = plan.download()
    np.testing.assert_array_equal(last[0], multi[2][0])
    plan.set_sigma(sig[0])
    plan.run()
    np.testing.assert_array_equal(plan.download()[0], multi[0][0])


def test_lead_group_bit_identical():
    """The lead group (dbslmm_options.lead_min: the biggest tiled blocks' Gram tiles first, their
    sequence on its own streams beside the rest of the Gram and the other blocks' sequence) only
    reorders work: single solves and h2f runs give the same betas bit for bit as one sequence."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=13, sizes=SIZES)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    res = {}
    for lead in (600, -1):
        prob.opts.update(tiled_min=128, gram_huge_min=384, lead_min=lead)
        plan = Plan(Context(0), prob)
        plan.run()
        one = plan.download()
        multi = plan.run_multi(sig)
        plan.run()
        again = plan.download()
        res[lead] = (one, multi, again)
    (one, multi, again), (one0, multi0, _) = res[600], res[-1]
    for x, y in zip(one, one0):
        np.testing.assert_array_equal(x, y)
    for x, y in zip(again, one0):
        np.testing.assert_array_equal(x, y)
    for c in range(3):
        for x, y in zip(multi[c], multi0[c]):
            np.testing.assert_array_equal(x, y)
    assert np.all(one[2] == 0)


def test_block_beyond_16k_snps():
    """One LD block of 17,000 SNPs (above round 1's 16,320 cap; the tiled path now takes
    m < 32,640): the h2f copies and a plain run against the direct fp64 solve (NumPy Cholesky on
    the host cores, as tests/test_fullscale.py)."""
    from dbslmm_amd import Context, Plan
    from test_fullscale import _block_ref, _threads
    prob = _problem(seed=17, n_ref=128, sizes=[17000])
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    thr = _threads()
    O.use_blas(True)
    O.blas_threads(thr)
    try:
        ref = _block_ref(prob, 0, sig, thr, pcg=False)["chol"]
    finally:
        O.blas_threads(1)
    plan = Plan(Context(0), prob)
    multi = plan.run_multi(sig)
    for c in range(3):
        assert np.all(multi[c][2] == 0)
        assert normwise(np.concatenate([multi[c][0], multi[c][1]]), ref[c]) < 1e-9, c
    plan.set_sigma(sig[1])
    plan.run()
    bs, bl, st = plan.download()
    assert np.all(st == 0)
    assert normwise(np.concatenate([bs, bl]), ref[1]) < 1e-9


def test_block_at_tiled_size_cap():
    """One LD block of 32,639 SNPs, the largest the tiled path takes (m < 32,640 = 255 x 128):
    the 128-row tile / region indices reach 254 and the substitution's 64-row tile count 510, at
    the edges of the packed work-item fields.  Chebyshev h2f copies vs the direct
    fp64 solve; one SNP more is rejected at plan creation with the stated error."""
    from dbslmm_amd import Context, DbslmmError, Plan
    from test_fullscale import _block_ref, _threads
    cap = 255 * 128
    prob = _problem(seed=19, n_ref=128, sizes=[cap - 1])
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    ctx = Context(0)
    plan = Plan(ctx, prob)
    multi = plan.run_multi(sig)
    assert plan.workload()["cheb_iters"] > 0
    plan.close()
    thr = _threads()
    O.use_blas(True)
    O.blas_threads(thr)
    try:
        ref = _block_ref(prob, 0, sig, thr, pcg=False)["chol"]
    finally:
        O.blas_threads(1)
    for c in range(3):
        assert np.all(multi[c][2] == 0)
        assert normwise(np.concatenate([multi[c][0], multi[c][1]]), ref[c]) < 1e-9, c
    over = _problem(seed=19, n_ref=128, sizes=[cap])
    with pytest.raises(DbslmmError, match="m must be < 32640"):
        Plan(ctx, over)


# config 3 (500k x 5k) failed once on the driver's box -- block 1453 (m = 2659), in a
# lead group that mixes 512-column (m >= 4096) and 256-column super steps -- and passed on others.
LEAD_MIX = [4500, 2600, 800, 900, 1200, 300, 150, 40]


@pytest.mark.parametrize("delay_us", [0, 300, -300])
def test_lead_group_mixed_widths_under_delays(delay_us):
    """A lead group mixing super-step widths (4500 SNPs: R = 4, 2600: R = 2) beside rest blocks on
    the other streams, each run on a FRESH plan (its first run, right after plan_create's
    memsets).  dbslmm_options.debug_delay_us holds one side of every cross-stream dependency back
    (> 0: the bulk trailing launches, the rest sequence and the main stream after the lead fork;
    < 0: the chain launches and the lead sequence), so a missing event fails deterministically
    instead of on one box in four.  Betas must be bit-identical to the undelayed run and match the
    oracle's direct solve per block."""
    from dbslmm_amd import Context, Plan
    # (no missing calls: the Gram takes the LDS-DMA path of dbslmm_gram_huge, as at configs 3-5)
    prob = _problem(seed=23, n_ref=512, sizes=LEAD_MIX, miss_rate=0.0)
    prob.opts["debug_delay_us"] = 0
    plan = Plan(Context(0), prob)
    plan.run()
    ref_gpu = plan.download()
    plan.close()
    assert np.all(ref_gpu[2] == 0)
    if delay_us == 0:
        ref, _ = _oracle(prob)
        got = np.concatenate(ref_gpu[:2])
        for b in range(len(LEAD_MIX)):
            sl = np.r_[prob.s_ptr[b]:prob.s_ptr[b + 1]]
            ll = prob.n_s + np.r_[prob.l_ptr[b]:prob.l_ptr[b + 1]]
            idx = np.concatenate([sl, ll])
            assert normwise(got[idx], ref[idx]) < 1e-10, (b, LEAD_MIX[b])
        return
    prob.opts["debug_delay_us"] = delay_us
    for _ in range(2):
        plan = Plan(Context(0), prob)
        plan.run()
        got = plan.download()
        plan.close()
        for x, y in zip(got, ref_gpu):
            np.testing.assert_array_equal(x, y)


def test_phase_diagnosis_of_a_good_block():
    """The per-phase diagnosis tests/test_fullscale.py prints on a mismatch (Sigma after the Gram,
    L, y = L^-1 z, beta; dbslmm_options.debug_stop + dbslmm_plan_block_matrix) must itself hold
    on a correct block: every phase within 1e-10 of the oracle."""
    from test_fullscale import _diagnose, _threads
    prob = _problem(seed=29, n_ref=384, sizes=[2600, 700])
    thr = _threads()
    O.use_blas(True)
    O.blas_threads(thr)
    try:
        for b in range(2):
            d = _diagnose(prob, b, prob.sigma_s, thr)
            assert set(d) == {"sigma", "L", "L_diag", "y", "beta"}, d
            assert max(d.values()) < 1e-10, (b, d)
    finally:
        O.blas_threads(1)


def test_outputs_refused_after_debug_stop():
    """A debug_stop = 1 run stops after the Gram: its betas are never computed, so download and
    run_multi's outputs must be refused (E_STATE), not served from an earlier run or uninitialised
    memory; a following full run serves them again."""
    from dbslmm_amd import Context, DbslmmError, Plan
    prob = _problem(seed=41, n_ref=256, sizes=[700, 300, 40])
    plan = Plan(Context(0), prob)
    plan.run()
    good = plan.download()
    plan.close()
    prob.opts["debug_stop"] = 1
    plan = Plan(Context(0), prob)
    plan.run()
    plan.sync()
    assert plan.block_matrix(0).shape[0] >= 700     # the diagnostic read still works
    with pytest.raises(DbslmmError):
        plan.download()
    plan.close()
    prob.opts["debug_stop"] = 0
    plan = Plan(Context(0), prob)
    plan.run()
    for x, y in zip(plan.download(), good):
        np.testing.assert_array_equal(x, y)


def test_fused_cheb_with_lead_group_matches_unfused():
    """cheb_fused = 1 on a plan with a lead group: the fused launch covers all tiled items, so the
    plan turns the split substitutions off (before round 5 the option was silently ignored there);
    the h2f copies equal the per-pass launches bit for bit."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=43, n_ref=512, sizes=LEAD_MIX, miss_rate=0.0)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    res = {}
    for fused in (0, 1):
        prob.opts = dict(cheb_fused=fused, sub_split=-1 if fused == 0 else 0, h2f_iter=1)   # (fused: Chebyshev)
        plan = Plan(Context(0), prob)
        res[fused] = plan.run_multi(sig)
        plan.close()
    for c in range(3):
        for x, y in zip(res[1][c], res[0][c]):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("delay_us", [0, 300, -300])
def test_split_substitutions_bit_identical(delay_us):
    """dbslmm_options.sub_split = 1: the rest group's backward solve and h2f Chebyshev passes run
    on its own stream right after its factorisation, the lead group's on stream2, each with its own
    ticket counter and grid (here 8 / 24 persistent workgroups, fewer than the groups' items).  The
    tile arithmetic is the same, so single solves and h2f copies equal the one-sequence
    substitutions bit for bit -- also with one side of every cross-stream dependency delayed."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=37, n_ref=512, sizes=LEAD_MIX, miss_rate=0.0)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    res = {}
    for split in (-1, 1):
        prob.opts = dict(sub_split=split, sub_grid_lead=8, sub_grid_rest=24,
                         debug_delay_us=delay_us if split == 1 else 0)
        plan = Plan(Context(0), prob)
        plan.run()
        one = plan.download()
        multi = plan.run_multi(sig)
        plan.close()
        res[split] = (one, multi)
    for x, y in zip(res[1][0], res[-1][0]):
        np.testing.assert_array_equal(x, y)
    for c in range(3):
        for x, y in zip(res[1][1][c], res[-1][1][c]):
            np.testing.assert_array_equal(x, y)
    assert np.all(res[1][0][2] == 0)
