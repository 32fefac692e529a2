"""h2f tuning by Chebyshev iteration on one factor (trsv.hip): for the tiled blocks only the base
copy (median sigma) is factored; the other copies iterate M_b x = z - delta P_s x with the
persistent forward / backward substitution kernels.  Every copy must match a fresh single-sigma
solve within the iteration's target (cheb_tol, default 1e-9; checked at normwise CHEB_TOL), the base copy
bit for bit; statuses and the NaN of a
monomorphic block carry over; the merged-factorisation path (h2f_mode = 1) stays
bit-identical."""
import numpy as np
import pytest

from _common import CHEB_TOL, normwise
from test_tiled import _oracle, _problem

pytestmark = pytest.mark.gpu


def _fresh(prob, sig):
    from dbslmm_amd import DBSLMMFIT
    fit = DBSLMMFIT(0)
    out = []
    for f in sig:
        prob.sigma_s = f
        out.append(fit.est(prob))
    return out


def _cat(r):
    return np.concatenate([r[0], r[1]])


def _finite_normwise(a, b):
    ok = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), ok)
    return normwise(a[ok], b[ok])


@pytest.mark.parametrize("tiled_min", ["64", "512"])
@pytest.mark.parametrize("factors", [(0.8, 1.0, 1.2), (1.2, 0.8), (0.5, 0.7, 1.0, 1.3, 1.6, 2.0)])
def test_cheb_copies_match_fresh_solves(monkeypatch, tiled_min, factors):
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=5, mono_block=3)
    prob.opts.update(tiled_min=int(tiled_min), h2f_iter=1)   # Chebyshev (CG: test_cg_*)
    s0 = prob.sigma_s
    sig = [s0 * f for f in factors]
    plan = Plan(Context(0), prob)
    multi = plan.run_multi(sig)
    fresh = _fresh(prob, sig)
    base = int(np.argsort(sig, kind="stable")[len(sig) // 2])
    for c, (got, ref) in enumerate(zip(multi, fresh)):
        np.testing.assert_array_equal(got[2], ref[2])
        assert got[2][3] == 3
        if c == base:
            np.testing.assert_array_equal(_cat(got), _cat(ref))
        else:
            assert _finite_normwise(_cat(got), _cat(ref)) < CHEB_TOL, c
    # against the oracle's direct solve of the reference equations too
    prob.sigma_s = sig[0]
    ref, _ = _oracle(prob)
    ok = np.isfinite(ref) & np.isfinite(_cat(multi[0]))
    assert normwise(_cat(multi[0])[ok], ref[ok]) < CHEB_TOL   # (copy 0: iterated)


def test_cheb_off_is_bit_identical(monkeypatch):
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=6)
    prob.opts.update(tiled_min=64, h2f_mode=1)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    multi = Plan(Context(0), prob).run_multi(sig)
    for got, ref in zip(multi, _fresh(prob, sig)):
        np.testing.assert_array_equal(_cat(got), _cat(ref))


def test_cheb_repeatable_and_followed_by_plain_run(monkeypatch):
    """Two h2f runs give identical betas (fixed iteration count, fixed reduction order), and a
    plain run afterwards equals a fresh single-sigma plan."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=8)
    prob.opts["tiled_min"] = 64
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(Context(0), prob)
    a = plan.run_multi(sig)
    b = plan.run_multi(sig)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(_cat(x), _cat(y))
    plan.set_sigma(sig[0])
    plan.run()
    got = plan.download()
    ref = _fresh(prob, sig[:1])[0]
    np.testing.assert_array_equal(_cat(got), _cat(ref))


def test_run_multi_into_caller_buffers():
    """Plan.run_multi(out=...) writes the same results into the caller's (reused) arrays."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=7)
    prob.opts["tiled_min"] = 256
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(Context(0), prob)
    ref = plan.run_multi(sig)
    out = (np.full((3, prob.n_s), 7.0), np.full((3, prob.n_l), 7.0), np.full((3, prob.num_block), 9, dtype=np.int32))
    for _ in range(2):
        got = plan.run_multi(sig, out=out)
        for (a, b, c), (x, y, z) in zip(got, ref):
            np.testing.assert_array_equal(a, x)
            np.testing.assert_array_equal(b, y)
            np.testing.assert_array_equal(c, z)
    with pytest.raises(ValueError):
        plan.run_multi(sig, out=(out[0][:2], out[1], out[2]))


@pytest.mark.parametrize("cheb_tol", [1e-7, 1e-9, 1e-11])
def test_cheb_error_within_target(cheb_tol):
    """The iteration count is fixed on the host from dbslmm_options.cheb_tol (error <= 2 q^K x the
    initial error): every iterated copy must land within 10 x cheb_tol of
    a fresh single-sigma solve, normwise (a bound tied to the target, so a change of
    cheb_tol or of the iteration bounds cannot drift unnoticed), and a tighter target must not
    take fewer iterations."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=9)
    prob.opts.update(tiled_min=64, cheb_tol=cheb_tol, h2f_iter=1)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(Context(0), prob)
    multi = plan.run_multi(sig)
    iters = plan.workload()["cheb_iters"]
    assert iters > 0
    for c, (got, ref) in enumerate(zip(multi, _fresh(prob, sig))):
        assert _finite_normwise(_cat(got), _cat(ref)) <= 10 * cheb_tol, (c, iters)
    if cheb_tol < 1e-7:
        loose = dict(prob.opts, cheb_tol=cheb_tol * 100)
        prob.opts = loose
        p2 = Plan(Context(0), prob)
        p2.run_multi(sig)
        assert p2.workload()["cheb_iters"] < iters


@pytest.mark.parametrize("factors", [(0.8, 1.0, 1.2), (0.5, 0.7, 1.0, 1.3, 1.6, 2.0)])
def test_fused_cheb_launch_bit_identical(monkeypatch, factors):
    """dbslmm_options.cheb_fused = 1 runs all 2K passes of a copy group in one dbslmm_trsv_cheb launch
    (items of every pass interleaved across blocks, own-input waits on flags); the arithmetic is
    the per-pass kernels' own, so the betas are bit-identical (groups of 2 and of 1 copy)."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=5, mono_block=3)
    prob.opts.update(tiled_min=64, h2f_iter=1)   # the fused launch iterates by Chebyshev
    sig = [prob.sigma_s * f for f in factors]
    ref = Plan(Context(0), prob).run_multi(sig)
    prob.opts["cheb_fused"] = 1
    plan = Plan(Context(0), prob)
    for _ in range(2):   # the cached work list is reused
        got = plan.run_multi(sig)
        for x, y in zip(got, ref):
            np.testing.assert_array_equal(_cat(x), _cat(y))
            np.testing.assert_array_equal(x[2], y[2])


@pytest.mark.parametrize("large_cheb", [0, -1])
def test_large_blocks_above_cheb_kernel_size(large_cheb):
    """with tiled_min above 512, blocks of 512 <= m < tiled_min stay on the
    single-workgroup path (dbslmm_chol_large) but no longer fit the h2f iteration kernel
    (dbslmm_chol_cheb keeps ld <= 512 vectors in LDS): their h2f copies must then be factored, not
    iterated.  Every copy against a fresh single-sigma solve at CHEB_TOL (the base copy bit for
    bit), and large_cheb = -1 (every copy factored) against the same."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=21, sizes=[300, 520, 700, 999, 130])
    prob.opts.update(tiled_min=100000, large_cheb=large_cheb)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    multi = Plan(Context(0), prob).run_multi(sig)
    fresh = _fresh(prob, sig)
    base = int(np.argsort(sig, kind="stable")[len(sig) // 2])
    for c, (got, ref) in enumerate(zip(multi, fresh)):
        np.testing.assert_array_equal(got[2], ref[2])
        assert np.all(got[2] == 0)
        if c == base:
            np.testing.assert_array_equal(_cat(got), _cat(ref))
        else:
            assert normwise(_cat(got), _cat(ref)) < CHEB_TOL, c


@pytest.mark.parametrize("factors", [(0.8, 1.0, 1.2), (1.2, 0.8), (0.5, 0.7, 1.0, 1.3, 1.6)])
def test_whole_block_cheb_for_rest_group(factors):
    """dbslmm_options.sub_split = 2: the rest group's h2f copies iterate in dbslmm_tcheb (one
    workgroup per block, all passes in one launch, butterfly row sums) instead of the per-pass tile
    items.  A lead group (4500, 2600) and a rest group of tiled blocks (800, 900, 1200, one with a
    monomorphic SNP) with tiled_min 256.  Every copy against a fresh single-sigma solve at
    CHEB_TOL, the base copy and the lead group's blocks bit for bit against sub_split = 1, statuses
    (and the monomorphic SNP's NaN) identical."""
    from dbslmm_amd import Context, Plan
    from test_tiled import LEAD_MIX
    prob = _problem(seed=41, n_ref=512, sizes=LEAD_MIX, miss_rate=0.0, mono_block=3)
    prob.opts = dict(tiled_min=256)
    sig = [prob.sigma_s * f for f in factors]
    res = {}
    for split in (1, 2):
        prob.opts["sub_split"] = split
        plan = Plan(Context(0), prob)
        res[split] = plan.run_multi(sig)
        plan.close()
    prob.opts = dict(tiled_min=256)
    fresh = _fresh(prob, sig)
    base = int(np.argsort(sig, kind="stable")[len(sig) // 2])
    n_lead = LEAD_MIX[0] + LEAD_MIX[1]
    for c, (got, old, ref) in enumerate(zip(res[2], res[1], fresh)):
        np.testing.assert_array_equal(got[2], old[2])
        np.testing.assert_array_equal(got[2], ref[2])
        if c == base:
            np.testing.assert_array_equal(_cat(got), _cat(old))
        else:
            assert _finite_normwise(_cat(got), _cat(ref)) < CHEB_TOL, c
            # the lead group's small-effect betas (its blocks come first) are unchanged
            np.testing.assert_array_equal(got[0][:n_lead - 8], old[0][:n_lead - 8])


@pytest.mark.parametrize("tiled_min", ["64", "512"])
@pytest.mark.parametrize("factors", [(0.8, 1.0, 1.2), (1.2, 0.8), (0.5, 0.7, 1.0, 1.3, 1.6, 2.0)])
def test_cg_copies_match_fresh_solves(tiled_min, factors):
    """dbslmm_options.h2f_iter = 2: the tiled blocks' copies by preconditioned CG on the base factor
    (dbslmm_cg_update after each backward pass, converged blocks skipped by the later passes).
    Every copy against a fresh single-sigma solve at CHEB_TOL, the base copy bit for bit, statuses
    and the monomorphic block's NaN identical; two runs bit-identical (fixed reduction order)."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=5, mono_block=3)
    prob.opts.update(tiled_min=int(tiled_min), h2f_iter=2)
    sig = [prob.sigma_s * f for f in factors]
    plan = Plan(Context(0), prob)
    multi = plan.run_multi(sig)
    again = plan.run_multi(sig)
    wl = plan.workload()   # the passes the blocks ran before converging, capped by Chebyshev's count
    assert 0 < wl["h2f_pass_bytes"] <= 2 * wl["trsv_bytes"] * wl["cheb_iters"]
    prob.opts.pop("h2f_iter")
    fresh = _fresh(prob, sig)
    base = int(np.argsort(sig, kind="stable")[len(sig) // 2])
    for c, (got, ref, rep) in enumerate(zip(multi, fresh, again)):
        np.testing.assert_array_equal(got[2], ref[2])
        np.testing.assert_array_equal(_cat(got), _cat(rep))
        assert got[2][3] == 3
        if c == base:
            np.testing.assert_array_equal(_cat(got), _cat(ref))
        else:
            assert _finite_normwise(_cat(got), _cat(ref)) < CHEB_TOL, c


@pytest.mark.parametrize("cheb_tol", [1e-7, 1e-11])
def test_cg_error_within_target(cheb_tol):
    """CG's stopping bound |r| <= cheb_tol lambda_min(M_c) |x| bounds each block's relative error:
    every iterated copy within cheb_tol of a fresh solve, normwise (with a 2 x margin for the fresh
    solve's own rounding at the tight target)."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=9)
    prob.opts.update(tiled_min=64, cheb_tol=cheb_tol, h2f_iter=2)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    multi = Plan(Context(0), prob).run_multi(sig)
    prob.opts.pop("h2f_iter")
    for c, (got, ref) in enumerate(zip(multi, _fresh(prob, sig))):
        assert _finite_normwise(_cat(got), _cat(ref)) <= 2 * cheb_tol, c


@pytest.mark.parametrize("split", [-1, 1])
def test_cg_with_lead_group(split):
    """CG on a plan with a lead group (4500, 2600) and a rest group (800, 900, 1200, one block with a
    monomorphic SNP), per-group substitutions (sub_split 1) or one sequence (-1): every copy
    within CHEB_TOL of the Chebyshev run, the base copy and the statuses identical."""
    from dbslmm_amd import Context, Plan
    from test_tiled import LEAD_MIX
    prob = _problem(seed=41, n_ref=512, sizes=LEAD_MIX, miss_rate=0.0, mono_block=3)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    res = {}
    for it in (1, 2):
        prob.opts = dict(tiled_min=256, sub_split=split, h2f_iter=it)
        plan = Plan(Context(0), prob)
        res[it] = plan.run_multi(sig)
        plan.close()
    for c, (got, ref) in enumerate(zip(res[2], res[1])):
        np.testing.assert_array_equal(got[2], ref[2])
        if c == 1:
            np.testing.assert_array_equal(_cat(got), _cat(ref))
        else:
            assert _finite_normwise(_cat(got), _cat(ref)) < CHEB_TOL, c


@pytest.mark.parametrize("tiled_min", ["64", "512"])
def test_cg_cap_reports_not_converged(tiled_min):
    """an h2f copy that stops at the CG cap without meeting |r| <= cheb_tol
    lambda_min |x| was written with BLOCK_OK.  With the cap lowered to one iteration and a tight
    bound, every iterated copy of a tiled (tiled_min 64) or single-workgroup (512) block reports
    DBSLMM_BLOCK_NOT_CONVERGED with a finite iterate; the base copy (factored) stays OK; the
    default cap converges every copy (status OK)."""
    from dbslmm_amd import BLOCK_NOT_CONVERGED, Context, Plan
    prob = _problem(seed=5)
    prob.opts.update(tiled_min=int(tiled_min), solver=1, pcg_maxit=1, cheb_tol=1e-13)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(Context(0), prob)
    out = plan.run_multi(sig)
    base = 1
    m_b = np.diff(prob.s_ptr) + np.diff(prob.l_ptr)
    it_blocks = m_b + 1 > 64          # blocks iterated on the base factor (tiled / chol_large)
    assert it_blocks.sum() > 0
    for c in range(3):
        st = out[c][2]
        assert np.all(np.isfinite(_cat(out[c])))
        if c == base:
            assert np.all(st == 0)
        else:
            assert np.all(st[it_blocks] == BLOCK_NOT_CONVERGED), (c, st)
            assert np.all(st[~it_blocks] == 0)
    plan.close()
    prob.opts.update(pcg_maxit=0, cheb_tol=0.0)
    plan = Plan(Context(0), prob)
    for bs, bl, st in plan.run_multi(sig):
        assert np.all(st == 0)
    plan.close()
