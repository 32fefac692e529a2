"""GPU parity of the PCG route (pcg.hip, dbslmm_options.solver): Jacobi-PCG on every block's joint
LD matrix -- the reference's own algorithm (PCGv / PCGm, scr/dbslmmfit.cpp:629-678) -- streamed from
the exact integer Gram (uint16) or, for blocks with missing calls / n_ref > 16383, from the fp64
Sigma.

Bars: normwise <= 1e-10 against the oracle's direct fp64 solve of the reference equations (the
route's stopping rule bounds the relative 2-norm error of each block and copy by pcg_tol = 1e-12),
<= 1e-5 against the reference-faithful PCG golden vectors (BASELINE's criterion), the Manual rows
to one unit in the sixth digit; statuses: MONOMORPHIC blocks NaN as the factor route,
NOT_CONVERGED at the iteration cap with the iterate returned."""
import json
import os

import numpy as np
import pytest

import oracle as O
from _common import GOLD, normwise, synth_small_problem, td_problem
from test_tiled import _oracle, _problem

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(GOLD, "testdat_golden.json")))


def _prob(d, **opts):
    from dbslmm_amd import BlockProblem
    return BlockProblem(bed=d["bed"], n_ref=d["n_ref"], n_obs=d["n_obs"], sigma_s=d["sigma_s"],
                        s_ptr=d["s_ptr"], s_pos=d["s_pos"], z_s=d["z_s"], l_ptr=d.get("l_ptr"),
                        l_pos=d.get("l_pos"), z_l=d.get("z_l"), tau=d.get("tau", 0.8), opts=opts)


def _run(prob, sigmas=None):
    from dbslmm_amd import Context, Plan
    plan = Plan(Context(0), prob)
    if sigmas is None:
        plan.run()
        plan.sync()
        out = [plan.download()]
    else:
        out = plan.run_multi(sigmas)
    wl = plan.workload()
    plan.close()
    return out, wl


def _cat(r):
    return np.concatenate([r[0], r[1]])


def _ok(st, d):
    """status OK on every block with SNPs, EMPTY elsewhere"""
    m = np.diff(d["s_ptr"]) + (np.diff(d["l_ptr"]) if d.get("l_ptr") is not None else 0)
    return bool(np.all(np.where(m > 0, st == 0, st == 1)))


@pytest.mark.parametrize("lmm", [False, True], ids=["dbslmm", "lmm"])
def test_testdat_forced_pcg_matches_oracle_and_golden(lmm):
    """test_dat (the reference's example, one block of 716 SNPs, cond ~124): the auto rule keeps it
    on the factorisation (1/(sigma_s n) = 0.83); forced PCG must still meet every bar."""
    d = td_problem(lmm_only=lmm)
    (res,), wl = _run(_prob(d, solver=2))
    assert wl["pcg_route"] == 1 and wl["pcg_iters"] > 10
    got = _cat(res)
    kind = "lmm" if lmm else "dbslmm"
    gd, gp = GOLDEN[f"{kind}_tau0.8_nsnp996_direct"], GOLDEN[f"{kind}_tau0.8_nsnp996_pcg"]
    assert _ok(res[2], d)
    ref = np.concatenate([gd["beta_s"], gd["beta_l"]])
    assert normwise(got, ref) < 1e-10, normwise(got, ref)
    assert normwise(got, np.concatenate([gp["beta_s"], gp["beta_l"]])) < 1e-5
    # auto: the factorisation route on this panel
    (res2,), wl2 = _run(_prob(d))
    assert wl2["pcg_route"] == 0
    assert normwise(_cat(res2), got) < 1e-10


def test_missing_calls_take_the_fp64_sigma():
    """synth_small: missing calls (mean imputation) and n_ref % 4 = 3; those blocks' products read
    the fp64 Sigma the Gram wrote (the uint16 integer Gram cannot hold the mask terms)."""
    for lmm in (False, True):
        d = synth_small_problem(lmm)
        (res,), wl = _run(_prob(d, solver=2))
        assert wl["pcg_route"] == 1
        ref, _ = _oracle(_prob(d))
        got = _cat(res)
        ok = np.isfinite(ref)
        assert np.array_equal(np.isfinite(got), ok)
        assert normwise(got[ok], ref[ok]) < 1e-10


@pytest.mark.parametrize("factors", [(1.0,), (0.8, 1.0, 1.2), (0.5, 0.8, 1.0, 1.3)])
def test_auto_pcg_h2f_matches_factorisation(factors):
    """A panel whose prior shift puts the auto rule on PCG (d = 1/(sigma_s n) ~ 20, as configs
    3-5): every h2f copy against the factorisation route's direct solve of the same plan inputs
    (solver = 1) and against the oracle; a monomorphic block NaN + MONOMORPHIC as there."""
    prob = _problem(seed=7, n_ref=512, mono_block=4, miss_rate=0.0)
    prob.sigma_s = 0.5 / 1e6        # nsnp = 1M, n = 100 000: d = 20 (config 4)
    sig = [prob.sigma_s * f for f in factors]
    pc, wl = _run(prob, sig)
    assert wl["pcg_route"] == 1 and 5 < wl["pcg_iters"] < 40, wl["pcg_iters"]
    prob.opts["solver"] = 1
    fc, wlf = _run(prob, sig)
    assert wlf["pcg_route"] == 0
    for c in range(len(sig)):
        np.testing.assert_array_equal(pc[c][2], fc[c][2])
        assert pc[c][2][4] == 3
        a, b = _cat(pc[c]), _cat(fc[c])
        ok = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), ok)
        assert normwise(a[ok], b[ok]) < 1e-10, (c, normwise(a[ok], b[ok]))
    prob.opts.pop("solver")
    prob.sigma_s = sig[-1]
    ref, _ = _oracle(prob)
    a = _cat(pc[-1])
    ok = np.isfinite(ref) & np.isfinite(a)     # (the oracle's 0/0 column of the monomorphic block)
    assert normwise(a[ok], ref[ok]) < 1e-10


def test_pcg_repeatable_and_equal_to_single_copy_runs():
    """Bit-identical across runs; every copy of a multi-copy run agrees with a one-copy run of its
    sigma to the stopping bound: one multi-shift Krylov sequence serves every copy of a block
    without large SNPs, and a one-copy run solves each small block whole in dbslmm_pcg_block where
    the multi-copy run iterates the blocks with large SNPs copy by copy on the chip-wide kernels --
    bit for bit only where both runs take the chip-wide kernels (blocks with large SNPs and more
    than 8 tile rows)."""
    from dbslmm_amd import Context, Plan
    prob = _problem(seed=3, n_ref=384, miss_rate=0.0)
    prob.sigma_s = 0.5 / 5e5           # d = 10 (config 3)
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(Context(0), prob)
    a = plan.run_multi(sig)
    b = plan.run_multi(sig)
    for x, y in zip(a, b):
        assert all(np.array_equal(u, v) for u, v in zip(x, y))
    nl = np.diff(prob.l_ptr)
    for c, sg in enumerate(sig):
        (one,), _ = _run(prob, [sg])
        assert np.array_equal(one[2], a[c][2])
        for blk in range(prob.num_block):
            s0, s1, l0, l1 = prob.s_ptr[blk], prob.s_ptr[blk + 1], prob.l_ptr[blk], prob.l_ptr[blk + 1]
            g = np.concatenate([a[c][0][s0:s1], a[c][1][l0:l1]])
            o = np.concatenate([one[0][s0:s1], one[1][l0:l1]])
            m = s1 - s0 + l1 - l0
            if nl[blk] and m > 8 * 128:
                assert np.array_equal(g, o), (c, blk)
            else:
                assert normwise(g, o) < 1e-11, (c, blk, normwise(g, o))
    plan.close()


def test_not_converged_status_at_the_cap():
    """pcg_maxit below what the tolerance needs: every block still above its bound reports
    DBSLMM_BLOCK_NOT_CONVERGED and returns its iterate (finite, already close); blocks that met
    the bound in time stay OK (the reference prints "Matrix is Singular!" at maxiter and returns
    its iterate, dbslmmfit.cpp:664-666)."""
    from dbslmm_amd import BLOCK_NOT_CONVERGED
    prob = _problem(seed=9, n_ref=256, miss_rate=0.0)
    prob.sigma_s = 0.5 / 1e6
    prob.opts.update(solver=2, pcg_maxit=3, pcg_tol=1e-14)
    (res,), wl = _run(prob)
    st = res[2]
    assert np.all(st == BLOCK_NOT_CONVERGED), st
    assert wl["pcg_iters"] == 3
    got = _cat(res)
    assert np.all(np.isfinite(got))
    prob.opts.update(pcg_maxit=0, pcg_tol=0.0)
    ref, _ = _oracle(prob)
    assert 1e-12 < normwise(got, ref) < 1e-2
    (res2,), _ = _run(prob)
    assert np.all(res2[2] == 0)


def test_large_panel_fp64_sigma_path():
    """n_ref > 16383: the integer Gram no longer fits uint16, every block's product reads the fp64
    Sigma; still within 1e-10 of the direct solve."""
    prob = _problem(seed=5, n_ref=16500, sizes=[130, 300, 700], miss_rate=0.0)
    prob.sigma_s = 0.5 / 1e6
    (res,), wl = _run(prob)
    assert wl["pcg_route"] == 1
    ref, _ = _oracle(prob)
    assert normwise(_cat(res), ref) < 1e-10
    assert np.all(res[2] == 0)


@pytest.mark.parametrize("factors", [(1.0,), (0.8, 1.0, 1.2)])
def test_whole_block_kernel_matches_chip_path(factors):
    """dbslmm_pcg_block (blocks of one product column and <= 8 tile rows solved whole by one
    workgroup) against the chip-wide kernels on the same plan inputs (pcg_whole = -1): every
    copy within the stopping bound of each other and 1e-10 of the oracle; statuses and the
    monomorphic block as there; repeated runs bit-identical."""
    prob = _problem(seed=11, n_ref=512, sizes=[60, 200, 700, 1100, 130], mono_block=4, miss_rate=0.0)
    prob.sigma_s = 0.5 / 1e6
    sig = [prob.sigma_s * f for f in factors]
    fz, wl = _run(prob, sig)
    fz2, _ = _run(prob, sig)
    for x, y in zip(fz, fz2):
        assert all(np.array_equal(u, v, equal_nan=True) for u, v in zip(x, y))
    prob.opts["pcg_whole"] = -1
    ch, wlc = _run(prob, sig)
    prob.opts.pop("pcg_whole")
    assert wl["pcg_route"] == 1 and wlc["pcg_route"] == 1
    for c in range(len(sig)):
        np.testing.assert_array_equal(fz[c][2], ch[c][2])
        a, b = _cat(fz[c]), _cat(ch[c])
        ok = np.isfinite(b)
        assert np.array_equal(np.isfinite(a), ok)
        assert normwise(a[ok], b[ok]) < 1e-11, (c, normwise(a[ok], b[ok]))
    prob.sigma_s = sig[-1]
    ref, _ = _oracle(prob)
    a = _cat(fz[-1])
    ok = np.isfinite(ref) & np.isfinite(a)
    assert normwise(a[ok], ref[ok]) < 1e-10


def test_block_sizes_at_the_quadrant_and_whole_block_edges():
    """Block sizes at the edges the product loads mask (range-checked buffer loads: rows and columns
    past m, the quadrant after a wave's last) and at the whole-block limit (1024 SNPs = 8 tile rows
    solved whole; 1025 on the chip-wide path): 1, 63 / 64 / 65 and 1023 / 1024 / 1025 SNPs, large
    SNPs in every other block, n_ref % 4 = 1, three h2f copies -- every copy within 1e-10 of the
    oracle's direct solve, and the whole-block kernel within 1e-11 of the chip-wide path."""
    prob = _problem(seed=23, n_ref=509, sizes=[1, 63, 64, 65, 1023, 1024, 1025, 130], miss_rate=0.0)
    prob.sigma_s = 0.5 / 1e6
    factors = (0.8, 1.0, 1.2)
    sig = [prob.sigma_s * f for f in factors]
    fz, wl = _run(prob, sig)
    assert wl["pcg_route"] == 1
    prob.opts["pcg_whole"] = -1
    ch, _ = _run(prob, sig)
    prob.opts.pop("pcg_whole")
    base = prob.sigma_s
    for c, s in enumerate(sig):
        assert np.all(fz[c][2] == 0) and np.all(ch[c][2] == 0)
        assert normwise(_cat(fz[c]), _cat(ch[c])) < 1e-11, c
        prob.sigma_s = s
        ref, _ = _oracle(prob)
        assert normwise(_cat(fz[c]), ref) < 1e-10, (c, normwise(_cat(fz[c]), ref))
    prob.sigma_s = base
