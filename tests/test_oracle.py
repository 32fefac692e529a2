"""CPU tests: the oracle (NumPy restatement + C restatement) against the reference's own
known-answer test and the committed golden vectors.  No GPU needed."""
import json
import os

import numpy as np
import pytest

import oracle as O
import ref_numpy as R
from _common import (GOLD, TD, eff_lines, load_bed, normwise, rows_close, synth_small_problem,
                     td_problem)

GOLDEN = json.load(open(os.path.join(GOLD, "testdat_golden.json")))
KAT = [l.rstrip("\n") for l in open(os.path.join(GOLD, "kat_manual.txt")) if l.strip()]


def test_numpy_restatement_reproduces_manual_kat():
    """Rmd/Manual.Rmd:126-145, reproduced exactly at 6 digits (tau=1, nsnp=998, PCG)."""
    p = td_problem(nsnp=998, tau=1.0)
    res = R.est(p["bed"].tobytes(), p["n_ref"], p["n_obs"], p["sigma_s"], p["num_block"],
                p["info_s"], p["info_l"], tau=1.0, method="pcg")
    assert R.format_eff(res)[:20] == KAT


def test_golden_eff_txt_kat_prefix():
    assert GOLDEN["dbslmm_tau1.0_nsnp998_pcg"]["eff_txt"][:20] == KAT


@pytest.mark.parametrize("lmm", [False, True])
@pytest.mark.parametrize("tau,nsnp", [(0.8, 996), (1.0, 998)])
@pytest.mark.parametrize("method", ["pcg", "direct"])
def test_c_oracle_matches_golden(lmm, tau, nsnp, method):
    p = td_problem(lmm_only=lmm, nsnp=nsnp, tau=tau)
    g = GOLDEN[f"{'lmm' if lmm else 'dbslmm'}_tau{tau}_nsnp{nsnp}_{method}"]
    bs, bl, st, rc = O.est(p["bed"], p["n_ref"], p["n_obs"], p["sigma_s"], p["s_ptr"], p["s_pos"],
                           p["z_s"], p.get("l_ptr"), p.get("l_pos"), p.get("z_l"), tau=tau,
                           method=method)
    assert rc == 0
    ref = np.concatenate([g["beta_s"], g["beta_l"]])
    got = np.concatenate([bs, bl])
    tol = 1e-7 if method == "pcg" else 1e-12
    assert normwise(got, ref) < tol


def test_c_oracle_kat_rows():
    p = td_problem(nsnp=998, tau=1.0)
    bs, bl, _, rc = O.est(p["bed"], p["n_ref"], p["n_obs"], p["sigma_s"], p["s_ptr"], p["s_pos"],
                          p["z_s"], p["l_ptr"], p["l_pos"], p["z_l"], tau=1.0, method="pcg")
    lines = eff_lines(p["info_s"], p["info_l"], bs, bl)[:20]
    assert all(rows_close(a, b) for a, b in zip(lines, KAT))


def test_read_snp_im_c_vs_numpy_testdat():
    bed = load_bed(os.path.join(TD, "ref_chr1.bed"))
    idv = np.ones(400, dtype=np.int32)
    for pos in (0, 1, 100, 722):
        g1, m1 = O.read_snp_im(bed, pos, idv)
        g2, m2 = R.read_snp_im(bed, pos, idv)
        np.testing.assert_array_equal(g1, g2)
        assert m1 == m2
        np.testing.assert_allclose(O.normalize(g1), R.normalize(g2), rtol=0, atol=1e-15)


def test_read_snp_im_indicator_and_missing():
    """Test-panel style read: 0/1 indicator over the .fam rows, n % 4 != 0, missing calls."""
    d = os.path.join(GOLD, "synth_small")
    bed = load_bed(os.path.join(d, "ref.bed"))
    rng = np.random.default_rng(3)
    ind = (rng.random(203) < 0.7).astype(np.int32)
    n_miss_rows = 0
    for pos in range(0, 600, 7):
        g1, m1 = O.read_snp_im(bed, pos, ind)
        g2, m2 = R.read_snp_im(bed, pos, ind)
        np.testing.assert_array_equal(g1, g2)
        assert abs(m1 - m2) < 1e-15
        codes = R.decode_codes(bed[3 + pos * 51: 3 + pos * 51 + 51], 203)
        n_miss_rows += int((codes == 1).any())
    assert n_miss_rows > 0          # the fixture really exercises imputation


@pytest.mark.parametrize("lmm", [False, True])
def test_c_oracle_synth_small_golden(lmm):
    p = synth_small_problem(lmm)
    for method, g in (("pcg", p["gold_pcg"]), ("direct", p["gold_direct"])):
        bs, bl, _, rc = O.est(p["bed"], p["n_ref"], p["n_obs"], p["sigma_s"], p["s_ptr"],
                              p["s_pos"], p["z_s"], p.get("l_ptr"), p.get("l_pos"), p.get("z_l"),
                              method=method)
        assert rc == 0
        # two PCG implementations stopping at the reference's ABSOLUTE residual 1e-7
        # (dbslmmfit.cpp:648) agree only to ~1e-6 normwise here (A is ill-conditioned at
        # n_obs = 1e5, sigma_s = h2/600); the direct solves agree to rounding.
        tol = 1e-5 if method == "pcg" else 1e-12
        assert normwise(np.concatenate([bs, bl]), np.concatenate([g["beta_s"], g["beta_l"]])) < tol


def test_bed_maf_matches_read_snp_im():
    """Both restatements compute readSNPIm's af = 0.5 * sum(geno) / n with sum() in Armadillo's
    accumulate order (dtpr.cpp:361; the order decides the last bits once mean-imputed calls are
    added, and matchRef's strict |maf_ref - maf| < mafMax can flip on them): bit for bit, on
    test_dat and on the synthetic panel with missing calls."""
    for path, n_ref, n_snp in ((os.path.join(TD, "ref_chr1.bed"), 400, 723),
                               (os.path.join(GOLD, "synth_small", "ref.bed"), 203, 600)):
        bed = load_bed(path)
        maf = O.bed_maf(bed, n_ref, n_snp, threads=2)
        idv = np.ones(n_ref, dtype=np.int32)
        ref = np.array([R.read_snp_im(bed, pos, idv)[1] for pos in range(n_snp)])
        np.testing.assert_array_equal(maf, ref)


def test_joint_solve_identity():
    """beta = M^-1 [z_s; z_l] / sqrt(n) with M = [[S_ss + dI, S_sl], [S_ls, S_ll]] equals the
    reference's estBlock formulas (dbslmmfit.cpp:711-729) -- the identity the GPU path uses."""
    rng = np.random.default_rng(0)
    n_ref, ms, ml = 300, 60, 4
    G = rng.integers(0, 3, size=(n_ref, ms + ml)).astype(float)
    X = np.column_stack([R.normalize(G[:, j]) for j in range(ms + ml)])
    zs, zl = rng.standard_normal(ms), 6 * rng.standard_normal(ml)
    n, sig, tau = 5000, 1e-4, 0.8
    bs, bl, *_ = R.est_block_ls(n_ref, n, sig, X[:, :ms], X[:, ms:], zs, zl, tau, "direct")
    M = tau / n_ref * X.T @ X + (1 - tau) * np.eye(ms + ml)
    M[np.arange(ms), np.arange(ms)] += 1 / (sig * n)
    beta = np.linalg.solve(M, np.concatenate([zs, zl])) / np.sqrt(n)
    assert normwise(beta, np.concatenate([bs, bl])) < 1e-13
