"""GPU parity tests: the HIP path (through the C-ABI) against the oracle and the golden vectors.

Parity bars (see DESIGN.md "Parity"):
  * vs the oracle's direct fp64 solve of the reference equations: normwise <= 1e-10
    (same mathematics, different but exact-integer Gram and Cholesky);
  * vs the reference-faithful PCG (absolute residual 1e-7, dbslmmfit.cpp:648): normwise <= 1e-5,
    the BASELINE criterion (the PCG itself is only that accurate);
  * 6-digit output rows of the Manual example: equal up to 1 unit in the last printed digit.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from _common import (GOLD, TD, eff_lines, load_bed, normwise, rows_close, synth_small_problem,
                     td_problem)

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(GOLD, "testdat_golden.json")))
KAT = [l.rstrip("\n") for l in open(os.path.join(GOLD, "kat_manual.txt")) if l.strip()]


@pytest.fixture(scope="module")
def fit():
    from dbslmm_amd import DBSLMMFIT
    return DBSLMMFIT(0)


def _prob(d):
    from dbslmm_amd import BlockProblem
    return BlockProblem(bed=d["bed"], n_ref=d["n_ref"], n_obs=d["n_obs"], sigma_s=d["sigma_s"],
                        s_ptr=d["s_ptr"], s_pos=d["s_pos"], z_s=d["z_s"], l_ptr=d.get("l_ptr"),
                        l_pos=d.get("l_pos"), z_l=d.get("z_l"), tau=d.get("tau", 0.8))


def _oracle(d, method="direct", threads=8):
    bs, bl, st, rc = O.est(d["bed"], d["n_ref"], d["n_obs"], d["sigma_s"], d["s_ptr"], d["s_pos"],
                           d["z_s"], d.get("l_ptr"), d.get("l_pos"), d.get("z_l"),
                           tau=d.get("tau", 0.8), method=method, threads=threads)
    return np.concatenate([bs, bl]), st


def test_bed_maf_matches_oracle(fit):
    from dbslmm_amd import bed_maf
    for path, n_ref, n_snp in ((os.path.join(TD, "ref_chr1.bed"), 400, 723),
                               (os.path.join(GOLD, "synth_small", "ref.bed"), 203, 600)):
        bed = load_bed(path)
        got = bed_maf(fit.ctx, bed, n_ref, n_snp)
        ref = O.bed_maf(bed, n_ref, n_snp, threads=4)
        np.testing.assert_array_equal(got, ref)     # Armadillo accumulate order, bit for bit
    # rows with and without missing calls side by side: the no-missing rows take the exact-sum
    # shortcut, the others the sequential Armadillo-order chain (n_ref odd: a ragged last word)
    from dbslmm_amd import synth
    p = synth.simulate(3000, 1003, chroms=[1], seed=4, miss_rate=0.0004, large_every=0)
    has_miss = np.zeros(p.m, dtype=bool)
    nb = (1003 + 3) // 4
    rows = p.bed[3:].reshape(p.m, nb)
    for j in range(4):
        has_miss |= np.any(((rows >> (2 * j)) & 3) == 1, axis=1) if j < 3 else \
            np.any((((rows[:, :-1] >> 6) & 3) == 1), axis=1)
    assert 0.1 < has_miss.mean() < 0.9, has_miss.mean()
    got = bed_maf(fit.ctx, p.bed, 1003, p.m)
    np.testing.assert_array_equal(got, O.bed_maf(p.bed, 1003, p.m, threads=4))


def test_read_snp_std_matches_oracle(fit):
    from dbslmm_amd import read_snp_std
    for path, n_ref, rows in ((os.path.join(TD, "ref_chr1.bed"), 400, [0, 3, 99, 722]),
                              (os.path.join(GOLD, "synth_small", "ref.bed"), 203, list(range(0, 600, 37)))):
        bed = load_bed(path)
        X, maf = read_snp_std(fit.ctx, bed, n_ref, rows)
        idv = np.ones(n_ref, dtype=np.int32)
        for j, r in enumerate(rows):
            g, m = O.read_snp_im(bed, r, idv)
            np.testing.assert_allclose(X[:, j], O.normalize(g), rtol=0, atol=1e-12)
            assert abs(maf[j] - m) < 1e-14


@pytest.mark.parametrize("lmm", [False, True])
@pytest.mark.parametrize("tau,nsnp", [(0.8, 996), (1.0, 998)])
def test_est_testdat_vs_golden(fit, lmm, tau, nsnp):
    d = td_problem(lmm_only=lmm, nsnp=nsnp, tau=tau)
    bs, bl, st = fit.est(_prob(d))
    got = np.concatenate([bs, bl])
    kind = "lmm" if lmm else "dbslmm"
    gd = GOLDEN[f"{kind}_tau{tau}_nsnp{nsnp}_direct"]
    gp = GOLDEN[f"{kind}_tau{tau}_nsnp{nsnp}_pcg"]
    assert normwise(got, np.concatenate([gd["beta_s"], gd["beta_l"]])) < 1e-10
    assert normwise(got, np.concatenate([gp["beta_s"], gp["beta_l"]])) < 1e-5
    assert st[0] == 0 and np.all(st[1:] == 1)        # one non-empty block, the rest empty


def test_est_reproduces_manual_kat(fit):
    d = td_problem(nsnp=998, tau=1.0)
    bs, bl, _ = fit.est(_prob(d))
    lines = eff_lines(d["info_s"], d["info_l"], bs, bl)[:20]
    bad = [(a, b) for a, b in zip(lines, KAT) if not rows_close(a, b)]
    assert not bad, bad


@pytest.mark.parametrize("lmm", [False, True])
def test_est_synth_small_missing_calls(fit, lmm):
    d = synth_small_problem(lmm)
    bs, bl, st = fit.est(_prob(d))
    got = np.concatenate([bs, bl])
    gd, gp = d["gold_direct"], d["gold_pcg"]
    assert normwise(got, np.concatenate([gd["beta_s"], gd["beta_l"]])) < 1e-10
    assert normwise(got, np.concatenate([gp["beta_s"], gp["beta_l"]])) < 1e-5
    assert np.all(st == 0)


@pytest.mark.parametrize("n_ref", [64, 65, 66, 67, 130, 301])
def test_ragged_individuals_and_missing(fit, n_ref):
    from dbslmm_amd import synth
    p = synth.simulate(400, n_ref, pop="EUR", chroms=[21], seed=n_ref, miss_rate=0.01,
                       large_every=2, block_limit=6)
    d = vars(synth.make_problem(p)).copy()
    ref, _ = _oracle(d)
    bs, bl, st = fit.est(_prob(d))
    assert normwise(np.concatenate([bs, bl]), ref) < 1e-10


def test_large_single_block_multi_tile(fit):
    """One block of 300+ SNPs: 10 Cholesky tiles, trailing updates, 3 large SNPs."""
    from dbslmm_amd import synth
    p = synth.simulate(330, 512, pop="EUR", chroms=[22], seed=5, large_every=0, block_limit=1)
    p.large[[10, 100, 250]] = True
    p.z[[10, 100, 250]] = [8.0, -8.0, 8.0]
    for lmm in (False, True):
        d = vars(synth.make_problem(p, lmm_only=lmm)).copy()
        ref, _ = _oracle(d)
        bs, bl, st = fit.est(_prob(d))
        assert normwise(np.concatenate([bs, bl]), ref) < 1e-10
        assert st[0] == 0


def test_blocks_with_only_large_snps_and_empty_blocks(fit):
    from dbslmm_amd import BlockProblem
    from dbslmm_amd import synth
    p = synth.simulate(120, 256, pop="EUR", chroms=[22], seed=9, large_every=0, block_limit=4)
    blk = p.block
    # block 0: only large SNPs; block 1: empty; others: small only
    large = blk == 0
    keep = blk != 1
    nb = len(p.blocks)
    si = np.flatnonzero(~large & keep)
    li = np.flatnonzero(large)
    def ptr(idx):
        q = np.zeros(nb + 1, dtype=np.int64)
        np.add.at(q, blk[idx] + 1, 1)
        return np.cumsum(q)
    d = dict(bed=p.bed, n_ref=p.n_ref, n_obs=p.n_obs, sigma_s=p.h2 / p.m, s_ptr=ptr(si),
             s_pos=si.astype(np.int32), z_s=p.z[si], l_ptr=ptr(li), l_pos=li.astype(np.int32),
             z_l=p.z[li] * 3)
    ref, _ = _oracle(d)
    bs, bl, st = fit.est(_prob(d))
    assert normwise(np.concatenate([bs, bl]), ref) < 1e-10
    assert st[1] == 1 and st[0] == 0


def test_monomorphic_snp_gives_nan_block(fit):
    """nomalizeVec divides by sd = 0 -> the reference's whole block becomes NaN."""
    from dbslmm_amd import synth
    p = synth.simulate(90, 128, pop="EUR", chroms=[22], seed=11, large_every=0, block_limit=3)
    j = int(np.flatnonzero(p.block == p.block[0])[2])
    nb = (p.n_ref + 3) // 4
    p.bed[3 + j * nb: 3 + (j + 1) * nb] = 0xFF        # all individuals hom (code 3 -> 0.0)
    d = vars(synth.make_problem(p, lmm_only=True)).copy()
    bs, bl, st = fit.est(_prob(d))
    in_b0 = p.block[d["s_pos"]] == p.block[0]
    assert np.all(np.isnan(bs[in_b0]))
    assert np.all(np.isfinite(bs[~in_b0]))
    assert st[p.block[0]] == 3
    ref, _ = _oracle(d, method="pcg")
    assert np.all(np.isnan(ref[in_b0]))


def test_plan_rerun_bit_identical_and_sigma_update(fit):
    from dbslmm_amd import Plan, synth
    p = synth.simulate(3000, 500, seed=2, chroms=[1, 2])
    prob = synth.make_problem(p)
    plan = Plan(fit.ctx, prob)
    plan.run()
    b1 = plan.download()
    plan.enable_timing(True)
    for _ in range(3):
        plan.run()
    plan.sync()
    b2 = plan.download()
    for x, y in zip(b1, b2):
        np.testing.assert_array_equal(x, y)
    ms, n = plan.kernel_ms()
    assert n == 3 and np.all(ms[:4] > 0) and ms[4] >= 0
    plan.set_sigma(prob.sigma_s * 1.2)
    plan.run()
    b3 = plan.download()
    prob2 = synth.make_problem(p)
    prob2.sigma_s = prob.sigma_s * 1.2
    b4 = fit.est(prob2)
    np.testing.assert_array_equal(b3[0], b4[0])
    np.testing.assert_array_equal(b3[1], b4[1])


def test_bench_config_vs_oracle(fit):
    """Config 2 (50k SNPs x 2k individuals, 22 chr EUR blocks): full problem vs the oracle."""
    from dbslmm_amd import synth
    p = synth.simulate(50000, 2000, seed=1)
    d = vars(synth.make_problem(p)).copy()
    O.use_blas(True)
    ref_d, _ = _oracle(d, method="direct", threads=16)
    bs, bl, st = fit.est(_prob(d))
    got = np.concatenate([bs, bl])
    assert np.all(st[st != 1] == 0)
    assert normwise(got, ref_d) < 1e-10


def test_run_multi_sigma_matches_separate_solves(fit, monkeypatch):
    """h2f tuning: one Gram, three solves == three fresh plans (bit-identical), any block path
    (the merged-factorisation path; tests/test_h2f_cheb.py covers the Chebyshev one)."""
    from dbslmm_amd import Plan, synth
    p = synth.simulate(20000, 600, seed=3, chroms=[1, 2, 3], miss_rate=0.001)
    prob = synth.make_problem(p)
    prob.opts["h2f_mode"] = 1
    sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
    plan = Plan(fit.ctx, prob)
    multi = plan.run_multi(sig)
    for f, (bs, bl, st) in zip(sig, multi):
        q = synth.make_problem(p)
        q.sigma_s = f
        rs, rl, rst = fit.est(q)
        np.testing.assert_array_equal(bs, rs)
        np.testing.assert_array_equal(bl, rl)
        np.testing.assert_array_equal(st, rst)
    assert not np.array_equal(multi[0][0], multi[2][0])


def test_cached_and_staged_bed_upload_identical(fit):
    """dbslmm_ctx_cache_bed: one staged (pinned, chunked) upload serves bed_maf and plan_create;
    results equal the uncached path bit for bit.  The 200 MB image takes the staged path (> 2
    chunks of 64 MB, ragged tail)."""
    from dbslmm_amd import Context, Plan, bed_maf
    rng = np.random.default_rng(3)
    n_ref, n_snp = 1001, 800_003
    bps = (n_ref + 3) // 4
    bed = rng.integers(0, 256, size=3 + n_snp * bps, dtype=np.uint8)
    bed[:3] = (0x6C, 0x1B, 0x01)
    plain = bed_maf(fit.ctx, bed, n_ref, n_snp)
    ctx = Context(0)
    ctx.cache_bed(bed)
    np.testing.assert_array_equal(bed_maf(ctx, bed, n_ref, n_snp), plain)
    ctx.cache_bed(None)
    d = td_problem(nsnp=996, tau=0.8)
    ctx.cache_bed(d["bed"])
    from dbslmm_amd import BlockProblem
    prob = BlockProblem(bed=d["bed"], n_ref=d["n_ref"], n_obs=d["n_obs"], sigma_s=d["sigma_s"],
                        s_ptr=d["s_ptr"], s_pos=d["s_pos"], z_s=d["z_s"], l_ptr=d["l_ptr"],
                        l_pos=d["l_pos"], z_l=d["z_l"], tau=0.8)
    plan = Plan(ctx, prob)
    plan.run()
    a = plan.download()
    b = fit.est(prob)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_cache_bed_from_file_descriptor(fit, tmp_path):
    """dbslmm_ctx_cache_bed_fd (ABI 8, the CLI's path): the image read with pread from the file
    into the staged upload, keyed by a pointer that is never dereferenced; bed_maf and a plan
    created with that key equal the uncached path bit for bit.  Also: a plan created from the
    cached image keeps it alive after the context releases it (read in place)."""
    import ctypes as C
    from dbslmm_amd import BlockProblem, Context, Plan, bed_maf
    rng = np.random.default_rng(5)
    n_ref, n_snp = 1001, 300_001
    bps = (n_ref + 3) // 4
    bed = rng.integers(0, 256, size=3 + n_snp * bps, dtype=np.uint8)
    bed[:3] = (0x6C, 0x1B, 0x01)
    path = str(tmp_path / "x.bed")
    bed.tofile(path)
    plain = bed_maf(fit.ctx, bed, n_ref, n_snp)
    ctx = Context(0)
    fd = os.open(path, os.O_RDONLY)
    try:
        ctx.check(ctx.lib.dbslmm_ctx_cache_bed_fd(ctx.h, fd, bed.size, bed.ctypes.data_as(C.c_void_p)),
                  "ctx_cache_bed_fd")
    finally:
        os.close(fd)
    np.testing.assert_array_equal(bed_maf(ctx, bed, n_ref, n_snp), plain)
    d = td_problem(nsnp=996, tau=0.8)
    path2 = str(tmp_path / "td.bed")
    d["bed"].tofile(path2)
    fd = os.open(path2, os.O_RDONLY)
    try:
        ctx.check(ctx.lib.dbslmm_ctx_cache_bed_fd(ctx.h, fd, d["bed"].size,
                                                  d["bed"].ctypes.data_as(C.c_void_p)), "ctx_cache_bed_fd")
    finally:
        os.close(fd)
    prob = BlockProblem(bed=d["bed"], n_ref=d["n_ref"], n_obs=d["n_obs"], sigma_s=d["sigma_s"],
                        s_ptr=d["s_ptr"], s_pos=d["s_pos"], z_s=d["z_s"], l_ptr=d["l_ptr"],
                        l_pos=d["l_pos"], z_l=d["z_l"], tau=0.8)
    plan = Plan(ctx, prob)
    ctx.cache_bed(None)                  # the plan holds its own reference to the cached image
    plan.run()
    a = plan.download()
    b = fit.est(prob)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
