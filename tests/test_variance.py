"""Test-set variance: the n_test x num_block `diags` matrix DBSLMMFIT::est saves
to variance.txt (scr/dbslmmfit.cpp:116,191-214,242; calcBlock :366-626; calc_nt_by_nt_matrix,
scr/calc_asymptotic_variance.cpp:22-137).

The oracle is the NumPy restatement of the literal formulas (oracle/ref_numpy.py nt_diag_ls /
nt_diag_s: explicit inverses, as the reference).  The GPU evaluates the same quantity from the
Cholesky factor of the joint matrix the solve already holds (identity checked on CPU below).  No
reference artefact pins variance.txt (the reference ships no test indicator file and no output),
so parity is against the restatement only ("parity unpinned" beyond it)."""
import os

import numpy as np
import pytest

import ref_numpy as R
from _common import BLOCKS_EUR1, TD, l_snps, load_bed

TOL = 1e-8   # relative, per block column (fp64 throughout; oracle uses explicit inverses)


def factor_form(Xs, Xl, n_ref, n_obs, sigma, Ts, Tl, tau=0.8):
    """What the GPU computes: y = L^-1 [x_s; 0], y' = L^-1 [0; x_l] with M = L L^T the joint
    matrix [[Sigma_ss + I/(n sigma), Sigma_sl], [Sigma_ls, Sigma_ll]]."""
    ss, sl, ll = R.block_sigmas(Xs, Xl, n_ref, tau)
    ms = ss.shape[0]
    d = 1.0 / (n_obs * sigma)
    M = ss + d * np.eye(ms)
    if sl is not None:
        M = np.block([[M, sl], [sl.T, ll]])
    L = np.linalg.cholesky(M)
    m = M.shape[0]
    U = np.zeros((m, Ts.shape[0]))
    U[:ms] = Ts.T
    Y = np.linalg.solve(L, U)
    q1 = (Y[:ms] ** 2).sum(0)
    w2 = (Y[ms:] ** 2).sum(0)
    q3 = 0.0
    if sl is not None:
        Yl = np.linalg.solve(L[ms:, ms:], Tl.T)
        q3 = (Yl ** 2).sum(0)
    xs2 = (Ts ** 2).sum(1)
    return q3 / n_obs + n_obs * sigma * sigma * (d * xs2 - d * d * (q1 - w2))


@pytest.mark.parametrize("ml", [0, 1, 4])
def test_factor_form_equals_literal_formulas(ml):
    rng = np.random.default_rng(ml)
    n_ref, n_obs, sigma, ms, nt = 300, 5000, 2e-4, 40, 17
    Xs = rng.standard_normal((n_ref, ms))
    Xl = rng.standard_normal((n_ref, ml)) if ml else None
    Ts = rng.standard_normal((nt, ms))
    Tl = rng.standard_normal((nt, ml)) if ml else None
    ss, sl, ll = R.block_sigmas(Xs, Xl, n_ref)
    lit = R.nt_diag_ls(ll, sl, ss, sigma, n_obs, Tl, Ts) if ml else R.nt_diag_s(ss, sigma, n_obs, Ts)
    got = factor_form(Xs, Xl, n_ref, n_obs, sigma, Ts, Tl)
    assert np.max(np.abs(got - lit)) / np.max(np.abs(lit)) < 1e-12


# ----------------------------------------------------------------------------- test_dat
def td_indicator(n_total):
    """No indicator file ships with the reference: every 5th test individual (from the 3rd) is
    held out (0), the rest are test individuals (1)."""
    return np.array([0 if i % 5 == 2 else 1 for i in range(n_total)], dtype=np.int32)


def td_variance_problem(lmm_only, drop_test_mono=False, nsnp=996, maf_max=0.2):
    """The test_dat run of dbslmm.cpp:262-320 with -dat_str test_chr1: training problem, the test
    positions calcBlock pairs with it (makePosObjectForTestBim + addBlock, positional per block)
    and the indicator.  drop_test_mono removes the SNPs monomorphic among the test individuals
    from the summary (with them the reference's block column is NaN: nomalizeVec 0/0)."""
    from _common import csr_from_infos
    n_ref = R.get_row(os.path.join(TD, "ref_chr1.fam"))
    bim = R.read_bim(os.path.join(TD, "ref_chr1"), n_ref, abs(maf_max - 1.0) >= 1e-10)
    blocks = R.read_block(BLOCKS_EUR1)
    summ = R.read_summ(os.path.join(TD, "summary_gemma_chr1.assoc.txt"))
    base = R.read_test_bim(os.path.join(TD, "test_chr1.bim"))
    n_total = R.get_row(os.path.join(TD, "test_chr1.fam"))
    ind = td_indicator(n_total)
    tbed = load_bed(os.path.join(TD, "test_chr1.bed"))
    bad = set()
    if drop_test_mono:
        for e in R.make_pos_for_test_bim(base, R.match_ref(summ, bim, maf_max)[0]):
            g, _ = R.read_snp_im(tbed, e["pos"], ind)
            if np.all(g == g[0]):
                bad.add(e["snp"])
        summ = [x for x in summ if x.snp not in bad]
    L = l_snps()
    ss = summ if lmm_only else [x for x in summ if x.snp not in L]
    sl = [] if lmm_only else [x for x in summ if x.snp in L]
    inter_s = R.match_ref(ss, bim, maf_max)[0]
    inter_l = R.match_ref(sl, bim, maf_max)[0]
    info_s, info_l = R.add_block(inter_s, blocks), R.add_block(inter_l, blocks)
    t_info_s = R.add_block(R.make_pos_for_test_bim(base, inter_s), blocks)
    t_info_l = R.add_block(R.make_pos_for_test_bim(base, inter_l), blocks)
    nb = len(blocks)

    def aligned(info, t_info):
        out = []
        for b in range(nb):
            n = sum(1 for x in info if x["block"] == b)
            t = [x["pos"] for x in t_info if x["block"] == b]
            assert len(t) >= n
            out += t[:n]
        return np.array(out, dtype=np.int32)
    s_ptr, s_pos, z_s = csr_from_infos(info_s, nb)
    prob = dict(bed=load_bed(os.path.join(TD, "ref_chr1.bed")), n_ref=n_ref, n_obs=2400,
                sigma_s=0.5 / nsnp, s_ptr=s_ptr, s_pos=s_pos, z_s=z_s)
    if not lmm_only:
        prob["l_ptr"], prob["l_pos"], prob["z_l"] = csr_from_infos(info_l, nb)
    return dict(n_ref=n_ref, nb=nb, info_s=info_s, info_l=None if lmm_only else info_l,
                t_info_s=t_info_s, t_info_l=None if lmm_only else t_info_l, tbed=tbed,
                ts_pos=aligned(info_s, t_info_s), tl_pos=None if lmm_only else aligned(info_l, t_info_l),
                ind=ind, sigma=0.5 / nsnp, n_obs=2400, prob=prob, dropped=bad)


def td_oracle(v):
    with np.errstate(all="ignore"):
        return R.variance_diags(v["prob"]["bed"], v["n_ref"], v["n_obs"], v["sigma"], v["nb"], v["info_s"],
                                v["info_l"], v["tbed"], v["ind"], v["t_info_s"], v["t_info_l"])


@pytest.mark.parametrize("lmm_only", [False, True])
def test_oracle_variance_testdat(lmm_only):
    """As shipped, test_dat has SNPs monomorphic in the test panel: the reference's column is
    NaN.  Without them the column is finite and positive."""
    v = td_variance_problem(lmm_only)
    D = td_oracle(v)
    assert D.shape == (int(v["ind"].sum()), v["nb"])
    used = sorted({x["block"] for x in v["info_s"]})
    assert np.all(np.isnan(D[:, used]))
    unused = [b for b in range(v["nb"]) if b not in used]
    assert np.all(D[:, unused] == 0)
    v = td_variance_problem(lmm_only, drop_test_mono=True)
    D = td_oracle(v)
    assert np.all(np.isfinite(D[:, used])) and np.all(D[:, used] > 0)


def _colwise(got, ref):
    worst = 0.0
    for b in range(ref.shape[1]):
        s = np.max(np.abs(ref[:, b]))
        if s == 0:
            assert np.all(got[:, b] == 0)
            continue
        worst = max(worst, np.max(np.abs(got[:, b] - ref[:, b])) / s)
    return worst


@pytest.mark.gpu
@pytest.mark.parametrize("lmm_only", [False, True])
@pytest.mark.parametrize("drop", [False, True])
def test_gpu_variance_testdat(lmm_only, drop):
    from dbslmm_amd import BlockProblem, Context, Plan
    v = td_variance_problem(lmm_only, drop_test_mono=drop)
    D = td_oracle(v)
    plan = Plan(Context(0), BlockProblem(**v["prob"]))
    plan.run()
    plan.sync()
    got = plan.variance(v["tbed"], v["ind"], v["ts_pos"], v["tl_pos"])
    assert got.shape == D.shape
    assert np.array_equal(np.isnan(got), np.isnan(D))
    fin = np.isfinite(D)
    assert _colwise(np.where(fin, got, 0.0), np.where(fin, D, 0.0)) < TOL


# ----------------------------------------------------------------------------- synthetic
SIZES = [5, 63, 64, 130, 600, 0, 40]


def synth_variance_case(seed=3, n_ref=300, n_total=150, mono_block=None):
    from dbslmm_amd import BlockProblem, synth
    total = sum(SIZES)
    p = synth.simulate(total + 10, n_ref, pop="EUR", chroms=[1], seed=seed, miss_rate=0.003,
                       large_every=0)
    t = synth.simulate(total + 10, n_total, pop="EUR", chroms=[1], seed=seed + 100, miss_rate=0.003,
                       large_every=0)
    rng = np.random.default_rng(seed)
    bid = np.repeat(np.arange(len(SIZES)), SIZES)
    large = np.zeros(total, dtype=bool)
    for b in (2, 3, 4, 6):
        idx = np.flatnonzero(bid == b)
        large[rng.choice(idx, size=1 + b % 3, replace=False)] = True
    z = rng.standard_normal(total)
    z[large] = 6.0 * np.sign(z[large])
    bed = p.bed.copy()
    if mono_block is not None:
        j = int(np.flatnonzero(bid == mono_block)[1])
        nb = (n_ref + 3) // 4
        bed[3 + j * nb: 3 + (j + 1) * nb] = 0xFF
    perm = rng.permutation(total + 10).astype(np.int32)   # SNP r sits at test row perm[r]
    nbk = len(SIZES)

    def csr(mask):
        idx = np.flatnonzero(mask)
        ptr = np.zeros(nbk + 1, dtype=np.int64)
        np.add.at(ptr, bid[idx] + 1, 1)
        return np.cumsum(ptr), idx.astype(np.int32), z[idx]
    s_ptr, s_pos, z_s = csr(~large)
    l_ptr, l_pos, z_l = csr(large)
    tbed = np.zeros(3 + (total + 10) * ((n_total + 3) // 4), dtype=np.uint8)
    tb = (n_total + 3) // 4
    tbed[:3] = t.bed[:3]
    for r in range(total + 10):
        tbed[3 + perm[r] * tb: 3 + (perm[r] + 1) * tb] = t.bed[3 + r * tb: 3 + (r + 1) * tb]
    ind = (rng.random(n_total) < 0.75).astype(np.int32)
    prob = BlockProblem(bed=bed, n_ref=n_ref, n_obs=50000, sigma_s=0.3 / total, s_ptr=s_ptr,
                        s_pos=s_pos, z_s=z_s, l_ptr=l_ptr, l_pos=l_pos, z_l=z_l)
    return prob, tbed, ind, perm[s_pos], perm[l_pos]


def synth_oracle(prob, tbed, ind, ts_pos, tl_pos, sigma=None):
    sigma = prob.sigma_s if sigma is None else sigma
    D = np.zeros((int(ind.sum()), prob.num_block))
    for b in range(prob.num_block):
        rs = prob.s_pos[prob.s_ptr[b]:prob.s_ptr[b + 1]]
        rl = prob.l_pos[prob.l_ptr[b]:prob.l_ptr[b + 1]]
        if rs.size == 0:
            continue
        Xs = R.read_block_matrix(prob.bed, rs, prob.n_ref)
        Ts = R.read_test_block_matrix(tbed, ts_pos[prob.s_ptr[b]:prob.s_ptr[b + 1]], ind)
        with np.errstate(all="ignore"):
            if rl.size:
                Xl = R.read_block_matrix(prob.bed, rl, prob.n_ref)
                Tl = R.read_test_block_matrix(tbed, tl_pos[prob.l_ptr[b]:prob.l_ptr[b + 1]], ind)
                ss, sl, ll = R.block_sigmas(Xs, Xl, prob.n_ref)
                try:
                    D[:, b] = R.nt_diag_ls(ll, sl, ss, sigma, prob.n_obs, Tl, Ts)
                except np.linalg.LinAlgError:
                    D[:, b] = np.nan
            else:
                ss, _, _ = R.block_sigmas(Xs, None, prob.n_ref)
                try:
                    D[:, b] = R.nt_diag_s(ss, sigma, prob.n_obs, Ts)
                except np.linalg.LinAlgError:
                    D[:, b] = np.nan
    return D


@pytest.mark.gpu
@pytest.mark.parametrize("tiled_min", ["64", "100000"])
def test_gpu_variance_synthetic_all_paths(monkeypatch, tiled_min):
    """Blocks on the one-wave (m < 64), one-workgroup and tiled factor paths, an empty block,
    n_test > 64 (two workgroups of test individuals), permuted test rows, missing calls."""
    from dbslmm_amd import Context, Plan
    prob, tbed, ind, tsp, tlp = synth_variance_case()
    prob.opts["tiled_min"] = int(tiled_min)
    ref = synth_oracle(prob, tbed, ind, tsp, tlp)
    plan = Plan(Context(0), prob)
    plan.run()
    plan.sync()
    got = plan.variance(tbed, ind, tsp, tlp)
    assert np.all(got[:, SIZES.index(0)] == 0)
    assert np.all(np.isfinite(got))
    assert _colwise(got, ref) < TOL


@pytest.mark.gpu
def test_gpu_variance_monomorphic_block_is_nan():
    from dbslmm_amd import Context, Plan
    prob, tbed, ind, tsp, tlp = synth_variance_case(mono_block=3)
    plan = Plan(Context(0), prob)
    plan.run()
    plan.sync()
    got = plan.variance(tbed, ind, tsp, tlp)
    assert np.all(np.isnan(got[:, 3]))
    ref = synth_oracle(prob, tbed, ind, tsp, tlp)
    keep = [b for b in range(prob.num_block) if b != 3]
    assert _colwise(got[:, keep], ref[:, keep]) < TOL


@pytest.mark.gpu
def test_gpu_variance_after_run_multi_uses_last_sigma():
    from dbslmm_amd import Context, Plan
    prob, tbed, ind, tsp, tlp = synth_variance_case(seed=5)
    plan = Plan(Context(0), prob)
    sig = [prob.sigma_s * 0.8, prob.sigma_s * 1.2]
    plan.run_multi(sig)
    got = plan.variance(tbed, ind, tsp, tlp)
    ref = synth_oracle(prob, tbed, ind, tsp, tlp, sigma=sig[-1])
    assert _colwise(got, ref) < TOL


def test_variance_abi_rejects_misaligned_positions():
    """Host-side argument checks run before any GPU work (no GPU needed to reach them)."""
    from dbslmm_amd import Plan
    p = Plan.__new__(Plan)

    class _P:
        n_s, n_l, num_block = 3, 0, 1
    p.prob = _P()
    with pytest.raises(ValueError):
        p.variance(np.zeros(8, np.uint8), np.ones(4, np.int32), np.zeros(2, np.int32))


def read_arma_ascii(path):
    lines = open(path).read().split("\n")
    assert lines[0] == "ARMA_MAT_TXT_FN008"
    r, c = map(int, lines[1].split())
    vals = np.array([[float(x) for x in ln.split()] for ln in lines[2:2 + r]])
    assert vals.shape == (r, c)
    return vals


@pytest.mark.gpu
@pytest.mark.parametrize("drop", [False, True])
def test_cli_writes_variance_txt(tmp_path, drop):
    """dbslmm -dat_str test_chr1 -test_indicator_file ... writes ./variance.txt (arma_ascii,
    scr/dbslmmfit.cpp:242); values = the oracle's diags.  Formatting follows Armadillo's
    save_arma_ascii as restated (no reference output file to pin it)."""
    import subprocess
    from _common import ROOT
    from test_cli import REF, SUMM, split_summary
    v = td_variance_problem(False, drop_test_mono=drop)
    D = td_oracle(v)
    summ = str(tmp_path / "summ.txt")
    with open(SUMM) as f, open(summ, "w") as o:
        for line in f:
            if line.split("\t")[1] not in v["dropped"]:
                o.write(line)
    s, l = split_summary(tmp_path, summ)
    ind = str(tmp_path / "ind.txt")
    open(ind, "w").write("".join(f"{x}\n" for x in v["ind"]))
    cli = os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm")
    r = subprocess.run([cli, "-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996",
                        "-h", "0.5", "-mafMax", "0.2", "-eff", str(tmp_path / "o"),
                        "-dat_str", os.path.join(TD, "test_chr1"), "-test_indicator_file", ind],
                       capture_output=True, text=True, cwd=str(tmp_path), timeout=300)
    assert r.returncode == 0, r.stderr
    got = read_arma_ascii(str(tmp_path / "variance.txt"))
    assert got.shape == D.shape
    assert np.array_equal(np.isnan(got), np.isnan(D))
    fin = np.isfinite(D)
    assert _colwise(np.where(fin, got, 0.0), np.where(fin, D, 0.0)) < TOL


@pytest.mark.gpu
def test_cli_h2f_sharded_variance_matches_one_gpu(tmp_path):
    """-h2f 0.8,1,1.2 with -dat_str/-test_indicator_file: the variance of the last factor after a
    Chebyshev h2f run (the shards re-run that sigma before the variance).  --gpu-ids 0,0 (two
    shards on the test GPU, one of them idle: test_dat is one LD block) writes the same
    variance.txt and <eff> files byte for byte as one GPU."""
    import subprocess
    from _common import ROOT
    from test_cli import REF, SUMM, split_summary
    v = td_variance_problem(False, drop_test_mono=True)
    summ = str(tmp_path / "summ.txt")
    with open(SUMM) as f, open(summ, "w") as o:
        for line in f:
            if line.split("\t")[1] not in v["dropped"]:
                o.write(line)
    s, l = split_summary(tmp_path, summ)
    ind = str(tmp_path / "ind.txt")
    open(ind, "w").write("".join(f"{x}\n" for x in v["ind"]))
    cli = os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm")
    outs = []
    for name, extra in (("one", []), ("two", ["--gpu-ids", "0,0"])):
        d = tmp_path / name
        d.mkdir()
        r = subprocess.run([cli, "-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp",
                            "996", "-h", "0.5", "-h2f", "0.8,1,1.2", "-mafMax", "0.2", "-eff",
                            str(d / "o.dbslmm"), "-dat_str", os.path.join(TD, "test_chr1"),
                            "-test_indicator_file", ind] + extra,
                           capture_output=True, text=True, cwd=str(d), timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append([open(d / f).read() for f in ("variance.txt", "o_h2f0.8.dbslmm.txt",
                                                  "o_h2f1.dbslmm.txt", "o_h2f1.2.dbslmm.txt")])
    assert outs[0] == outs[1]
    assert read_arma_ascii(str(tmp_path / "one" / "variance.txt")).size > 0
