"""The drop-in `dbslmm` CLI: argument handling and host parsing (CPU), end-to-end (GPU)."""
import json
import os
import subprocess

import numpy as np
import pytest

import ref_numpy as R
from _common import BLOCKS_EUR1, CHEB_TOL, GOLD, ROOT, TD, l_snps, rows_close

CLI = os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm")
SUMM = os.path.join(TD, "summary_gemma_chr1.assoc.txt")
REF = os.path.join(TD, "ref_chr1")
KAT = [l.rstrip("\n") for l in open(os.path.join(GOLD, "kat_manual.txt")) if l.strip()]


def run(args, cwd=None):
    return subprocess.run([CLI] + args, capture_output=True, text=True, cwd=cwd, timeout=300)


def split_summary(tmp, summ=SUMM):
    L = set(l_snps())
    s_path, l_path = os.path.join(tmp, "s.txt"), os.path.join(tmp, "l.txt")
    with open(summ) as f, open(s_path, "w") as fs, open(l_path, "w") as fl:
        for line in f:
            (fl if line.split("\t")[1] in L else fs).write(line)
    return s_path, l_path


def test_cli_built():
    assert os.access(CLI, os.X_OK), "build first: __graft_entry__.build()"


def test_help_and_header():
    r = run(["-h"])
    assert r.returncode == 0 and "-mafMax" in r.stdout
    r = run([])
    assert r.returncode == 0 and "DBSLMM" in r.stdout


@pytest.mark.parametrize("args,msg", [
    (["-r", REF, "-b", BLOCKS_EUR1, "-h", "0.5", "-eff", "x"], "-s is no parameter"),
    (["-s", SUMM, "-r", REF, "-b", "/nonexistent", "-h", "0.5", "-eff", "x"], "dose not exist"),
    (["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "1.5", "-n", "10", "-nsnp", "10", "-eff", "x"],
     "-h is not correct"),
    (["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "0.5", "-t", "0", "-n", "10", "-nsnp", "10",
      "-eff", "x"], "-t is not correct"),
])
def test_argument_errors_exit_1(args, msg):
    r = run(args)
    assert r.returncode == 1 and msg in r.stderr


def test_value_starting_with_dash_is_skipped(tmp_path):
    """Assign skips a value that starts with '-' (scr/dbslmm.cpp:74): -h -0.5 leaves h unset."""
    r = run(["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-h", "-0.5", "-n", "2400", "-nsnp", "996",
             "-mafMax", "1", "-eff", str(tmp_path / "o"), "--dry-run"])
    assert r.returncode == 1 and "-h is not correct" in r.stderr


def test_dry_run_matches_reference_host_pipeline(tmp_path):
    s, l = split_summary(tmp_path)
    r = run(["-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996", "-h",
             "0.5", "-mafMax", "1", "-eff", str(tmp_path / "o"), "--dry-run"])
    assert r.returncode == 0, r.stderr
    bim = R.read_bim(REF, 400, False)
    blocks = R.read_block(BLOCKS_EUR1)
    info_s = R.add_block(R.match_ref(R.read_summ(s), bim, 1.0)[0], blocks)
    info_l = R.add_block(R.match_ref(R.read_summ(l), bim, 1.0)[0], blocks)
    assert f"dry-run: blocks {len(blocks)} small {len(info_s)} large {len(info_l)}" in r.stdout
    # .badsnps: unmatched small SNPs flagged 0, then unmatched large flagged 1
    bad = open(str(tmp_path / "o") + ".badsnps").read().split("\n")
    _, good = R.match_ref(R.read_summ(s), bim, 1.0)
    exp = [f"{x.snp} 0" for x, g in zip(R.read_summ(s), good) if not g]
    assert bad[:len(exp)] == exp


@pytest.mark.gpu
def test_cli_end_to_end_manual_kat(tmp_path):
    """dbslmm on the reference example (tau=1 as in the Manual): <eff>.txt first 20 rows equal
    Rmd/Manual.Rmd:126-145 up to one unit in the 6th digit; every row vs the oracle."""
    s, l = split_summary(tmp_path)
    eff = str(tmp_path / "out")
    r = run(["-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "998", "-h",
             "0.5", "-mafMax", "0.2", "-t", "1", "-eff", eff, "--tau", "1.0"], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    lines = open(eff + ".txt").read().strip().split("\n")
    assert len(lines) == 716
    assert all(rows_close(a, b) for a, b in zip(lines[:20], KAT)), lines[:20]
    import json
    g = json.load(open(os.path.join(GOLD, "testdat_golden.json")))
    ref = g["dbslmm_tau1.0_nsnp998_pcg"]["eff_txt"]
    # identical SNP / allele / flag columns and order; beta normwise within the BASELINE 1e-5
    # (elementwise 6-digit equality is not attainable for near-zero betas)
    assert [x.split()[:2] + x.split()[4:] for x in lines] == [x.split()[:2] + x.split()[4:] for x in ref]
    got = np.array([float(x.split()[2]) for x in lines])
    exp = np.array([float(x.split()[2]) for x in ref])
    assert np.max(np.abs(got - exp)) / np.max(np.abs(exp)) < 2e-5


@pytest.mark.gpu
def test_cli_lmm_only_tau08(tmp_path):
    eff = str(tmp_path / "lmm")
    r = run(["-s", SUMM, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996", "-h", "0.5",
             "-mafMax", "0.2", "-eff", eff, "--precise-out"])
    assert r.returncode == 0, r.stderr
    import json
    g = json.load(open(os.path.join(GOLD, "testdat_golden.json")))
    got = np.array([float(x.split()[2]) for x in open(eff + ".txt").read().strip().split("\n")])
    ref = np.array(g["lmm_tau0.8_nsnp996_direct"]["beta_s"])
    assert got.size == ref.size
    assert np.max(np.abs(got - ref)) / np.max(np.abs(ref)) < 1e-10


def _eff_rows(text):
    rows = [l.split() for l in text.splitlines() if l.strip()]
    keys = [(r[0], r[1], r[4]) for r in rows]
    vals = np.array([[float(r[2]), float(r[3])] for r in rows])
    return keys, vals


@pytest.mark.gpu
@pytest.mark.parametrize("cheb", ["0", "1"])
def test_cli_h2f_tuning_matches_separate_runs(tmp_path, monkeypatch, cheb):
    """-h2f 0.8,1,1.2 (one Gram, three solves) writes the R driver's file names
    (<prefix>_h2f<hh>.dbslmm.txt, software/DBSLMM.R:204-219) with the same rows as three runs
    with -h 0.5*hh: identical with the merged factorisations (--h2f-merged); with the
    Chebyshev path (one factor, the other factors iterated) the same rows and values within
    cheb_tol (CHEB_TOL) of the largest |beta| (the base factor's file stays identical)."""
    s, l = split_summary(tmp_path)
    base = ["-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996",
            "-mafMax", "0.2", "--precise-out"]
    prefix = str(tmp_path / "chr1")
    merged = ["--h2f-merged"] if cheb == "0" else []
    r = run(base + merged + ["-h", "0.5", "-h2f", "0.8,1,1.2", "-eff", prefix + ".dbslmm"])
    assert r.returncode == 0, r.stderr
    for hh in ("0.8", "1", "1.2"):
        tuned = open(f"{prefix}_h2f{hh}.dbslmm.txt").read()
        single = str(tmp_path / f"single{hh}")
        r = run(base + ["-h", repr(0.5 * float(hh)), "-eff", single])
        assert r.returncode == 0, r.stderr
        ref = open(single + ".txt").read()
        if cheb == "0" or hh == "1":
            assert tuned == ref
        else:
            kt, vt = _eff_rows(tuned)
            kr, vr = _eff_rows(ref)
            assert kt == kr
            assert np.max(np.abs(vt - vr)) <= CHEB_TOL * np.max(np.abs(vr))


@pytest.mark.gpu
def test_cli_h2f_unwritable_output_named_and_cleaned(tmp_path):
    """when one of the -h2f outputs cannot be written (here a directory holds its
    name), the error names that file, not the first one, and no other output is left behind
    truncated or partly written."""
    s, l = split_summary(tmp_path)
    prefix = str(tmp_path / "chr1")
    blocked = f"{prefix}_h2f1.dbslmm.txt"
    os.mkdir(blocked)
    r = run(["-s", s, "-l", l, "-r", REF, "-b", BLOCKS_EUR1, "-n", "2400", "-nsnp", "996",
             "-mafMax", "0.2", "-h", "0.5", "-h2f", "0.8,1,1.2", "-eff", prefix + ".dbslmm"])
    assert r.returncode != 0
    assert "_h2f1.dbslmm.txt cannot be written" in r.stderr, r.stderr
    for hh in ("0.8", "1.2"):
        assert not os.path.exists(f"{prefix}_h2f{hh}.dbslmm.txt")


@pytest.mark.gpu
def test_cli_gpu_ids_shards_match_single_gpu(tmp_path):
    """--gpu-ids 0,0,0 (the LD blocks of chromosome 1 sharded over three contexts; on a node
    --gpus N uses devices 0..N-1) writes the same <eff>.txt byte for byte as one GPU."""
    from dbslmm_amd import synth
    panel = synth.simulate(6000, 300, pop="EUR", chroms=[1], seed=11, large_every=4)
    f = synth.write_plink(panel, str(tmp_path / "p"))
    base = ["-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]),
            "-nsnp", str(f["nsnp"]), "-h", "0.5", "--precise-out"]
    outs = []
    for extra, name in (([], "one"), (["--gpu-ids", "0,0,0"], "three")):
        eff = str(tmp_path / name)
        r = run(base + extra + ["-eff", eff], cwd=str(tmp_path))
        assert r.returncode == 0, r.stderr
        outs.append(open(eff + ".txt").read())
    assert "Sharding the LD blocks over 3 GPUs" in r.stdout
    assert len(outs[0].splitlines()) > 5000
    assert outs[0] == outs[1]


def _filtered_panel(tmp_path, layout, seed=5):
    """3-chromosome synthetic panel whose GEMMA summaries exercise every host filter of BatchRun:
    swapped alleles and a wrong a2 (matchRef compares a1/a2 strictly, no strand flips:
    scr/dtpr.cpp:387-392), SNPs absent from the .bim, summary MAFs that differ from the .bed MAF by
    more than -mafMax and by exactly -mafMax (strict `<`, :389), plus SNPs outside the LD blocks
    (addBlock's sequential [start, end) scan, :455-481): layout "tail" cuts the last block short
    (its last SNPs are never assigned), "gap" removes a block in the middle of chromosome 20 (the
    scan stalls there and nothing after it is assigned)."""
    from dbslmm_amd import synth
    panel = synth.simulate(7000, 250, pop="EUR", chroms=[19, 20, 21], seed=seed, large_every=3,
                           miss_rate=0.002)
    f = synth.write_plink(panel, str(tmp_path / "p"))
    rng = np.random.default_rng(seed)
    # duplicate SNP ids in the .bim: std::map::insert keeps the first line (dtpr.cpp:108-118)
    lines = open(f["ref"] + ".bim").read().splitlines()
    for k in rng.choice(np.arange(100, len(lines)), size=8, replace=False):
        t = lines[k].split("\t")
        t[1] = lines[k - 37].split("\t")[1]
        lines[k] = "\t".join(t)
    open(f["ref"] + ".bim", "w").write("\n".join(lines) + "\n")
    bim = R.read_bim(f["ref"], panel.n_ref, True)         # .bed MAF (IO::readBim, constr)
    for key in ("s", "l"):
        out = []
        for line in open(f[key]).read().splitlines():
            t = line.split("\t")
            u = rng.random()
            if u < 0.03:
                t[5], t[6] = t[6], t[5]                       # allele flip: rejected
            elif u < 0.04:
                t[6] = "T"                                    # a2 mismatch
            elif u < 0.07:
                maf = bim[t[1]][3]                            # |maf_bim - maf| = 0.25: rejected
                t[7] = "%.17g" % (maf + 0.25 if maf < 0.25 else maf - 0.25)
            elif u < 0.09:
                t[7] = "%.17g" % (bim[t[1]][3] + 0.2)         # boundary of the strict <
            elif u < 0.10:
                t[1] += "_absent"                             # not in the .bim
            out.append("\t".join(t))
        open(f[key], "w").write("\n".join(out) + "\n")
    blocks = [list(b) for b in panel.blocks]
    if layout == "tail":
        bmax = int(panel.block.max())
        last = np.flatnonzero(panel.block == bmax)
        blocks[bmax][2] = int(panel.ps[last[-min(12, last.size - 1)]])   # its last SNPs fall outside
    else:
        c20 = [i for i, b in enumerate(blocks) if b[0] == 20]
        del blocks[c20[len(c20) // 2]]
    with open(f["b"], "w") as fb:
        for c, s, e in blocks:
            fb.write(f"chr{c}\t{s}\t{e}\n")
    return panel, f, bim


def _oracle_host(f, bim, maf_max):
    """ref_numpy restatement of BatchRun's host steps (scr/dbslmm.cpp:252-317)."""
    blocks = R.read_block(f["b"])
    summ_s, summ_l = R.read_summ(f["s"]), R.read_summ(f["l"])
    inter_s, good_s = R.match_ref(summ_s, bim, maf_max)
    inter_l, good_l = R.match_ref(summ_l, bim, maf_max)
    info_s, info_l = R.add_block(inter_s, blocks), R.add_block(inter_l, blocks)
    bad = [f"{x.snp} 0" for x, g in zip(summ_s, good_s) if not g] + \
          [f"{x.snp} 1" for x, g in zip(summ_l, good_l) if not g]
    return blocks, inter_s, inter_l, info_s, info_l, bad


@pytest.mark.parametrize("layout", ["tail", "gap"])
def test_dry_run_filters_match_oracle_multichrom(tmp_path, layout):
    """CPU: the CLI's host pipeline (-mafMax 1: no MAF pass) on the 3-chromosome panel with
    allele mismatches, absent SNPs and out-of-block SNPs: block / SNP counts and .badsnps equal
    the restatement's."""
    panel, f, bim = _filtered_panel(tmp_path, layout)
    bim1 = {k: (v[0], v[1], v[2], 0.0) for k, v in bim.items()}      # constr = false: maf 0
    blocks, inter_s, inter_l, info_s, info_l, bad = _oracle_host(f, bim1, 1.0)
    eff = str(tmp_path / "o")
    r = run(["-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]), "-nsnp",
             str(f["nsnp"]), "-h", "0.5", "-mafMax", "1", "-eff", eff, "--dry-run"])
    assert r.returncode == 0, r.stderr
    assert f"dry-run: blocks {len(blocks)} small {len(info_s)} large {len(info_l)}" in r.stdout
    assert len(info_s) < len(inter_s)                     # out-of-block SNPs were dropped
    assert open(eff + ".badsnps").read().splitlines() == bad
    assert len(bad) > 100


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["tail", "gap"])
def test_cli_filters_multichrom_match_oracle(tmp_path, layout):
    """The drop-in CLI on the filtered 3-chromosome panel vs the oracle, row for row
    (VERDICT r02 item 1a): the GPU MAF pass + matchRef (-mafMax 0.2, strict <), addBlock,
    DBSLMMFIT::est and the writer (scr/dbslmm.cpp:252-364).  <eff>.txt: identical SNP / allele /
    flag columns in the reference's order (large rows, then small), betas within 1e-10 normwise of
    the oracle's direct fp64 solve; the default 6-digit file equals the precise file's values
    through C's %g; .badsnps identical."""
    panel, f, bim = _filtered_panel(tmp_path, layout)
    blocks, inter_s, inter_l, info_s, info_l, bad = _oracle_host(f, bim, 0.2)
    nb = len(blocks)
    res = R.est(panel.bed, panel.n_ref, f["n"], 0.5 / f["nsnp"], nb, info_s, info_l, tau=0.8,
                method="chol")
    exp = R.format_eff(res)
    base = ["-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]), "-nsnp",
            str(f["nsnp"]), "-h", "0.5", "-mafMax", "0.2"]
    precise, plain = str(tmp_path / "precise"), str(tmp_path / "plain")
    r = run(base + ["-eff", precise, "--precise-out"], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert f"After filtering, {len(inter_s)} small effect SNPs are selected." in r.stdout
    r = run(base + ["-eff", plain], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    assert open(plain + ".badsnps").read().splitlines() == bad
    rows_p = [x.split() for x in open(precise + ".txt").read().splitlines()]
    rows_g = [x.split() for x in open(plain + ".txt").read().splitlines()]
    rows_e = [x.split() for x in exp]
    assert len(rows_e) == len(info_s) + len(info_l) > 3000
    key = lambda rows: [(x[0], x[1], x[4]) for x in rows]
    assert key(rows_p) == key(rows_e) == key(rows_g)
    got = np.array([float(x[2]) for x in rows_p])
    ref = np.concatenate([res.beta_l, res.beta_s])
    assert np.max(np.abs(got - ref)) <= 1e-10 * np.max(np.abs(ref))
    noscl = np.array([float(x[3]) for x in rows_p])
    maf = np.array([e["maf"] for e in info_l + info_s])
    assert np.allclose(noscl, got / np.sqrt(2 * maf * (1 - maf)), rtol=1e-15, atol=0)
    # the default writer is C's %g at precision 6 of the same doubles
    assert [(x[2], x[3]) for x in rows_g] == [(R.format_g(float(x[2])), R.format_g(float(x[3])))
                                              for x in rows_p]
    # and the oracle's %g rows agree up to one unit in the 6th digit (beta differences ~1e-13)
    assert sum(not rows_close(" ".join(a), " ".join(b)) for a, b in zip(rows_g, rows_e)) == 0


@pytest.mark.gpu
def test_cli_timing_and_mafmax_multichrom(tmp_path):
    """--timing prints the phase wall times as one JSON line on stderr; the run goes through the
    cached .bed (one upload for the MAF pass and the plan) and writes the same rows as a run
    without it -- over three chromosomes in one call (blocks in chromosome order)."""
    from dbslmm_amd import synth
    panel = synth.simulate(9000, 256, pop="EUR", chroms=[20, 21, 22], seed=4, large_every=5)
    f = synth.write_plink(panel, str(tmp_path / "p"))
    base = ["-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]),
            "-nsnp", str(f["nsnp"]), "-h", "0.5", "-mafMax", "0.2", "--precise-out"]
    eff = str(tmp_path / "t")
    r = run(base + ["-eff", eff, "--timing"], cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr
    line = [x for x in r.stderr.splitlines() if x.startswith("TIMING ")]
    assert len(line) == 1, r.stderr
    ph = json.loads(line[0][7:])
    for k in ("ctx", "bed_upload", "maf", "parse", "plan", "solve", "write", "total"):
        assert ph[k] >= 0.0, k
    rows = open(eff + ".txt").read().splitlines()
    assert ph["snps"] == len(rows) > 8000
    # a second run writes the same rows (deterministic reductions)
    eff2 = str(tmp_path / "u")
    r = run(base + ["-eff", eff2], cwd=str(tmp_path))
    assert r.returncode == 0 and open(eff2 + ".txt").read().splitlines() == rows
