"""The drop-in `dbslmm` CLI: argument handling and host parsing (CPU), end-to-end (GPU)."""
import json
import os
import subprocess

import numpy as np
import pytest

import ref_numpy as R
from _common import BLOCKS_EUR1, GOLD, ROOT, TD, l_snps, rows_close

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
    1e-10 of the largest |beta| (the base factor's file stays identical)."""
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
            assert np.max(np.abs(vt - vr)) <= 1e-10 * np.max(np.abs(vr))


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
