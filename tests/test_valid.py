"""The `valid` tool (scr/validate.cpp): external-validation R^2 terms per block.

Parity is against the NumPy restatement (oracle/ref_numpy.py: read_dbslmm, read_ext, match_summ,
match_all, valid_blocks); no reference artefact pins `valid`'s output (parity unpinned beyond the
restatement, as DESIGN.md records).  Inputs: the reference's test_dat chr1 panel, its DBSLMM
result from the committed golden vectors (-d) and an external summary derived from its GEMMA
file (-s: snp a1 maf z)."""
import json
import os
import subprocess

import numpy as np
import pytest

import ref_numpy as R
from _common import BLOCKS_EUR1, GOLD, ROOT, TD, load_bed, normwise

VALID = os.path.join(ROOT, "dbslmm_amd", "bin", "valid")
REF = os.path.join(TD, "ref_chr1")


def make_inputs(tmp, flip_every=7):
    """-d: the golden DBSLMM output of test_dat; -s: external summary from its GEMMA file, with
    every `flip_every`-th A1 swapped (exercises matchSumm's sign flip) and every 11th SNP dropped."""
    g = json.load(open(os.path.join(GOLD, "testdat_golden.json")))
    d_path = os.path.join(tmp, "d.txt")
    with open(d_path, "w") as f:
        f.write("\n".join(g["dbslmm_tau0.8_nsnp996_pcg"]["eff_txt"]) + "\n")
    s_path = os.path.join(tmp, "ext.txt")
    with open(os.path.join(TD, "summary_gemma_chr1.assoc.txt")) as f, open(s_path, "w") as o:
        for i, line in enumerate(f):
            t = line.rstrip("\n").split("\t")
            if i % 11 == 5:
                continue
            z = float(t[8]) / float(t[9]) * 0.9
            a1, a2 = t[5], t[6]
            if i % flip_every == 3:
                a1 = a2
            o.write(f"{t[1]} {a1} {t[7]} {z:.6g}\n")
    return d_path, s_path


def oracle_csr(d_path, s_path, maf_max=0.2):
    n_ref = R.get_row(REF + ".fam")
    summc = R.match_summ(R.read_dbslmm(d_path), R.read_ext(s_path))
    bim = R.read_bim_b(REF, n_ref, abs(maf_max - 1.0) >= 1e-10)
    summp = R.match_all(summc, bim, maf_max)
    blocks = R.read_block(BLOCKS_EUR1)
    bed = load_bed(REF + ".bed")
    nume, deno, rows = R.valid_blocks(bed, n_ref, summp, blocks)
    ptr = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    flat = [j for r in rows for j in r]
    pos = np.array([summp[j][3] for j in flat], dtype=np.int32)
    z1 = np.array([summp[j][1] for j in flat])
    z2 = np.array([summp[j][2] for j in flat])
    return n_ref, bed, ptr, pos, z1, z2, nume, deno


def test_oracle_deno_is_quadratic_form(tmp_path):
    """deno = z1^T (X^T X / n) z1 equals |X z1|^2 / n (the form the GPU evaluates)."""
    n_ref, bed, ptr, pos, z1, z2, nume, deno = oracle_csr(*make_inputs(str(tmp_path)))
    assert ptr[-1] > 100
    for b in range(len(ptr) - 1):
        if ptr[b + 1] == ptr[b]:
            continue
        X = R.read_block_matrix(bed, pos[ptr[b]:ptr[b + 1]], n_ref)
        y = X @ z1[ptr[b]:ptr[b + 1]]
        assert abs(y @ y / n_ref - deno[b]) <= 1e-12 * abs(deno[b])
        assert abs(z1[ptr[b]:ptr[b + 1]] @ z2[ptr[b]:ptr[b + 1]] - nume[b]) <= 1e-12 * abs(nume[b])


@pytest.mark.parametrize("args,msg", [
    (["-s", "x", "-r", REF, "-b", BLOCKS_EUR1, "-r2", "o"], "-d is no parameter"),
    (["-d", "/nonexistent", "-s", "/nonexistent", "-r", REF, "-b", BLOCKS_EUR1, "-r2", "o"], "dose not exist"),
])
def test_valid_argument_errors(args, msg):
    r = subprocess.run([VALID] + args, capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and msg in r.stderr


@pytest.mark.gpu
def test_valid_blocks_gpu_vs_oracle_testdat(tmp_path):
    from dbslmm_amd import Context, valid_blocks
    n_ref, bed, ptr, pos, z1, z2, nume, deno = oracle_csr(*make_inputs(str(tmp_path)))
    gn, gd = valid_blocks(Context(0), bed, n_ref, ptr, pos, z1, z2)
    assert normwise(gn, nume) < 1e-13
    assert normwise(gd, deno) < 1e-12


@pytest.mark.gpu
def test_valid_blocks_gpu_missing_calls_and_monomorphic():
    from dbslmm_amd import Context, synth, valid_blocks
    p = synth.simulate(3000, 301, pop="EUR", chroms=[21, 22], seed=13, miss_rate=0.02, large_every=0)
    nb = (p.n_ref + 3) // 4
    mono = int(np.flatnonzero(p.block == p.block[100])[0])
    p.bed[3 + mono * nb: 3 + (mono + 1) * nb] = 0x00          # all hom -> sd 0 -> NaN block
    rng = np.random.default_rng(3)
    order = np.argsort(p.block, kind="stable")
    ptr = np.concatenate([[0], np.cumsum(np.bincount(p.block, minlength=len(p.blocks)))]).astype(np.int64)
    pos = order.astype(np.int32)
    z1, z2 = rng.standard_normal(p.m), rng.standard_normal(p.m)
    gn, gd = valid_blocks(Context(0), p.bed, p.n_ref, ptr, pos, z1, z2)
    for b in range(len(ptr) - 1):
        sl = slice(ptr[b], ptr[b + 1])
        if ptr[b + 1] == ptr[b]:
            assert gd[b] == 0.0 and gn[b] == 0.0
            continue
        X = R.read_block_matrix(p.bed, pos[sl], p.n_ref)
        ref = z1[sl] @ (X.T @ X / p.n_ref) @ z1[sl]
        if b == p.block[mono]:
            assert np.isnan(gd[b]) and np.isnan(ref)
        else:
            assert abs(gd[b] - ref) <= 1e-11 * abs(ref)
            assert abs(gn[b] - z1[sl] @ z2[sl]) <= 1e-12 * (abs(gn[b]) + 1e-300)


@pytest.mark.gpu
@pytest.mark.parametrize("maf_max", [0.2, 1.0])
def test_valid_cli_end_to_end(tmp_path, maf_max):
    d_path, s_path = make_inputs(str(tmp_path))
    out = str(tmp_path / "r2")
    r = subprocess.run([VALID, "-d", d_path, "-s", s_path, "-r", REF, "-mafMax", str(maf_max),
                        "-b", BLOCKS_EUR1, "-r2", out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines, nume, deno = R.valid(d_path, s_path, REF, maf_max, BLOCKS_EUR1)
    got = open(out + ".txt").read().strip("\n").split("\n")
    assert len(got) == len(lines)
    for a, b in zip(got, lines):
        if a != b:   # 6 significant digits: allow one unit in the last place
            x, y = np.array(a.split(), float), np.array(b.split(), float)
            assert np.all(np.abs(x - y) <= 1e-5 * np.abs(y) + 1e-300), (a, b)
