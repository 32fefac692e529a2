"""Shared fixtures / problem builders for the tests (test infrastructure: may use oracle/)."""
from __future__ import annotations

import json
import math
import os

import numpy as np

import ref_numpy as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
TD = os.path.join(GOLD, "test_dat")
BLOCKS_EUR1 = os.path.join(ROOT, "dbslmm_amd", "data", "block_data", "EUR", "chr1.bed")


def load_bed(path) -> np.ndarray:
    return np.fromfile(path, dtype=np.uint8)


# dbslmm_options.cheb_tol default: the normwise bound of the h2f copies the Chebyshev iteration
# solves on the base copy's factor (include/dbslmm_hip.h); direct solves are held to 1e-10
CHEB_TOL = 1e-9


def normwise(a, ref) -> float:
    a = np.asarray(a, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if ref.size == 0:
        return 0.0
    return float(np.max(np.abs(a - ref)) / np.max(np.abs(ref)))


def csr_from_infos(infos, num_block):
    ptr = np.zeros(num_block + 1, dtype=np.int64)
    for e in infos:
        ptr[e["block"] + 1] += 1
    ptr = np.cumsum(ptr)
    pos = np.array([e["pos"] for e in infos], dtype=np.int32)
    z = np.array([e["z"] for e in infos], dtype=np.float64)
    return ptr, pos, z


def l_snps():
    return [l.strip() for l in open(os.path.join(GOLD, "l_snps.txt")) if l.strip()]


def td_problem(lmm_only=False, nsnp=996, tau=0.8, maf_max=0.2):
    """test_dat run through the reference host pipeline (BatchRun) -> CSR arrays."""
    n_ref = R.get_row(os.path.join(TD, "ref_chr1.fam"))
    bim = R.read_bim(os.path.join(TD, "ref_chr1"), n_ref, abs(maf_max - 1.0) >= 1e-10)
    blocks = R.read_block(BLOCKS_EUR1)
    summ = R.read_summ(os.path.join(TD, "summary_gemma_chr1.assoc.txt"))
    L = l_snps()
    ss = summ if lmm_only else [s for s in summ if s.snp not in L]
    sl = [] if lmm_only else [s for s in summ if s.snp in L]
    info_s = R.add_block(R.match_ref(ss, bim, maf_max)[0], blocks)
    info_l = R.add_block(R.match_ref(sl, bim, maf_max)[0], blocks)
    nb = len(blocks)
    s_ptr, s_pos, z_s = csr_from_infos(info_s, nb)
    d = dict(bed=load_bed(os.path.join(TD, "ref_chr1.bed")), n_ref=n_ref, n_obs=2400,
             sigma_s=0.5 / nsnp, tau=tau, s_ptr=s_ptr, s_pos=s_pos, z_s=z_s,
             info_s=info_s, info_l=info_l, num_block=nb)
    if not lmm_only:
        d["l_ptr"], d["l_pos"], d["z_l"] = csr_from_infos(info_l, nb)
    return d


def synth_small_problem(lmm_only=False):
    d = os.path.join(GOLD, "synth_small")
    meta = json.load(open(os.path.join(d, "meta.json")))
    gold = json.load(open(os.path.join(d, "golden.json")))
    key = "lmm" if lmm_only else "dbslmm"
    g = gold[f"{key}_pcg"]
    blk = np.array(meta["block"])
    z = np.array(meta["z"])
    nb = meta["num_block"]

    def csr(pos):
        pos = np.array(pos, dtype=np.int32)
        ptr = np.zeros(nb + 1, dtype=np.int64)
        np.add.at(ptr, blk[pos] + 1, 1)
        return np.cumsum(ptr), pos, z[pos]

    s_ptr, s_pos, z_s = csr(g["pos_s"])
    out = dict(bed=load_bed(os.path.join(d, "ref.bed")), n_ref=meta["n_ref"], n_obs=meta["n_obs"],
               sigma_s=meta["h2"] / meta["nsnp"], tau=0.8, s_ptr=s_ptr, s_pos=s_pos, z_s=z_s,
               num_block=nb, gold_pcg=gold[f"{key}_pcg"], gold_direct=gold[f"{key}_direct"])
    if not lmm_only:
        out["l_ptr"], out["l_pos"], out["z_l"] = csr(g["pos_l"])
    return out


def eff_lines(info_s, info_l, beta_s, beta_l):
    res = R.EstResult(np.asarray(beta_s), np.asarray(beta_l), info_s, info_l)
    return R.format_eff(res)


def rows_close(a: str, b: str, ulps: int = 1) -> bool:
    """Output rows equal, allowing +-ulps in the 6th significant digit of numeric fields."""
    ta, tb = a.split(), b.split()
    if len(ta) != len(tb) or ta[0] != tb[0] or ta[1] != tb[1] or ta[-1] != tb[-1]:
        return False
    for x, y in zip(ta[2:4], tb[2:4]):
        fx, fy = float(x), float(y)
        if fx == fy:
            continue
        scale = 10 ** (math.floor(math.log10(max(abs(fx), abs(fy)))) - 5)
        if abs(fx - fy) > ulps * scale * 1.0000001:
            return False
    return True
