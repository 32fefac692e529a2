"""Generate the committed golden fixtures under tests/golden/ (run from the repo root).

Inputs are the reference's own example data (tests/golden/test_dat/ = fboehm/DBSLMM test_dat/,
copied verbatim) and the EUR chr1 LD blocks (dbslmm_amd/data/block_data/EUR/chr1.bed = the
reference's block_data/EUR/chr1.bed).  Expected outputs come from the NumPy restatement
oracle/ref_numpy.py, which is itself pinned by the Manual known-answer test (kat_manual.txt,
the 20 rows printed in the reference's Rmd/Manual.Rmd:126-145).

    python tests/golden/make_golden.py

Outputs:
  kat_manual.txt            20 expected output rows (copied from Rmd/Manual.Rmd:126-145)
  l_snps.txt                the 7 large-effect rsIDs of that example
  testdat_golden.json       beta per SNP for test_dat, tau 0.8 and 1.0, DBSLMM and LMM-only,
                            reference PCG and direct solve (float repr = 17 significant digits)
  synth_small/              a small synthetic panel with missing calls and n % 4 = 3, plus its
                            golden beta (ref.bed, meta.json, golden.json)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import ref_numpy as R  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
TD = os.path.join(GOLD, "test_dat")
BLOCKS = os.path.join(ROOT, "dbslmm_amd", "data", "block_data", "EUR", "chr1.bed")

KAT = """rs13302957 G 0.546652 1.82642 1
rs3748588 T 0.273432 1.64563 1
rs74045047 A -0.282306 -0.5378 1
rs3845292 G 0.159231 0.22554 1
rs113288277 T -0.0524222 -0.18273 1
rs112797925 A 0.252739 1.12303 1
rs12743678 A 0.741517 1.51564 1
rs141242758 C 0.00548007 0.0124342 0
rs28544273 A 0.0114189 0.0248473 0
rs3115860 C 0.00628248 0.013297 0
rs2073813 A 0.00771072 0.0164301 0
rs3131969 A 0.00191854 0.00404717 0
rs3131968 A 0.00191854 0.00404717 0
rs3131967 T 0.00191854 0.00404717 0
rs3115858 A 0.00415565 0.00876637 0
rs3131962 A 0.0112978 0.0237545 0
rs3115853 G 0.00251826 0.00529485 0
rs4951929 C 0.00443819 0.0093624 0
rs4951862 C 0.00256037 0.00540112 0
rs3131956 A 0.00341574 0.00720553 0
"""
L_SNPS = KAT.split("\n")[:7]
L_SNPS = [r.split()[0] for r in L_SNPS]


def testdat_infos(lmm_only: bool, maf_max: float = 0.2):
    """Host pipeline of BatchRun (dbslmm.cpp:232-317) on test_dat with the 7 large SNPs."""
    n_ref = R.get_row(os.path.join(TD, "ref_chr1.fam"))
    bim = R.read_bim(os.path.join(TD, "ref_chr1"), n_ref, abs(maf_max - 1.0) >= 1e-10)
    blocks = R.read_block(BLOCKS)
    summ = R.read_summ(os.path.join(TD, "summary_gemma_chr1.assoc.txt"))
    if lmm_only:
        ss, sl = summ, []
    else:
        ss = [s for s in summ if s.snp not in L_SNPS]
        sl = [s for s in summ if s.snp in L_SNPS]
    inter_s, _ = R.match_ref(ss, bim, maf_max)
    inter_l, _ = R.match_ref(sl, bim, maf_max)
    return n_ref, blocks, R.add_block(inter_s, blocks), R.add_block(inter_l, blocks)


def testdat_golden():
    bed = open(os.path.join(TD, "ref_chr1.bed"), "rb").read()
    out = {}
    for lmm in (False, True):
        n_ref, blocks, info_s, info_l = testdat_infos(lmm)
        kind = "lmm" if lmm else "dbslmm"
        out[kind] = dict(snp_s=[e["snp"] for e in info_s], snp_l=[e["snp"] for e in info_l])
        # tau 0.8 = current reference code with nsnp = wc -l (SURVEY config 1);
        # tau 1.0 / nsnp 998 = the setting that reproduces the Manual example
        for tau, nsnp in ((0.8, 996), (1.0, 998)):
            for method in ("pcg", "direct"):
                res = R.est(bed, n_ref, 2400, 0.5 / nsnp, len(blocks), info_s, info_l, tau=tau,
                            method=method)
                out[f"{kind}_tau{tau}_nsnp{nsnp}_{method}"] = dict(
                    beta_s=[float(x) for x in res.beta_s], beta_l=[float(x) for x in res.beta_l],
                    eff_txt=R.format_eff(res) if method == "pcg" else [])
    return out


def synth_small():
    """n_ref = 203 (n % 4 = 3), 0.5 % missing calls, 12 EUR chr22 blocks."""
    from dbslmm_amd import synth
    p = synth.simulate(600, 203, pop="EUR", chroms=[22], seed=7, miss_rate=0.005, large_every=3,
                       block_limit=12)
    d = os.path.join(GOLD, "synth_small")
    os.makedirs(d, exist_ok=True)
    p.bed.tofile(os.path.join(d, "ref.bed"))
    nb = len(p.blocks)
    infos_s, infos_l = [], []
    for j in range(p.m):
        e = dict(snp=f"s{j}", ps=int(p.ps[j]), pos=j, a1="A", maf=float(min(p.af[j], 1 - p.af[j])),
                 z=float(p.z[j]), block=int(p.block[j]))
        (infos_l if p.large[j] else infos_s).append(e)
    meta = dict(n_ref=p.n_ref, n_obs=p.n_obs, h2=p.h2, nsnp=p.m, num_block=nb, seed=7,
                block=p.block.tolist(), large=p.large.astype(int).tolist(), z=p.z.tolist())
    json.dump(meta, open(os.path.join(d, "meta.json"), "w"))
    bed = p.bed.tobytes()
    gold = {}
    for lmm in (False, True):
        s = infos_s + infos_l if lmm else infos_s
        s = sorted(s, key=lambda e: e["pos"]) if lmm else s
        l_ = [] if lmm else infos_l
        for method in ("pcg", "direct"):
            res = R.est(bed, p.n_ref, p.n_obs, p.h2 / p.m, nb, s, l_, tau=0.8, method=method)
            gold[f"{'lmm' if lmm else 'dbslmm'}_{method}"] = dict(
                pos_s=[e["pos"] for e in s], beta_s=[float(x) for x in res.beta_s],
                pos_l=[e["pos"] for e in l_], beta_l=[float(x) for x in res.beta_l])
    json.dump(gold, open(os.path.join(d, "golden.json"), "w"))


def main():
    with open(os.path.join(GOLD, "kat_manual.txt"), "w") as f:
        f.write(KAT)
    with open(os.path.join(GOLD, "l_snps.txt"), "w") as f:
        f.write("\n".join(L_SNPS) + "\n")
    json.dump(testdat_golden(), open(os.path.join(GOLD, "testdat_golden.json"), "w"))
    synth_small()


if __name__ == "__main__":
    main()
