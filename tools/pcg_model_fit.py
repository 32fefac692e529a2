"""Fit the PCG shard model's rates (multi.hip shard::kPcg*) from a calibration run: per config the
per-block iterations (tools/r06_cal.py iters_c*.json) and the rocprofv3 kernel trace of the bench
(prof/c*_results.db).  Work per launch is weighted by the blocks still iterating: a block's tiles
and tile rows count in the launches up to its own iteration count.  CPU; usage:
python tools/pcg_model_fit.py CAL_DIR [PROF_DIR]"""
import json
import math
import os
import sqlite3
import sys

import numpy as np


def kernels(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels").fetchall()
    out = {}
    for name, s, e in rows:
        out.setdefault(name.split("(")[0], []).append((e - s) * 1e-3)
    return {k: np.array(v) for k, v in out.items()}


def main(cal, prof=None):
    prof = prof or os.path.join(cal, "prof")
    for cfg in (3, 4, 5):
        f = os.path.join(cal, f"iters_c{cfg}.json")
        db = os.path.join(prof, f"c{cfg}_results.db")
        if not (os.path.exists(f) and os.path.exists(db)):
            continue
        r = json.load(open(f))
        m, ml, it = np.array(r["m"]), np.array(r["ml"]), np.array(r["iters"])
        K = 3 if cfg == 4 else 1
        ne = m > 0
        m, ml, it = m[ne], ml[ne], it[ne]
        Tb = np.ceil(m / 128)
        tiles = Tb * (Tb + 1) / 2
        nc = np.where((K > 1) & (ml > 0), K, 1)
        k = kernels(db)
        runs = len(k.get("dbslmm_pcg_init", [])) or 8
        sym = k.get("dbslmm_pcg_symv16d", k.get("dbslmm_pcg_symv16"))
        per_run = {n: v.sum() / runs for n, v in k.items()}
        work_t = (tiles * it).sum()
        work_tn = (tiles * nc * it).sum()
        work_r = (Tb * nc * it).sum()
        n_ref = 5000 if cfg == 3 else 10000
        kp = math.ceil(n_ref / 128) * 128
        hm = 384 if kp >= 4096 else 768
        ops = n_ref * m * (m + 1.0)
        print(f"config {cfg}: runs {runs}, launches/run {len(sym) / runs:.1f}, it max {it.max()}")
        print(f"  symv  {sym.sum() / runs:8.1f} us/run  -> {sym.sum() / runs / work_t * 1e3:.2f} ns per tile-iteration"
              f" ({sym.sum() / runs / work_tn * 1e3:.2f} per tile-column)")
        rw = per_run.get("dbslmm_pcg_rows", 0) + per_run.get("dbslmm_pcg_update", 0)
        print(f"  rows+update {rw:8.1f} us/run -> {rw / work_r * 1e3:.2f} ns per tile-row-column-iteration")
        gh = per_run.get("dbslmm_gram_huge", 0)
        gb = per_run.get("dbslmm_gram_big", 0) + per_run.get("dbslmm_gram_i8", 0)
        print(f"  gram huge {gh:8.1f} us -> {ops[m >= hm].sum() / gh * 1e-9 * 1e3 / 1e3:.3f} Pops/s;"
              f" big {gb:8.1f} us -> {ops[m < hm].sum() / max(gb, 1e-9) * 1e-9:.3f} Pops/s")
        up = per_run.get("dbslmm_unpack_stats", 0)
        ub = m.sum() * (math.ceil(n_ref / 4) + kp / 4)
        print(f"  unpack {up:8.1f} us -> {ub / up * 1e-6:.2f} TB/s")
        oth = sum(v for n, v in per_run.items() if "rocclr" in n or n in ("dbslmm_pcg_init", "dbslmm_pcg_final",
                                                                          "dbslmm_set_scalar"))
        print(f"  other (copies, fills, init, final) {oth:8.1f} us/run; step {r['step_ms']:.3f} ms")


if __name__ == "__main__":
    main(*sys.argv[1:])
