"""Fit the PCG-route shard model (multi.hip shard::kPcg*, PcgDev::time) to one-GPU rehearsals
(tools/r06_dev.py dev_c*.json): the model's own structure, evaluated on each rehearsed device's
blocks with the a-priori iteration counts the C++ planner uses --

  unpack  = u0 + bytes / u_rate                        (phase dbslmm_unpack_stats)
  gram    = g0 + huge_ops / g_huge + big_ops / g_big   (phase dbslmm_gram)
  pcg     = max(chip, fused, share (chip + fused)) + chip_iters * floor
            fused = max(quads / fused rate, longest sequence, sum of sequences / n_cu)
            (a sequence = one workgroup's Krylov run: iterations x quadrants x seq_us)
  wall    = unpack + gram + pcg + run + dl * results

Stage by stage: unpack and gram by linear least squares on their phases, the PCG constants by a
bounded nonlinear fit of the relative error of the dbslmm_pcg phase, run / dl on the rest of the
wall.  Prints the constants (C++ units) and every device's error.  CPU; usage:
python tools/fit_shard_model2.py DIR [configs, default 3,4,5]"""
import json
import math
import os
import sys

import numpy as np
from scipy.optimize import least_squares

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fit_shard_model import CFG, shape   # noqa: E402

FTB, NCU, TAU, TOL, NOBS = 8, 256, 0.8, 1e-12, 100_000


def iters_model(dmin, large):
    kap = 1.0 + 10.0 / max(1e-3, dmin + 1.0 - TAU)
    q = (math.sqrt(kap) - 1.0) / (math.sqrt(kap) + 1.0)
    return math.ceil(math.log(2.0 / TOL) / -math.log(q)) + (2 if large else 0)


def device_features(m, ml, n_ref, K, dmin):
    kp = math.ceil(n_ref / 128) * 128
    hm = 384 if kp >= 4096 else 768
    it = np.array([iters_model(dmin, x > 0) for x in ml], dtype=float)
    Tb, Q = np.ceil(m / 128), np.ceil(m / 64)
    nc = np.where((K > 1) & (ml > 0), K, 1)
    fused = Tb <= FTB
    ops = n_ref * m * (m + 1.0)
    seq = (it * Q * (Q + 1) / 2)[fused]                  # quadrant-iterations of one sequence
    return dict(unpack=float((m * (math.ceil(n_ref / 4) + kp / 4)).sum()),
                huge=float(ops[m >= hm].sum()), big=float(ops[m < hm].sum()),
                fq=float((nc[fused] * seq).sum()), seq_max=float(seq.max()) if seq.size else 0.0,
                ct=float((it * Tb * (Tb + 1) / 2 * (1 + 0.5 * (nc - 1)))[~fused].sum()),
                cr=float((it * Tb * nc)[~fused].sum()),
                citmax=float(it[~fused].max()) if (~fused).any() else 0.0,
                results=float((m * K).sum()))


def pcg_ms(f, p):
    fq_ns, seq_us, tile_ns, row_ns, floor_us, share = p
    fused = max(f["fq"] * fq_ns * 1e-6, f["seq_max"] * seq_us * 1e-3, f["fq"] * seq_us * 1e-3 / NCU)
    chip = (f["ct"] * tile_ns + f["cr"] * row_ns) * 1e-6
    return max(chip, fused, share * (chip + fused)) + f["citmax"] * floor_us * 1e-3


def main(d, cfgs=(3, 4, 5)):
    rows = []
    for cfg in cfgs:
        fn = os.path.join(d, f"dev_c{cfg}.json")
        if not os.path.exists(fn):
            continue
        rec = json.load(open(fn))
        m, ml, n_ref, K = shape(cfg)
        f_ = CFG[cfg][4]
        fac = (0.8, 1.0, 1.2) if f_ == 3 else (1.0,)
        nsnp = CFG[cfg][0]
        sig = [0.5 / nsnp * x for x in fac]               # sigma_s = h / nsnp (h = 0.5)
        dmin = min(1.0 / (s * NOBS) for s in sig)
        for N, devs in rec["results"].items():
            for dv in devs:
                ids = np.array(dv["block_ids"], dtype=int)
                ph = dv["phases"]
                rows.append(dict(cfg=cfg, N=int(N), f=device_features(m[ids], ml[ids], n_ref, K, dmin),
                                 wall=dv["wall_ms"], unpack=ph["dbslmm_unpack_stats"], gram=ph["dbslmm_gram"],
                                 pcg=ph["dbslmm_pcg"]))
    U = np.array([[1.0, r["f"]["unpack"]] for r in rows]); ut = np.array([r["unpack"] for r in rows])
    (u0, ur), *_ = np.linalg.lstsq(U / ut[:, None], np.ones_like(ut), rcond=None)
    G = np.array([[1.0, r["f"]["huge"], r["f"]["big"]] for r in rows]); gt = np.array([r["gram"] for r in rows])
    (g0, gh, gb), *_ = np.linalg.lstsq(G / gt[:, None], np.ones_like(gt), rcond=None)
    pt = np.array([r["pcg"] for r in rows])
    p0 = [2.39, 0.43, 5.76, 43.6, 32.9, 0.69]
    res = least_squares(lambda p: np.array([pcg_ms(r["f"], p) for r in rows]) / pt - 1.0, p0,
                        bounds=([0.1, 0.01, 0.1, 1.0, 0.0, 0.5], [20, 5, 50, 500, 100, 1.0]))
    pp = res.x
    pm = np.array([pcg_ms(r["f"], pp) for r in rows])
    front = U @ [u0, ur] + G @ [g0, gh, gb]
    R = np.array([r["f"]["results"] for r in rows]); wall = np.array([r["wall"] for r in rows])
    (o0, o1), *_ = np.linalg.lstsq(np.stack([np.ones_like(R), R * 1e-6], 1) / wall[:, None],
                                   (wall - front - pm) / wall, rcond=None)
    print(f"constexpr double kPcgUnpackMs0 = {u0:.4f}, kPcgUnpackBps = {1e3 / ur:.3e};")
    print(f"constexpr double kPcgGramMs0 = {g0:.4f};")
    print(f"constexpr double kPcgGramOpsHuge = {1e3 / gh:.3e}, kPcgGramOpsBig = {1e3 / gb:.3e};")
    print(f"constexpr double kPcgFusedQuadNs = {pp[0]:.3f};\nconstexpr double kPcgSeqQuadUs = {pp[1]:.4f};")
    print(f"constexpr double kPcgTileNs = {pp[2]:.3f};\nconstexpr double kPcgRowNs = {pp[3]:.2f};")
    print(f"constexpr double kPcgIterFloorUs = {pp[4]:.2f};\nconstexpr double kPcgShare = {pp[5]:.3f};")
    print(f"constexpr double kPcgRunMs = {o0:.4f};\nconstexpr double kPcgDownloadMsPerM = {o1:.4f};")
    model = front + pm + o0 + o1 * R * 1e-6
    err = (model - wall) / wall
    for r, mo, e, pmi in zip(rows, model, err, pm):
        print(f"  c{r['cfg']} N={r['N']}: wall {r['wall']:.3f} model {mo:.3f} ({e:+.1%})  pcg {r['pcg']:.3f} vs {pmi:.3f}")
    for cfg in cfgs:
        for N in (1, 2, 4, 8):
            sel = [i for i, r in enumerate(rows) if r["cfg"] == cfg and r["N"] == N]
            if sel:
                st, pr = wall[sel].max(), model[sel].max()
                print(f"c{cfg} N={N}: step {st:.3f} predicted {pr:.3f} ({(pr - st) / st:+.1%})")


if __name__ == "__main__":
    main(sys.argv[1], tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (3, 4, 5))
