"""Fit the PCG-route shard model (multi.hip shard::kPcg*) to one-GPU rehearsals: per config the
per-device phase times of tools/r06_dev.py (unpack, Gram, PCG iterations, wall; block lists and
measured iterations per device) against the model's features of the same blocks.  Prints the
fitted rates and each device's model error.  CPU; usage:
python tools/fit_shard_model.py DIR [configs, default 3,4,5]"""
import json
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbslmm_amd import synth   # noqa: E402

CFG = {3: (500_000, 5_000, "EUR", False, 1), 4: (1_000_000, 10_000, "EUR", False, 3),
       5: (1_000_000, 10_000, "AFR", True, 1)}
FTB = 8


def shape(cfg):
    snps, n_ref, pop, lmm, K = CFG[cfg]
    pan = synth.simulate(snps, n_ref, pop=pop, seed=1, engine="none")
    prob = synth.make_problem(pan, lmm_only=lmm)
    m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    ml = np.diff(prob.l_ptr) if prob.l_ptr is not None else np.zeros_like(m)
    return m, ml, n_ref, K


def features(m, ml, n_ref, K, it):
    """per-device feature dict from its blocks (m, ml, measured iterations it)"""
    kp = math.ceil(n_ref / 128) * 128
    hm = 384 if kp >= 4096 else 768
    Tb = np.ceil(m / 128)
    nc = np.where((K > 1) & (ml > 0), K, 1)
    fused = Tb <= FTB
    Q = np.ceil(m / 64)
    ops = n_ref * m * (m + 1.0)
    return dict(
        unpack=float((m * (math.ceil(n_ref / 4) + kp / 4)).sum()),
        gram_huge=float(ops[m >= hm].sum()), gram_big=float(ops[m < hm].sum()), kp=kp,
        fq=float((nc * it * Q * (Q + 1) / 2)[fused].sum()),
        ct=float((it * Tb * (Tb + 1) / 2 * (1 + 0.5 * (nc - 1)))[~fused].sum()),
        cr=float((it * Tb * nc)[~fused].sum()),
        citmax=float(it[~fused].max()) if (~fused).any() else 0.0,
        results=float((m * K).sum()))


def main(d, cfgs=(3, 4, 5)):
    rows = []
    for cfg in cfgs:
        f = os.path.join(d, f"dev_c{cfg}.json")
        if not os.path.exists(f):
            continue
        rec = json.load(open(f))
        m, ml, n_ref, K = shape(cfg)
        for N, devs in rec["results"].items():
            for dv in devs:
                ids = np.array(dv["block_ids"], dtype=int)
                it = np.array(dv["iters"], dtype=float)
                ft = features(m[ids], ml[ids], n_ref, K, it)
                ph = dv["phases"]
                rows.append(dict(cfg=cfg, N=int(N), ft=ft, wall=dv["wall_ms"], unpack=ph["dbslmm_unpack_stats"],
                                 gram=ph["dbslmm_gram"], pcg=ph["dbslmm_pcg"]))
    if not rows:
        print("no data")
        return
    # unpack: bytes / rate
    ub = np.array([r["ft"]["unpack"] for r in rows]); ut = np.array([r["unpack"] for r in rows])
    u_rate = (ub @ ub) / (ub @ ut) * 1e-9   # TB/s... bytes per ms -> (bytes/ms)/1e9 = TB/s
    print(f"unpack: {u_rate:.3f} TB/s  (rel. err max {np.max(np.abs(ub / (u_rate * 1e9) - ut) / ut):.2%})")
    # gram: time = a * huge_ops * (kp + k0)/kp + b * big_ops
    k0 = 4074.0
    A = np.array([[r["ft"]["gram_huge"] * (r["ft"]["kp"] + k0) / r["ft"]["kp"], r["ft"]["gram_big"]] for r in rows])
    gt = np.array([r["gram"] for r in rows])
    (ga, gb), *_ = np.linalg.lstsq(A, gt, rcond=None)
    print(f"gram: huge {1e-12 / ga:.3f} Pops/s at kpad -> inf (k0 {k0:.0f}), big {1e-12 / gb:.3f} Pops/s  "
          f"(rel. err max {np.max(np.abs(A @ [ga, gb] - gt) / gt):.2%})")
    # pcg: time = max(chip, fused); fit fused rate on devices where fused dominates, chip on the rest
    F = np.array([r["ft"]["fq"] for r in rows]); CT = np.array([r["ft"]["ct"] for r in rows])
    CR = np.array([r["ft"]["cr"] for r in rows]); CI = np.array([r["ft"]["citmax"] for r in rows])
    pt = np.array([r["pcg"] for r in rows])
    X = np.stack([F, CT, CR, CI], axis=1)
    coef, *_ = np.linalg.lstsq(X, pt, rcond=None)
    print("pcg (linear): us per fused quadrant-iteration %.4f, chip tile-iteration %.4f, chip row-col-iteration %.4f, "
          "per chip iteration %.2f" % tuple(c * 1e3 for c in coef))
    pred = X @ coef
    print(f"  rel. err max {np.max(np.abs(pred - pt) / pt):.2%}, mean {np.mean(np.abs(pred - pt) / pt):.2%}")
    ov = np.array([r["wall"] - r["unpack"] - r["gram"] - r["pcg"] for r in rows])
    R = np.array([r["ft"]["results"] for r in rows])
    (oa, ob), *_ = np.linalg.lstsq(np.stack([np.ones_like(R), R * 1e-6], 1), ov, rcond=None)
    print(f"other (wall - phases): {oa:.3f} ms + {ob:.3f} ms per M results")
    for r, p in zip(rows, pred):
        full = r["ft"]["unpack"] / (u_rate * 1e9) + A[rows.index(r)] @ [ga, gb] + p + oa + ob * r["ft"]["results"] * 1e-6
        print(f"  c{r['cfg']} N={r['N']}: wall {r['wall']:.3f} model {full:.3f} ({(full - r['wall']) / r['wall']:+.1%})"
              f"  pcg {r['pcg']:.3f} vs {p:.3f}")


if __name__ == "__main__":
    main(sys.argv[1], tuple(int(x) for x in sys.argv[2].split(",")) if len(sys.argv) > 2 else (3, 4, 5))
