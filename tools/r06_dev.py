"""Round 6: per-device breakdown of the PCG shard plan's rehearsal -- for config C and N devices,
each device's units plan timed alone on this GPU: wall step, HIP-event phase times (unpack, Gram,
PCG iterations), iterations, and the model's prediction.  GPU; usage:
python tools/r06_dev.py OUT_JSON [config] [N,N..]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbslmm_amd import Context, KERNEL_NAMES, Plan, synth      # noqa: E402
from dbslmm_amd.dist import shard_units_problem                 # noqa: E402

CFG = {3: (500_000, 5_000, "EUR", False, (1.0,)), 4: (1_000_000, 10_000, "EUR", False, (0.8, 1.0, 1.2)),
       5: (1_000_000, 10_000, "AFR", True, (1.0,))}


def main(out, cfg=4, ns=(1, 2, 4, 8), only=None):
    snps, n_ref, pop, lmm, f = CFG[cfg]
    pan = synth.simulate(snps, n_ref, pop=pop, seed=1, engine="gpu")
    prob = synth.make_problem(pan, lmm_only=lmm)
    del pan
    sig = [prob.sigma_s * x for x in f]
    K = len(sig)
    ctx = Context(0)
    m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    rec = dict(config=cfg, results={})
    for N in ns:
        ud, model = shard_units_problem(prob, sig, N)
        devs = []
        for d in range(N):
            if only is not None and d != only:
                continue
            plan = Plan.units(ctx, prob, ud, d)
            o = (np.zeros((K, prob.n_s)), np.zeros((K, prob.n_l)), np.zeros((K, prob.num_block), dtype=np.int32))
            for _ in range(3):
                plan.run_multi(sig, out=o)
            plan.enable_timing(True)
            batches = []
            for _ in range(7):                    # the median of seven batches of five solves (host noise)
                t0 = time.perf_counter()
                for _ in range(5):
                    plan.run_multi(sig, out=o)
                batches.append((time.perf_counter() - t0) / 5 * 1e3)
            wall = float(np.median(batches))
            ms, n = plan.kernel_ms()
            it = plan.block_iters()
            mine = ud[:, 0] == d
            devs.append(dict(wall_ms=wall, phases={KERNEL_NAMES[k]: float(ms[k]) for k in range(len(ms))},
                             blocks=int(mine.sum()), snps=int(m[mine].sum()), max_m=int(m[mine].max()),
                             iters_max=int(it.max()), model_ms=float(model[d]),
                             block_ids=np.flatnonzero(mine).tolist(), iters=it[mine].tolist()))
            plan.close()
            print(f"N={N} dev {d}: wall {wall:.3f} ms model {model[d]:.3f}  " +
                  " ".join(f"{k[7:]}={v:.3f}" for k, v in devs[-1]["phases"].items() if v > 0) +
                  f"  blocks {devs[-1]['blocks']} max_m {devs[-1]['max_m']} it {devs[-1]['iters_max']}", flush=True)
        rec["results"][str(N)] = devs
    json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    ns = tuple(int(x) for x in sys.argv[3].split(",")) if len(sys.argv) > 3 else (1, 2, 4, 8)
    only = int(sys.argv[4]) if len(sys.argv) > 4 else None      # one device of the plan (profiling)
    main(sys.argv[1], cfg, ns, only)
