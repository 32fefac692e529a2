"""Round 6: the largest config-4 block (9.7k SNPs, h2f x 3) solved alone on the PCG route -- its
own units plan (every other block on a second, untimed device), wall time per run and HIP-event
phases.  The VERDICT r05 bar: <= 4 ms.  GPU; usage: python tools/r06_big.py OUT_JSON [config]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbslmm_amd import Context, KERNEL_NAMES, Plan, synth      # noqa: E402
from r06_dev import CFG                                          # noqa: E402


def main(out, cfg=4):
    snps, n_ref, pop, lmm, f = CFG[cfg]
    pan = synth.simulate(snps, n_ref, pop=pop, seed=1, engine="gpu")
    prob = synth.make_problem(pan, lmm_only=lmm)
    del pan
    sig = [prob.sigma_s * x for x in f]
    K = len(sig)
    m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    rec = dict(config=cfg, results=[])
    ctx = Context(0)
    for b in np.argsort(-m)[:3]:                 # the three largest blocks, each alone
        ud = np.ones((prob.num_block, K), dtype=np.int32)
        ud[b, :] = 0
        plan = Plan.units(ctx, prob, ud, 0)
        o = (np.zeros((K, prob.n_s)), np.zeros((K, prob.n_l)), np.zeros((K, prob.num_block), dtype=np.int32))
        for _ in range(3):
            plan.run_multi(sig, out=o)
        plan.enable_timing(True)
        batches = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(10):
                plan.run_multi(sig, out=o)
            batches.append((time.perf_counter() - t0) / 10 * 1e3)
        ms, _ = plan.kernel_ms()
        it = plan.block_iters()
        r = dict(block=int(b), m=int(m[b]), wall_ms=float(np.median(batches)), iters=int(it.max()),
                 status=o[2][:, b].tolist(),
                 phases={KERNEL_NAMES[k]: float(ms[k]) for k in range(len(ms)) if ms[k] > 0})
        rec["results"].append(r)
        plan.close()
        print(json.dumps(r), flush=True)
    json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4)
