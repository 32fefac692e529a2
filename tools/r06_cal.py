"""Round 6: calibration data of the PCG shard model (multi.hip shard::pcg_*): per config 3-5 the
per-block SNPs / large SNPs / PCG iterations (dbslmm_plan_block_iters) and the one-GPU step, and the
model's prediction beside it.  GPU; usage: python tools/r06_cal.py OUT_DIR"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dbslmm_amd import Context, Plan, synth            # noqa: E402
from dbslmm_amd.dist import shard_units_problem        # noqa: E402

CFG = {3: (500_000, 5_000, "EUR", False, (1.0,)), 4: (1_000_000, 10_000, "EUR", False, (0.8, 1.0, 1.2)),
       5: (1_000_000, 10_000, "AFR", True, (1.0,))}


def main(out):
    os.makedirs(out, exist_ok=True)
    ctx = Context(0)
    for cfg, (snps, n_ref, pop, lmm, f) in CFG.items():
        pan = synth.simulate(snps, n_ref, pop=pop, seed=1, engine="gpu")
        prob = synth.make_problem(pan, lmm_only=lmm)
        del pan
        sig = [prob.sigma_s * x for x in f]
        plan = Plan(ctx, prob)
        for _ in range(3):
            plan.run_multi(sig)
        t0 = time.perf_counter()
        for _ in range(5):
            plan.run_multi(sig)
        ms = (time.perf_counter() - t0) / 5 * 1e3
        it = plan.block_iters()
        wl = plan.workload()
        plan.close()
        m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
        ml = np.diff(prob.l_ptr) if prob.l_ptr is not None else np.zeros_like(m)
        _, model = shard_units_problem(prob, sig, 1)
        rec = dict(config=cfg, step_ms=ms, model_ms=float(model[0]), pcg_iters=wl["pcg_iters"],
                   m=m.tolist(), ml=ml.tolist(), iters=it.tolist())
        json.dump(rec, open(os.path.join(out, f"iters_c{cfg}.json"), "w"))
        print(f"config {cfg}: step {ms:.3f} ms, model {model[0]:.3f} ms, max iters {int(it.max())}, "
              f"mean iters (blocks w/o large) {it[(m > 0) & (ml == 0)].mean():.2f}, "
              f"(with large) {it[ml > 0].mean() if (ml > 0).any() else float('nan'):.2f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r06/cal")
