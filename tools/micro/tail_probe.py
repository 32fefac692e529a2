"""Config-4 step with and without the result download (diagnostic probe, round 4): run_multi into
the caller's arrays (the bench step) vs run_multi with no result arrays (the solve alone), vs
plan.run_multi + the download split out.  python tools/micro/tail_probe.py [reps]"""
import ctypes as C
import sys
import time

sys.path[:0] = ["."]
import numpy as np
from dbslmm_amd import Context, Plan, synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
panel = synth.simulate(1_000_000, 10_000, seed=1, engine="gpu")
prob = synth.make_problem(panel)
del panel
sig = np.ascontiguousarray([prob.sigma_s * f for f in (0.8, 1.0, 1.2)], dtype=np.float64)
plan = Plan(Context(0), prob)
outs = (np.zeros((3, prob.n_s)), np.zeros((3, prob.n_l)), np.zeros((3, prob.num_block), dtype=np.int32))
lib = plan.ctx.lib
null = C.c_void_p(0)


def with_dl():
    plan.run_multi(sig, out=outs)


def without_dl():
    plan.ctx.check(lib.dbslmm_plan_run_multi(plan.h, sig.ctypes.data_as(C.c_void_p), 3, null, null, null),
                   "run_multi")


for f in (with_dl, without_dl):
    for _ in range(3):
        f()
res = {}
for rnd in range(3):
    for f in (with_dl, without_dl):
        t = time.perf_counter()
        for _ in range(reps):
            f()
        res.setdefault(f.__name__, []).append((time.perf_counter() - t) / reps * 1e3)
for k, v in res.items():
    print(f"{k:12s} ms/step " + " ".join(f"{x:.2f}" for x in v), flush=True)
