"""Diagnostics: per-tile timeline of the forward substitution for the largest tiled block
(DBSLMM_TRSV_STAMPS=1, config-4 h2f run): claim -> last hand-off staged -> stream done -> publish.
Needs the diagnostic build (make -C dbslmm_amd/csrc diag -> libdbslmm_hip_diag.so).
    python tools/trsv_stamps.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DBSLMM_TRSV_STAMPS"] = "1"
os.environ["DBSLMM_LIB_PATH"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                             "dbslmm_amd", "libdbslmm_hip_diag.so")
from dbslmm_amd import Context, Plan, synth  # noqa: E402

panel = synth.simulate(1000000, 10000, pop="EUR", seed=1, engine="gpu", device=0)
prob = synth.make_problem(panel)
plan = Plan(Context(0), prob)
sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
plan.run_multi(sig)
plan.run_multi(sig)
T = 150
out = np.zeros(8 * 4096, dtype=np.uint64)
fn = plan.ctx.lib.dbslmm_diag_trsv_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
rc = fn(plan.h, out.ctypes.data_as(ctypes.c_void_p), len(out))
assert rc == 0, rc
s = out[:8 * T].reshape(T, 8).astype(np.int64)
t0 = s[s > 0].min()
s = np.where(s > 0, (s - t0) * 10, 0) / 1000.0   # us
print("tile  claim  staged  streamed  published   step | reduced  vs-ready  stored  (us after streamed)")
prev = 0.0
for i in range(T):
    if s[i, 3] == 0:
        break
    print(f"{i:4d} {s[i,0]:7.1f} {s[i,1]:7.1f} {s[i,2]:8.1f} {s[i,3]:9.1f}   {s[i,3]-prev:6.2f} | "
          f"{s[i,4]-s[i,2]:6.2f} {s[i,5]-s[i,2]:6.2f} {s[i,6]-s[i,2]:6.2f}")
    prev = s[i, 3]
