"""Tiled factorisation of one big block (diagnostic): tchol time per region and, with the
stamps build (make -C dbslmm_amd/csrc stamps), the region kernel's phases.
    python tools/region_probe.py [m] [n_ref]"""
import ctypes as C
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAMPS = os.environ.get("STAMPS") == "1"
if STAMPS:
    os.environ["DBSLMM_LIB_PATH"] = os.path.join(HERE, "dbslmm_amd", "libdbslmm_hip_stamps.so")
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
from dbslmm_amd import BlockProblem, Context, Plan, _lib  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
n_ref = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
rng = np.random.default_rng(1)
nb = (n_ref + 3) // 4
geno = rng.choice(np.array([0, 2, 3], dtype=np.uint8), size=(m, 4 * nb), p=[0.25, 0.5, 0.25])
packed = (geno[:, 0::4] | (geno[:, 1::4] << 2) | (geno[:, 2::4] << 4) | (geno[:, 3::4] << 6)).astype(np.uint8)
bed = np.concatenate([np.array([0x6C, 0x1B, 0x01], np.uint8), packed.ravel()])
nl = 8
pos = rng.permutation(m)
prob = BlockProblem(bed=bed, n_ref=n_ref, n_obs=50000, sigma_s=0.5 / 1e6,
                    s_ptr=np.array([0, m - nl]), s_pos=np.sort(pos[nl:]), z_s=rng.standard_normal(m - nl),
                    l_ptr=np.array([0, nl]), l_pos=np.sort(pos[:nl]), z_l=rng.standard_normal(nl))
ctx = Context(0)
plan = Plan(ctx, prob)
L = _lib.load()
out = np.zeros(16)
if STAMPS:
    L.dbslmm_debug_stamps.argtypes = [C.c_void_p]
plan.run()
plan.sync()
if STAMPS:
    L.dbslmm_debug_stamps(out.ctypes.data_as(C.c_void_p))
reps = 5
plan.enable_timing(True)
for _ in range(reps):
    plan.run()
plan.sync()
ms, nrun = plan.kernel_ms()
nreg = (m + 127) // 128
print("m", m, "regions", nreg, "per run (ms):", {k: round(v / max(nrun, 1), 3) for k, v in zip(_lib.KERNEL_NAMES, ms)})
if STAMPS:
    L.dbslmm_debug_stamps(out.ctypes.data_as(C.c_void_p))
    R = 4 if m >= 4096 else 2                      # regions per super step (plan.hip kWideMin)
    n_first = max(0, (nreg - 1) // R)               # first regions of super steps 1.. (no pending update)
    for lab, ph, n in (("other regions", out[:8], nreg - n_first), ("first of super step", out[8:16], n_first)):
        ph = ph / reps / max(n, 1) / 1e3
        print(("%s (%d) per launch us: load+update %.1f  4 steps %.1f  X10 %.1f  writeback %.1f"
               " | in the steps: factor (t>0) %.1f  panel %.1f  trailing %.1f  factor t=0 %.1f") % ((lab, n) + tuple(ph)))
