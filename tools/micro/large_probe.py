"""Blocks of the single-workgroup path (dbslmm_chol_large: ld > 64, below the tiled threshold),
diagnostic: the kernel's time per run and, with the stamps build (make -C dbslmm_amd/csrc stamps,
STAMPS=1), its phases per block.
    python tools/micro/large_probe.py [m] [blocks] [n_ref]"""
import ctypes as C
import os
import sys
HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
STAMPS = os.environ.get("STAMPS") == "1"
if STAMPS:
    os.environ["DBSLMM_LIB_PATH"] = os.path.join(HERE, "dbslmm_amd", "libdbslmm_hip_stamps.so")
sys.path.insert(0, HERE)
import numpy as np  # noqa: E402
from dbslmm_amd import BlockProblem, Context, Plan, _lib  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 300
nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 376
n_ref = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
rng = np.random.default_rng(1)
nb = (n_ref + 3) // 4
rows = m * nblk
geno = rng.choice(np.array([0, 2, 3], dtype=np.uint8), size=(rows, 4 * nb), p=[0.25, 0.5, 0.25])
packed = (geno[:, 0::4] | (geno[:, 1::4] << 2) | (geno[:, 2::4] << 4) | (geno[:, 3::4] << 6)).astype(np.uint8)
del geno
bed = np.concatenate([np.array([0x6C, 0x1B, 0x01], np.uint8), packed.ravel()])
s_ptr = np.arange(nblk + 1, dtype=np.int64) * m
prob = BlockProblem(bed=bed, n_ref=n_ref, n_obs=50000, sigma_s=0.5 / 1e6, s_ptr=s_ptr,
                    s_pos=np.arange(rows, dtype=np.int32), z_s=rng.standard_normal(rows))
prob.opts["tiled_min"] = 1 << 20   # every block on the single-workgroup path
plan = Plan(Context(0), prob)
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
print("m", m, "blocks", nblk, "per run (ms):", {k: round(v / max(nrun, 1), 3) for k, v in zip(_lib.KERNEL_NAMES, ms)})
if STAMPS:
    L.dbslmm_debug_stamps(out.ctypes.data_as(C.c_void_p))
    ph = out[:4] / reps / nblk / 1e3    # counter ticks -> us per block (the scale region_probe.py uses; it matches the kernel traces)
    print("per block us: diag0 %.1f  panels %.1f  trailing (+ lookahead factor) %.1f  backward %.1f" % tuple(ph))
