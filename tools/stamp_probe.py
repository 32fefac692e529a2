"""Per-phase tick counters of the large Cholesky path (needs libdbslmm_hip_stamps.so)."""
import ctypes as C, os, sys
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DBSLMM_LIB_PATH"] = os.path.join(HERE, "dbslmm_amd", "libdbslmm_hip_stamps.so")
sys.path.insert(0, HERE); sys.path.insert(0, os.path.join(HERE, "tools"))
import numpy as np
from dbslmm_amd import _lib
exec(open(os.path.join(HERE, "tools", "chol_probe.py")).read().split("cases = {")[0])
L = _lib.load(); L.dbslmm_debug_stamps.argtypes = [C.c_void_p]
out = np.zeros(8)
for name, mask in {"largest": m_blk == m_blk.max(), "m64-128": (m_blk > 63) & (m_blk <= 128)}.items():
    prob = subset(mask); plan = Plan(ctx, prob)
    plan.run(); plan.sync(); L.dbslmm_debug_stamps(out.ctypes.data_as(C.c_void_p))
    reps = 5
    for _ in range(reps): plan.run()
    plan.sync(); L.dbslmm_debug_stamps(out.ctypes.data_as(C.c_void_p))
    nb = int(mask.sum())
    print(name, "blocks", nb, "per-block us: diag %.1f panel %.1f trailing %.1f backward %.1f | factor_diag: load %.1f factor %.1f inverse %.1f writeback %.1f" % tuple(out[:8] / reps / nb / 1e3))
