"""Diagnostics: h2f run_multi on a small tiled problem, path chosen by the environment."""
import os
import sys
import time
here = os.path.dirname(os.path.abspath(__file__))
for d in ("..", "../tests", "../oracle"):
    sys.path.insert(0, os.path.join(here, d))
if os.environ.get("DBG_PKG"):
    sys.path.insert(0, os.environ["DBG_PKG"])
os.environ.setdefault("DBSLMM_TILED_MIN", "64")
from test_tiled import _problem  # noqa: E402
from dbslmm_amd import Context, Plan  # noqa: E402
prob = _problem(seed=5)
plan = Plan(Context(0), prob)
sig = [prob.sigma_s * f for f in (0.8, 1.0, 1.2)]
t = time.time()
import dbslmm_amd
print(dbslmm_amd.__file__)
print("start", os.environ.get("DBSLMM_H2F_CHEB"), os.environ.get("DBSLMM_TRSV_FUSE"), flush=True)
plan.run_multi(sig)
print("run_multi done", time.time() - t, flush=True)
