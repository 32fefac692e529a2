import sys, numpy as np
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/oracle")
from _common import td_problem, normwise
from test_pcg import _prob, _run, _cat
import json
G = json.load(open("/root/repo/tests/golden/testdat_golden.json"))
d = td_problem(lmm_only=False)
gd = G["dbslmm_tau0.8_nsnp996_direct"]
ref = np.concatenate([gd["beta_s"], gd["beta_l"]])
for maxit in (1, 2, 3, 5, 10, 40, 0):
    (res,), wl = _run(_prob(d, solver=2, pcg_maxit=maxit))
    got = _cat(res)
    print("maxit", maxit, "iters", wl["pcg_iters"], "normwise", normwise(got, ref), "max|b|", np.abs(got).max(), "st", set(res[2].tolist()), flush=True)
