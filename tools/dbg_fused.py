"""Round 6 debug: run-to-run differences of the PCG route per block, whole-block kernel on / off."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "tests"),
                os.path.join(os.path.dirname(HERE), "oracle")]
from test_tiled import _problem          # noqa: E402
from dbslmm_amd import Context, Plan     # noqa: E402


def runs(prob, sig, k=3):
    out = []
    for _ in range(k):
        p = Plan(Context(0), prob)
        r = p.run_multi(sig)
        out.append((r, p.block_iters(), p.workload()["pcg_iters"]))
        p.close()
    return out


prob = _problem(seed=11, n_ref=512, sizes=[60, 200, 700, 1100, 130], mono_block=4, miss_rate=0.0)
prob.sigma_s = 0.5 / 1e6
for fz in ("1", "0"):
    os.environ["DBSLMM_PCG_FUSED"] = fz
    for f in ((1.0,), (0.8, 1.0, 1.2)):
        sig = [prob.sigma_s * x for x in f]
        o = runs(prob, sig)
        print(f"fused={fz} copies={len(f)} iters per block {[x[1].tolist() for x in o]}")
        for c in range(len(f)):
            for b in range(prob.num_block):
                s0, s1, l0, l1 = prob.s_ptr[b], prob.s_ptr[b + 1], prob.l_ptr[b], prob.l_ptr[b + 1]
                v = [np.concatenate([x[0][c][0][s0:s1], x[0][c][1][l0:l1]]) for x in o]
                d = max(float(np.nanmax(np.abs(v[0] - w))) if np.isfinite(v[0]).any() else 0.0 for w in v[1:])
                st = [int(x[0][c][2][b]) for x in o]
                print(f"  copy {c} block {b} m={s1 - s0 + l1 - l0} status {st} run-to-run max|d| {d:.3e}")
