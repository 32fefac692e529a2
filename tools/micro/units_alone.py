"""One device's units plan of the N-device shard plan (config 4, h2f 0.8 / 1 / 1.2) timed alone on
this GPU -- what rank d of an N-GPU torchrun launch runs -- for kernel traces of a single device.
    python tools/micro/units_alone.py N d [runs] [KEY=VALUE ...]   (dbslmm_options fields)"""
import sys
import time
sys.path[:0] = ["."]
import numpy as np
from dbslmm_amd import Context, Plan, synth
from dbslmm_amd.dist import shard_units

N, d = int(sys.argv[1]), int(sys.argv[2])
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
panel = synth.simulate(1000000, 10000, pop="EUR", seed=1, engine="gpu", device=0)
full = synth.make_problem(panel)
del panel
sig = [full.sigma_s * f for f in (0.8, 1.0, 1.2)]
full.opts["shard_copies"] = 3
for kv in sys.argv[4:]:
    k, v = kv.split("=", 1)
    full.opts[k] = int(v)
m_b = np.diff(full.s_ptr) + (np.diff(full.l_ptr) if full.l_ptr is not None else 0)
ud, model = shard_units(m_b, full.n_ref, N, 3)
own = np.any(ud == d, axis=1)
print(f"device {d} of {N}: {int(own.sum())} blocks, {int(m_b[own].sum())} SNPs, model {model[d]:.2f} ms", flush=True)
plan = Plan.units(Context(0), full, ud, d)
o = (np.zeros((3, full.n_s)), np.zeros((3, full.n_l)), np.zeros((3, full.num_block), dtype=np.int32))
for _ in range(2):
    plan.run_multi(sig, out=o)
t = time.perf_counter()
for _ in range(runs):
    plan.run_multi(sig, out=o)
print(f"ms per run {(time.perf_counter() - t) / runs * 1e3:.2f}", flush=True)
plan.close()
