"""One big LD block alone (m SNPs x n_ref individuals): the tiled sequence without contention from
other blocks, for kernel-trace timing of the region / panel / trailing launches."""
import sys, time
sys.path[:0] = ['.']
import numpy as np
from dbslmm_amd import Context, Plan, synth

m = int(sys.argv[1]) if len(sys.argv) > 1 else 9600
n_ref = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
panel = synth.simulate(m, n_ref, block_limit=1, engine="gpu", large_every=0)
prob = synth.make_problem(panel)
print("blocks", prob.num_block, "m", np.diff(prob.s_ptr), flush=True)
plan = Plan(Context(0), prob)
for _ in range(2):
    plan.run()
plan.sync()
t = time.perf_counter()
for _ in range(3):
    plan.run()
plan.sync()
print("ms per run %.2f" % ((time.perf_counter() - t) / 3 * 1e3), flush=True)
