"""Gram phase alone on uniform LD blocks: B blocks of m SNPs x n_ref individuals (LMM-only, lead
group off), the Gram's HIP-event time and its rate against the i8 / FP4 dense peaks.

    python tools/micro/gram_probe.py [m [B [n_ref]]]     (m = 0: the config-4 EUR layout)
"""
import sys
sys.path[:0] = ['.']
import numpy as np
from dbslmm_amd import BlockProblem, Context, Plan, KERNEL_NAMES, synth

m = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n_ref = int(sys.argv[3]) if len(sys.argv) > 3 else 10000
if m > 0:
    panel = synth.simulate(m * nb, n_ref, engine="gpu", large_every=0)
    n = m * nb
    prob = BlockProblem(bed=panel.bed, n_ref=n_ref, n_obs=100000, sigma_s=0.5 / n,
                        s_ptr=np.arange(0, n + 1, m, dtype=np.int64),
                        s_pos=np.arange(n, dtype=np.int32), z_s=panel.z[:n].copy(),
                        opts=dict(lead_min=-1))
else:
    panel = synth.simulate(1000000, n_ref, engine="gpu")
    prob = synth.make_problem(panel)
    prob.opts = dict(lead_min=-1)
plan = Plan(Context(0), prob)
plan.enable_timing(True)
for _ in range(2):
    plan.run()
plan.sync()
reps = 5
acc = np.zeros(len(KERNEL_NAMES))
for _ in range(reps):
    plan.run()
    plan.sync()
    ms, _ = plan.kernel_ms()
    acc += ms
acc /= reps
wl = plan.workload()
g = KERNEL_NAMES.index("dbslmm_gram_i8")
t = acc[g] * 1e-3
print(f"m={m} blocks={nb} n_ref={n_ref}: gram {acc[g]:.3f} ms, alg {wl['gram_ops_alg']:.3e} ops -> "
      f"{wl['gram_ops_alg'] / t / 1e12:.0f} TOPS ({wl['gram_ops_alg'] / t / 5e15:.3f} of i8, "
      f"{wl['gram_ops_alg'] / t / 1e16:.3f} of FP4); executed {wl['gram_ops_exec'] / t / 1e16:.3f} of FP4",
      flush=True)
print({k: round(float(v), 3) for k, v in zip(KERNEL_NAMES, acc)}, flush=True)
