"""Time the three kernels on subsets of the config-2 blocks (diagnostic)."""
import sys, os, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from dbslmm_amd import Context, Plan, BlockProblem, synth

p = synth.simulate(int(sys.argv[1]) if len(sys.argv) > 1 else 50000, 2000, seed=1)
full = synth.make_problem(p)
ctx = Context(0)
m_blk = np.diff(full.s_ptr) + np.diff(full.l_ptr)

def subset(mask):
    nb = len(m_blk)
    keep_b = np.flatnonzero(mask)
    s_idx = np.concatenate([np.arange(full.s_ptr[b], full.s_ptr[b+1]) for b in keep_b]) if len(keep_b) else np.zeros(0, int)
    l_idx = np.concatenate([np.arange(full.l_ptr[b], full.l_ptr[b+1]) for b in keep_b]) if len(keep_b) else np.zeros(0, int)
    s_ptr = np.concatenate([[0], np.cumsum(np.diff(full.s_ptr)[keep_b])])
    l_ptr = np.concatenate([[0], np.cumsum(np.diff(full.l_ptr)[keep_b])])
    return BlockProblem(bed=full.bed, n_ref=full.n_ref, n_obs=full.n_obs, sigma_s=full.sigma_s,
                        s_ptr=s_ptr, s_pos=full.s_pos[s_idx], z_s=full.z_s[s_idx],
                        l_ptr=l_ptr, l_pos=full.l_pos[l_idx], z_l=full.z_l[l_idx])

cases = {
    "all": m_blk >= 0,
    "small(m<=63)": (m_blk > 0) & (m_blk <= 63),
    "large(m>63)": m_blk > 63,
    "largest": m_blk == m_blk.max(),
    "m64-128": (m_blk > 63) & (m_blk <= 128),
}
for name, mask in cases.items():
    prob = subset(mask)
    plan = Plan(ctx, prob)
    for _ in range(3): plan.run()
    plan.sync()
    plan.enable_timing(True)
    for _ in range(10): plan.run()
    plan.sync()
    ms, n = plan.kernel_ms()
    print(f"{name:14s} blocks={int(mask.sum()):5d} snps={prob.n_s+prob.n_l:6d} max_m={int(m_blk[mask].max()) if mask.any() else 0:4d}"
          f"  unpack={ms[0]*1e3:8.1f}us gram={ms[1]*1e3:8.1f}us chol={ms[2]*1e3:8.1f}us", flush=True)
