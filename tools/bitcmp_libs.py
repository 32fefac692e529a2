"""Bit-identity of two library builds on one workload: each build solves the same synthetic panel
in its own child process (DBSLMM_LIB_PATH) and writes its betas; the parent compares them.
python tools/bitcmp_libs.py CONFIG lib_a.so lib_b.so   (CONFIG 3: 500k x 5k, 4: 1M x 10k h2f)"""
import os
import subprocess
import sys

import numpy as np

CFG = {3: (500_000, 5_000, None), 4: (1_000_000, 10_000, (0.8, 1.0, 1.2))}

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    cfg, out = int(sys.argv[2]), sys.argv[3]
    sys.path[:0] = ["."]
    from dbslmm_amd import Context, Plan, synth
    snps, n_ref, h2f = CFG[cfg]
    panel = synth.simulate(snps, n_ref, seed=1, engine="gpu")
    prob = synth.make_problem(panel)
    del panel
    plan = Plan(Context(0), prob)
    for _ in range(2):   # the second run goes through the captured graphs
        if h2f:
            res = plan.run_multi([prob.sigma_s * f for f in h2f])
        else:
            plan.run()
            res = [plan.download()]
    np.savez(out, **{f"s{i}": r[0] for i, r in enumerate(res)}, **{f"l{i}": r[1] for i, r in enumerate(res)},
             **{f"t{i}": r[2] for i, r in enumerate(res)})
    sys.exit(0)

cfg = int(sys.argv[1])
outs = []
for k, lib in enumerate(sys.argv[2:4]):
    out = f"gpurun_out/bitcmp_{k}.npz"
    env = dict(os.environ, DBSLMM_LIB_PATH=os.path.abspath(lib))
    r = subprocess.run([sys.executable, __file__, "--child", str(cfg), out], env=env, timeout=600)
    if r.returncode:
        sys.exit(f"{lib}: rc {r.returncode}")
    outs.append(np.load(out))
a, b = outs
bad = 0
for key in a.files:
    x, y = a[key], b[key]
    same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    diff = 0.0 if same or x.dtype.kind != "f" else float(np.max(np.abs(x - y)))
    print(f"{key}: n={x.size} bit-identical={same}" + ("" if same else f" max|diff|={diff:.3g}"))
    bad += not same
print("BITCMP", "OK" if not bad else f"{bad} arrays differ")
sys.exit(1 if bad else 0)
