"""End-to-end CLI run of config 4 (diagnostic): writes the synthetic panel as PLINK files, runs the
dbslmm CLI once plain and once under rocprofv3 --kernel-trace (output under gpurun_out/e2e_prof)."""
import json, os, subprocess, sys, tempfile, time
sys.path[:0] = ['.']
from dbslmm_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
panel = synth.simulate(1000000, 10000, engine="gpu")
d = tempfile.mkdtemp(prefix="e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
f = synth.write_plink(panel, d)
cmd = [os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm"), "-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"],
       "-n", str(f["n"]), "-nsnp", str(f["nsnp"]), "-h", "0.5", "-mafMax", "0.2", "-h2f", "0.8,1,1.2",
       "-eff", os.path.join(d, "eff"), "--timing"]
hold = None
if os.environ.get("HOLD") == "1":   # keep a solved plan of the same workload alive (as bench.py does)
    from dbslmm_amd import Context, Plan
    prob = synth.make_problem(panel)
    hold = Plan(Context(0), prob)
    sig = [prob.sigma_s * x for x in (0.8, 1.0, 1.2)]
    for _ in range(3):
        hold.run_multi(sig)
    hold.sync()
    print("holding a plan", flush=True)
for i in range(2):
    t = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True)
    print("run", i, "rc", r.returncode, "wall %.3f" % (time.perf_counter() - t),
          [x for x in r.stderr.splitlines() if x.startswith("TIMING")], flush=True)
out = os.path.join(ROOT, "gpurun_out", "e2e_prof")
os.makedirs(out, exist_ok=True)
r = subprocess.run(["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", out, "-o", "cli", "--"] + cmd,
                   capture_output=True, text=True)
print("prof rc", r.returncode, [x for x in r.stderr.splitlines() if x.startswith("TIMING")], flush=True)
