"""End-to-end CLI timing of config 4 (diagnostic, round 4): PLINK files written once; process
start-up + exit alone (`dbslmm` with no arguments); the CLI run three times with --timing; then
once under rocprofv3 with the kernel, HIP runtime and memory-copy traces (gpurun_out/e2e2/)."""
import os, subprocess, sys, tempfile, time
sys.path[:0] = ['.']
from dbslmm_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cli = os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm")
panel = synth.simulate(1000000, 10000, engine="gpu")
d = tempfile.mkdtemp(prefix="e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
f = synth.write_plink(panel, d)
del panel
cmd = [cli, "-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]), "-nsnp", str(f["nsnp"]),
       "-h", "0.5", "-mafMax", "0.2", "-h2f", "0.8,1,1.2", "-eff", os.path.join(d, "eff"), "--timing"]
print(subprocess.run(["df", "-T", d], capture_output=True, text=True).stdout, flush=True)
for i in range(3):
    t = time.perf_counter()
    subprocess.run([cli], capture_output=True)
    print("startup+exit (no args) %.3f s" % (time.perf_counter() - t), flush=True)
for pt in os.environ.get("VARIANTS", "--parse-threads 8").split(","):
    for i in range(int(os.environ.get("RUNS", "3"))):
        t = time.perf_counter()
        c2 = list(cmd)
        if os.environ.get("FRESH_EFF") == "1":
            c2[c2.index("-eff") + 1] = os.path.join(d, f"eff_{pt.replace(' ', '')}_{i}")
        r = subprocess.run(c2 + pt.split(), capture_output=True, text=True)
        t_end, wall = time.time(), time.perf_counter() - t
        ex = [float(x.split()[1]) for x in r.stderr.splitlines() if x.startswith("EXIT_AT")]
        print(pt, "run", i, "rc", r.returncode, "wall %.3f" % wall,
              "exit %.3f" % (t_end - ex[-1]) if ex else "",
              [x for x in r.stderr.splitlines() if x.startswith("TIMING")], flush=True)
if os.environ.get("PROF", "1") == "1":
    out = os.path.join(ROOT, "gpurun_out", "e2e2")
    os.makedirs(out, exist_ok=True)
    r = subprocess.run(["rocprofv3", "--kernel-trace", "--hip-runtime-trace", "--memory-copy-trace",
                        "--output-format", "csv", "-d", out, "-o", "cli", "--"] + cmd, capture_output=True, text=True)
    print("prof rc", r.returncode, [x for x in r.stderr.splitlines() if x.startswith("TIMING")], flush=True)
