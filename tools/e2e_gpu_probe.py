"""Runs tools/micro/e2e_gpu_probe on the config-4 reference panel (PLINK files written once), three
times, with and without a plan-sized allocation, timing each process from outside too."""
import os, subprocess, sys, tempfile, time
sys.path[:0] = ['.']
from dbslmm_amd import synth
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
panel = synth.simulate(1000000, 10000, engine="gpu")
d = tempfile.mkdtemp(prefix="e2eg_", dir=os.environ.get("TMPDIR", "/tmp"))
f = synth.write_plink(panel, d)
exe = os.path.join(ROOT, "tools", "micro", "e2e_gpu_probe")
for gib in ("0", "0", "0", "12", "30"):
    t = time.perf_counter()
    r = subprocess.run([exe, f["ref"] + ".bed", "10000", str(panel.m), gib], capture_output=True, text=True)
    print(f"--- alloc {gib} GiB: process wall {time.perf_counter() - t:.4f} s rc {r.returncode}\n{r.stdout}{r.stderr[-300:]}", flush=True)
