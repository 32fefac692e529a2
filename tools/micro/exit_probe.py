"""Where does the dbslmm CLI's wall time go outside its own phases?  (0.19 s of
the end-to-end wall time lay outside the CLI's phase total.)  Writes the config-4 panel as PLINK
files once, then runs the CLI several times and splits each run into
    spawn   parent's spawn -> the CLI's main()   (exec + dynamic loading; `pre_main` from inside)
    inside  main() -> EXIT_AT                      (the CLI's own phases)
    exit    EXIT_AT -> the parent sees the exit    (_Exit, kernel-side teardown, pipes)
with output to the panel directory and to /dev/shm, stdout to a pipe or to /dev/null.
    python tools/micro/exit_probe.py [snps] [n_ref]"""
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

sys.path[:0] = ["."]
from dbslmm_amd import synth  # noqa: E402

snps = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
n_ref = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
d = tempfile.mkdtemp(prefix="exitp_", dir=os.environ.get("TMPDIR", "/tmp"))
panel = synth.simulate(snps, n_ref, seed=1, engine="gpu")
f = synth.write_plink(panel, d)
del panel
cli = os.path.join("dbslmm_amd", "bin", "dbslmm")
base = [cli, "-s", f["s"], "-l", f["l"], "-r", f["ref"], "-b", f["b"], "-n", str(f["n"]), "-nsnp",
        str(f["nsnp"]), "-h", "0.5", "-mafMax", "0.2", "-h2f", "0.8,1,1.2", "--timing"]
shm = tempfile.mkdtemp(prefix="exitp_", dir="/dev/shm") if os.path.isdir("/dev/shm") else d
variants = [("pipe", d, subprocess.PIPE), ("pipe", d, subprocess.PIPE), ("shm", shm, subprocess.PIPE),
            ("devnull", d, subprocess.DEVNULL), ("pipe", d, subprocess.PIPE)]
if os.environ.get("EXIT_PROBE_H2F"):   # 3 h2f copies (22 GB of block matrices) vs 1 (7.5 GB), alternating
    variants = [("h2f", d, subprocess.PIPE), ("single", d, subprocess.PIPE)] * 3
if os.environ.get("EXIT_PROBE_QUEUES"):   # hardware queues of the CLI process: default (4) vs 2 / 3
    variants = [("pipe", d, subprocess.PIPE), ("q2", d, subprocess.PIPE), ("q3", d, subprocess.PIPE)] * 3
settle = float(os.environ.get("EXIT_PROBE_SETTLE", "0"))   # seconds between runs
for label, outdir, sink in variants:
    if settle:
        time.sleep(settle)
    cmd = base + ["-eff", os.path.join(outdir, "eff")]
    if label == "single":
        cmd = [x for x in cmd if x not in ("-h2f", "0.8,1,1.2")]
    t0 = time.time()
    env = None
    if label in ("q2", "q3"):
        env = dict(os.environ, GPU_MAX_HW_QUEUES=label[1])
    p = subprocess.Popen(cmd, stdout=sink, stderr=subprocess.PIPE, text=True, env=env)
    _, err = p.communicate(timeout=600)
    t1 = time.time()
    ph = {}
    exit_at = None
    for line in err.splitlines():
        if line.startswith("TIMING "):
            ph = json.loads(line[7:])
        if line.startswith("EXIT_AT "):
            exit_at = float(line.split()[1])
    total = ph.get("total", 0.0)
    start_main = exit_at - total if exit_at else None
    print(f"{label:8s} rc {p.returncode} wall {t1 - t0:.3f}  spawn {start_main - t0 if exit_at else -1:.3f} "
          f"(pre_main {ph.get('pre_main', -1):.3f})  inside {total:.3f}  exit {t1 - exit_at if exit_at else -1:.3f}  "
          f"ctx {ph.get('ctx', -1):.3f} upload {ph.get('bed_upload', -1):.3f} gpu_wait {ph.get('gpu_wait', -1):.3f} "
          f"solve {ph.get('solve', -1):.3f} write {ph.get('write', -1):.3f}", flush=True)
for x in (d, shm):
    shutil.rmtree(x, ignore_errors=True)
