"""One line per bench.py JSON log: ms/step and the per-kernel times.
    python tools/bench_summary.py gpurun_out/bench_c4.log [...]"""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"{path}: no JSON line ({e})")
        continue
    ks = " ".join("%s=%.2f" % (k["kernel"].replace("dbslmm_", ""), k["ms"]) for k in d["kernels"])
    e2e = d.get("end_to_end") or {}
    print(f"{path}: {d['ms_per_step']:.2f} ms/step {d['value'] / 1e6:.2f} M SNPs/s | {ks}"
          + (f" | e2e {e2e['seconds']:.2f} s" if "seconds" in e2e else ""))
