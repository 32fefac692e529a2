"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE counter CSVs into per-kernel HBM bytes per launch.

FETCH_SIZE and WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM section): the read side is doubled here.
    python tools/pmc_traffic.py gpurun_out/pmc profiles/r01/pmc_traffic.json
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(src, dst):
    f = per_kernel(os.path.join(src, "fetch_counter_collection.csv"))
    w = per_kernel(os.path.join(src, "write_counter_collection.csv"))
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                     "`python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline`",
           "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch",
           "kernels": {}}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("dbslmm_"):
            continue
        fk, wk = f.get(k, 0.0), w.get(k, 0.0)
        out["kernels"][k] = dict(fetch_kb=fk, write_kb=wk, hbm_bytes=(2 * fk + wk) * 1024.0)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
