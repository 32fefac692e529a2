#!/bin/bash
# short benches of the given configs (default: 2 3 4), one line of kernel times each
mkdir -p gpurun_out
for N in ${@:-2 3 4}; do
  timeout -k 10 400 python bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$N.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "config $N rc=$rc"; tail -5 gpurun_out/cfg_$N.log; exit $rc; }
  python - "$N" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/cfg_{sys.argv[1]}.log").read().strip().splitlines()[-1])
ks = {k["kernel"]: round(k["ms"], 3) for k in d["kernels"]}
g = [k for k in d["kernels"] if k["kernel"] == "dbslmm_gram_i8"][0]
print(f"config {sys.argv[1]}: {d['value']/1e6:.2f} M SNPs/s, {d['ms_per_step']:.2f} ms/step", ks,
      f"gram alg {g['achieved']:.0f} TOPS exec {g['executed_tops']:.0f} TOPS")
PY
done
