#!/bin/bash
# config-N Gram time at several DBSLMM_GRAM_HUGE_MIN thresholds
N=${1:-5}
mkdir -p gpurun_out
for t in ${THR:-512 1024 1536 2048 4096}; do
  DBSLMM_GRAM_HUGE_MIN=$t timeout -k 10 300 python bench.py --config $N --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/gs_$t.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "thr $t rc=$rc"; tail -5 gpurun_out/gs_$t.log; exit $rc; }
  python - "$t" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/gs_{sys.argv[1]}.log").read().strip().splitlines()[-1])
g = [k for k in d["kernels"] if k["kernel"] == "dbslmm_gram_i8"][0]
print(sys.argv[1], "gram ms %.3f alg %.0f exec %.0f TOPS" % (g["ms"], g["achieved"], g["executed_tops"]))
PY
done
