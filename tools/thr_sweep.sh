#!/bin/bash
# config-N bench at several tiled thresholds (DBSLMM_TILED_MIN); stops at the first crash.
N=${1:-3}
mkdir -p gpurun_out
for t in 256 384 512 1024; do
  DBSLMM_TILED_MIN=$t timeout -k 10 300 python bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/thr_$t.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "thr $t rc=$rc"; tail -5 gpurun_out/thr_$t.log; exit $rc; }
  python - "$t" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/thr_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[1], "ms/step %.2f" % d["ms_per_step"], {k["kernel"]: round(k["ms"], 2) for k in d["kernels"]})
PY
done
