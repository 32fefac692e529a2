#!/bin/bash
set -u
mkdir -p gpurun_out/hwq
for r in 1 2 3; do
  for Q in 4 8; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --predict none --no-e2e --no-isolated --no-check > gpurun_out/hwq/q${Q}_$r.log 2>&1 || { echo "FAILED $Q $r"; exit 1; }
    python - $Q gpurun_out/hwq/q${Q}_$r.log << 'PY'
import json, sys
p = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {x["kernel"]: x for x in p["kernels"]}
print(f"HWQ={sys.argv[1]} {p['ms_per_step']:7.2f} ms  tchol {k['dbslmm_tchol']['ms']:6.2f}  trsv {k['dbslmm_trsv']['ms']:6.2f}  unpack {k['dbslmm_unpack_stats']['ms']:5.2f} gram {k['dbslmm_gram_i8']['ms']:5.2f}")
PY
  done
done
