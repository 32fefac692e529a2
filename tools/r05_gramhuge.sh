#!/bin/bash
# gram_huge_min sweep (mid-size blocks on the 256-tile LDS-DMA Gram instead of the 128-tile one):
# config 4 step and the Gram alone (isolated run); config 5 too.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05gh}; mkdir -p $O
for r in 1 2; do
for g in 384 256 192 128; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --predict none --no-e2e --opt gram_huge_min=$g > $O/c4_${g}_${r}.log 2>&1 || { echo FAILED; exit 1; }
  python - $g $O/c4_${g}_${r}.log << 'PY'
import json, sys
p = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {x["kernel"]: x for x in p["kernels"]}
g = k["dbslmm_gram_i8"]
print(f"gram_huge_min {sys.argv[1]:4s} {p['ms_per_step']:7.2f} ms  gram span {g['ms']:5.2f} alone {g['alone_ms']:5.2f} (frac {g['alone_frac']:.3f})  unpack alone {k['dbslmm_unpack_stats']['alone_ms']:5.2f}")
PY
done
done
echo done
