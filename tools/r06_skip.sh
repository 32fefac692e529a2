#!/bin/bash
# round 6: skipped loads of zero / upper sub-blocks; dbslmm_pcg_block depth 3 (default library) vs 2 (A/B library)
set -o pipefail
out=gpurun_out/r06/${1:-skip}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py > $out/tests.log 2>&1 || exit 1
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c$c.json 2> $out/c$c.err || exit 2
  DBSLMM_LIB_PATH=$PWD/gpurun_ab_depth2.so timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_d2.json 2> $out/c${c}_d2.err || exit 3
done
