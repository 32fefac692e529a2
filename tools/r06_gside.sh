#!/bin/bash
# round 6: the small / mid blocks' Gram kernels on a side stream beside the 256-tile Gram (default
# library) vs after it (ablibs/lib_gserial.so) -- parity, then configs 4 / 5 / 3 alternating, twice
set -o pipefail
out=gpurun_out/r06/${1:-gside}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_$r.json 2> $out/c${c}_$r.err || exit 2
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_gserial.so timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_serial_$r.json 2> $out/c${c}_serial_$r.err || exit 3
done
done
