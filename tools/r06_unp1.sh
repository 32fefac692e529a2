#!/bin/bash
# round 6: unpack with one aligned 16-B load per chunk (neighbour lane's load by DPP; default
# library) vs two loads per chunk (ablibs/lib_upairs.so) -- parity (unpack / stats / MAF tests and
# the PCG route), then configs 4 / 5 / 3 alternating, twice
set -o pipefail
out=gpurun_out/r06/${1:-unp1}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 900 $T tests/test_gpu.py tests/test_pcg.py tests/test_cli.py > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_$r.json 2> $out/c${c}_$r.err || exit 2
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_upairs.so timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_pairs_$r.json 2> $out/c${c}_pairs_$r.err || exit 3
done
done
