#!/bin/bash
# round 6: dbslmm_pcg_block quadrant loads through a range-checked buffer descriptor (counted
# waits, two quadrants in flight per wave) -- parity, then configs 4 / 5 / 3, the largest blocks
# alone and config 2 (factorisation vs PCG forced)
set -o pipefail
out=gpurun_out/r06/${1:-buf}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py > $out/tests.log 2>&1 || exit 1
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c$c.json 2> $out/c$c.err || exit 2
done
timeout -k 10 300 python -u tools/r06_big.py $out/big_c4.json 4 > $out/big_c4.log 2>&1 || exit 3
B2="--config 2 --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 200 python -u bench.py $B2 > $out/c2.json 2> $out/c2.err || exit 4
timeout -k 10 200 python -u bench.py $B2 --opt solver=2 > $out/c2_pcg.json 2> $out/c2_pcg.err || exit 5
