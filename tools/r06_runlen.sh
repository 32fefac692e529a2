#!/bin/bash
# round 6: product item run length -- parity, config 4 at run 8 / 4 / 2 (DBSLMM_PCG_RUN), the N = 8 rehearsal per device
set -o pipefail
out=gpurun_out/r06/${1:-runlen}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py > $out/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4.json 2> $out/c4.err || exit 2
for r in 4 2 1; do
  DBSLMM_PCG_RUN=$r timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_r$r.json 2> $out/c4_r$r.err || exit 3
done
timeout -k 10 300 python -u tools/r06_dev.py $out/dev_c4.json 4 2,4,8 > $out/dev_c4.log 2>&1 || exit 4
