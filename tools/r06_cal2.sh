#!/bin/bash
# round 6: shard-model calibration on the final PCG route -- per-device rehearsal of configs 3 / 4 / 5 at N = 1, 2, 4, 8
set -o pipefail
out=gpurun_out/r06/${1:-cal2}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pcg.py tests/test_multi.py > $out/tests.log 2>&1 || exit 1
for c in 4 5 3; do
  timeout -k 10 400 python -u tools/r06_dev.py $out/dev_c$c.json $c 1,2,4,8 > $out/dev_c$c.log 2>&1 || exit 2
done
