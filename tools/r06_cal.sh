#!/bin/bash
# round 6: PCG shard-model calibration -- kernel traces of configs 3-5, per-block iterations, the
# one-GPU rehearsal of N = 2, 4, 8 on config 4 and 5
set -o pipefail
out=gpurun_out/r06/${1:-cal}
mkdir -p $out
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-isolated"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pcg.py > $out/pcg_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/r06_cal.py $out > $out/cal.log 2>&1 || exit 2
for c in 3 4 5; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o c$c -- python3 /root/repo/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/prof_c$c.json 2> /root/repo/$out/prof_c$c.err) || exit 3
done
timeout -k 10 400 python -u bench.py --config 4 $B --predict 2,4,8 > $out/c4_pred.json 2> $out/c4_pred.err || exit 4
timeout -k 10 400 python -u bench.py --config 5 $B --predict 2,4,8 > $out/c5_pred.json 2> $out/c5_pred.err || exit 5
