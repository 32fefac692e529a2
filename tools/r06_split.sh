#!/bin/bash
# round 6: the solved-whole blocks' Gram on the second stream + x / p in LDS: parity, configs 4 / 5 / 3, kernel trace
set -o pipefail
out=gpurun_out/r06/${1:-split}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py tests/test_multi.py > $out/tests.log 2>&1 || exit 1
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c$c.json 2> $out/c$c.err || exit 2
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o c4 -- python3 /root/repo/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/prof_c4.json 2> /root/repo/$out/prof_c4.err) || exit 4
