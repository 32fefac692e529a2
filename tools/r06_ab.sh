#!/bin/bash
# round 6: PCG product variants (default library vs a DBSLMM_LIB_PATH variant), config 4/5/3 lines
set -o pipefail
out=gpurun_out/r06/${1:-ab}
mkdir -p $out
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none --no-isolated"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pcg.py > $out/pcg_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_a.json 2> $out/c4_a.err || exit 2
if [ -n "$2" ]; then
  DBSLMM_LIB_PATH=$2 timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_b.json 2> $out/c4_b.err || exit 3
  timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_a2.json 2> $out/c4_a2.err || exit 4
  DBSLMM_LIB_PATH=$2 timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_b2.json 2> $out/c4_b2.err || exit 5
fi
timeout -k 10 200 python -u bench.py --config 5 $B > $out/c5.json 2> $out/c5.err || exit 6
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o c4 -- python3 /root/repo/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/prof_c4.json 2> /root/repo/$out/prof_c4.err || exit 7
