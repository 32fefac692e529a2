#!/bin/bash
# round 6: first measurement of the PCG route (tests, config 3/4/5 bench lines, kernel stats)
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_pcg.py > gpurun_out/r06/pcg_tests.log 2>&1 || exit 1
for c in 4 3 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none --no-isolated > gpurun_out/r06/bench_c$c.json 2> gpurun_out/r06/bench_c$c.err || exit 2
done
timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated --opt solver=1 > gpurun_out/r06/bench_c4_factor.json 2> gpurun_out/r06/bench_c4_factor.err || exit 3
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/r06/prof -o c4 -- python3 /root/repo/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/gpurun_out/r06/prof_c4.json 2> /root/repo/gpurun_out/r06/prof_c4.err || exit 4
