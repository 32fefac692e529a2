#!/bin/bash
# rocprofv3 kernel trace of a short config-4 bench (BENCH_ARGS extra bench.py flags) -> gpurun_out/c4t
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/c4t
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4t -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --predict none --no-e2e ${BENCH_ARGS:-} > gpurun_out/c4t.log 2>&1
