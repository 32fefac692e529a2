#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cheb3 -o run -- python3 bench.py --config 3 --h2f 0.8,1,1.2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cheb3.log 2>&1 || exit 1
tail -1 gpurun_out/cheb3.log | cut -c1-300
