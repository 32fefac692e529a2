#!/bin/bash
# lookahead check: tiled parity tests, then A/B of the lookahead / graph switches on configs 4 and 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tiled.py tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/la_tests.log 2>&1 || { tail -30 gpurun_out/la_tests.log; exit 1; }
tail -2 gpurun_out/la_tests.log
bash tools/ab.sh 4 DBSLMM_LOOKAHEAD=0 "DBSLMM_LOOKAHEAD=1 DBSLMM_TGRAPH=0" DBSLMM_LOOKAHEAD=1 || exit 1
bash tools/ab.sh 3 DBSLMM_LOOKAHEAD=0 DBSLMM_LOOKAHEAD=1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/la -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/la_prof.log 2>&1
