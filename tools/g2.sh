#!/bin/bash
# GPU tests, then a rocprof kernel trace of config N (default 3); stops at the first crash.
N=${1:-3}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
bash tools/prof_c3.sh $N
