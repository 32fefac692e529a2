#!/bin/bash
# GPU tests then a config-3 bench; stops at the first crash / timeout (rc not in {0,1}).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c3.log 2>&1
rc=$?; echo "c3 rc=$rc"; tail -c 2500 gpurun_out/c3.log
exit $rc
