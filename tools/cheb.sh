#!/bin/bash
# Chebyshev h2f path: the GPU tests of every path it touches, then the config-4 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_h2f_cheb.py tests/test_tiled.py tests/test_variance.py tests/test_cli.py tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cheb_tests.log 2>&1; rc=$?
tail -5 gpurun_out/cheb_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab.sh 4 DBSLMM_H2F_CHEB=0 DBSLMM_H2F_CHEB=1 || exit 1
