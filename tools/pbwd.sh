#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pbwd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/pbwd_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab.sh 4 DBSLMM_PBWD=0 DBSLMM_PBWD=1 || exit 1
bash tools/ab.sh 5 DBSLMM_PBWD=0 DBSLMM_PBWD=1 || exit 1
bash tools/ab.sh 3 DBSLMM_PBWD=0 DBSLMM_PBWD=1 || exit 1
