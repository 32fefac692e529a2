#!/bin/bash
# bench config 4 (BENCH_ARGS) with each library variant given as arguments (dbslmm_amd/<name>.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  DBSLMM_LIB_PATH=$PWD/dbslmm_amd/$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/var_$v.log; exit 1; }
  python tools/bench_summary.py gpurun_out/var_$v.log
done
