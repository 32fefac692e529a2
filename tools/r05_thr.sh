#!/bin/bash
# rest sequence launched from a helper thread (T1) vs after the lead graph's launch (T0):
# configs 4 / 5, alternating fresh processes; a kernel trace of config 4 with T1
set -u
export TMPDIR=/tmp
bash tools/ab_libs.sh 4 3 ablibs/lib_T0.so ablibs/lib_T1.so || exit 1
bash tools/ab_libs.sh 5 2 ablibs/lib_T0.so ablibs/lib_T1.so || exit 1
BENCH_ARGS=--no-isolated DBSLMM_LIB_PATH=$PWD/ablibs/lib_T1.so bash tools/trace_c4.sh || exit 1
echo done
