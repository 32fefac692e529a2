#!/bin/bash
# next-pivot pipelining in the 32-column diagonal factorisations (LA) vs the round's tree (BASE):
# bit-identity at configs 3 / 4, the 9.6k block alone, chol_large blocks, the N = 8 device 0,
# configs 4 / 5
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05la}; mkdir -p $O
timeout -k 10 600 python tools/bitcmp_libs.py 4 ablibs/lib_BASE.so ablibs/lib_LA.so > $O/bitcmp4.txt 2>&1; tail -1 $O/bitcmp4.txt
timeout -k 10 600 python tools/bitcmp_libs.py 3 ablibs/lib_BASE.so ablibs/lib_LA.so > $O/bitcmp3.txt 2>&1; tail -1 $O/bitcmp3.txt
for r in 1 2; do
  for v in BASE LA; do
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 200 python tools/micro/tchol_alone.py 9600 > $O/alone_${v}_$r.log 2>&1 || { echo FAILED; exit 1; }
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 200 python tools/micro/large_probe.py 300 376 > $O/large_${v}_$r.log 2>&1 || { echo FAILED; exit 1; }
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 300 python tools/micro/units_alone.py 8 0 5 > $O/dev0_${v}_$r.log 2>&1 || { echo FAILED; exit 1; }
    echo "$v alone $(tail -1 $O/alone_${v}_$r.log) | large $(grep -o "'dbslmm_chol_large': np.float64([0-9.]*)" $O/large_${v}_$r.log) | dev0 $(grep 'ms per run' $O/dev0_${v}_$r.log)"
  done
done
bash tools/ab_libs.sh 4 2 ablibs/lib_BASE.so ablibs/lib_LA.so || exit 1
bash tools/ab_libs.sh 5 1 ablibs/lib_BASE.so ablibs/lib_LA.so || exit 1
echo done
