#!/bin/bash
# bulk trailing stream (stream3) at high (P0, default) vs normal (P1) priority: the 9.6k block
# alone, the N = 8 plan's device 0 (a 9.7k split copy + bulk) alone, config 4 and 5 steps
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05bprio}; mkdir -p $O
for r in 1 2; do
  for v in P0 P1; do
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 200 python tools/micro/tchol_alone.py 9600 > $O/alone_${v}_$r.log 2>&1 || { echo FAILED; exit 1; }
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 300 python tools/micro/units_alone.py 8 0 5 > $O/dev0_${v}_$r.log 2>&1 || { echo FAILED; exit 1; }
    echo "$v alone $(tail -1 $O/alone_${v}_$r.log) | dev0 $(grep 'ms per run' $O/dev0_${v}_$r.log)"
  done
done
bash tools/ab_libs.sh 4 2 ablibs/lib_P0.so ablibs/lib_P1.so || exit 1
bash tools/ab_libs.sh 5 2 ablibs/lib_P0.so ablibs/lib_P1.so || exit 1
echo done
