#!/bin/bash
# Gram head / capped tail (G<free CUs>) vs the round's tree (BASE): the 9.6k block alone, the N = 8
# plan's device 0 alone, config 4 / 5 steps, alternating fresh processes
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05gtail}; mkdir -p $O
for r in 1 2; do
  for v in BASE G0 G32 G64; do
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 200 python tools/micro/tchol_alone.py 9600 > $O/alone_${v}_$r.log 2>&1 || { echo FAILED; tail -3 $O/alone_${v}_$r.log; exit 1; }
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 300 python tools/micro/units_alone.py 8 0 5 > $O/dev0_${v}_$r.log 2>&1 || { echo FAILED; tail -3 $O/dev0_${v}_$r.log; exit 1; }
    echo "$v alone $(tail -1 $O/alone_${v}_$r.log) | dev0 $(grep 'ms per run' $O/dev0_${v}_$r.log)"
  done
done
bash tools/ab_libs.sh 4 2 ablibs/lib_BASE.so ablibs/lib_G32.so ablibs/lib_G64.so || exit 1
bash tools/ab_libs.sh 5 1 ablibs/lib_BASE.so ablibs/lib_G32.so ablibs/lib_G64.so || exit 1
echo done
