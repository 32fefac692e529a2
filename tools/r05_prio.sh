#!/bin/bash
# Wave-priority A/B of the chain kernels: the 9.6k block alone and config 4, alternating builds.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05prio}; mkdir -p $O
for r in 1 2; do
  for v in A B C; do
    DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 120 python tools/micro/tchol_alone.py 9600 > $O/alone_${v}_$r.log 2>&1 || { echo "FAILED alone $v"; exit 1; }
    echo "alone $v $r: $(tail -1 $O/alone_${v}_$r.log)"
  done
done
bash tools/ab_libs.sh 4 2 ablibs/lib_A.so ablibs/lib_B.so ablibs/lib_C.so

STAMPS=1 timeout -k 10 120 python tools/region_probe.py 9600 1000 > $O/region_stamps.log 2>&1 && tail -2 $O/region_stamps.log
echo done
