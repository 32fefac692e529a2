#!/bin/bash
# Far-trailing grid cap A/B: CUs left free for the chain 0 / 8 / 16 / 32; the 9.6k block alone
# and config 4 (alternating).
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05farcap}; mkdir -p $O
for v in A B C D; do
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 120 python tools/micro/tchol_alone.py 9600 > $O/alone_$v.log 2>&1 || { echo "FAILED alone $v"; exit 1; }
  echo "alone $v: $(tail -1 $O/alone_$v.log)"
done
bash tools/ab_libs.sh 4 2 ablibs/lib_A.so ablibs/lib_B.so ablibs/lib_C.so ablibs/lib_D.so
echo done
