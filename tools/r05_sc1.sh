#!/bin/bash
# sc1 (write-through) C stores in the bulk trailing (B) and also the Gram epilogue (C) vs plain (A):
# does the end-of-kernel L2 write-back of the chain's small kernels stretch them beside the bulk?
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05sc1}; mkdir -p $O
for v in A B C; do
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 120 python tools/micro/tchol_alone.py 9600 > $O/alone_$v.log 2>&1 || { echo "FAILED alone $v"; exit 1; }
  echo "alone $v: $(tail -1 $O/alone_$v.log)"
done
for v in A B; do
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python tools/micro/tchol_alone.py 9600 > $O/trace_$v.log 2>&1 || { echo "FAILED trace $v"; exit 1; }
done
bash tools/ab_libs.sh 4 2 ablibs/lib_A.so ablibs/lib_B.so ablibs/lib_C.so
echo done
