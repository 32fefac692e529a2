#!/bin/bash
# kernel traces of the 9.6k block alone: far trailing uncapped (A) / leaving 32 CUs free (B)
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05captrace}; mkdir -p $O
for v in A B; do
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o run -- python tools/micro/tchol_alone.py 9600 > $O/trace_$v.log 2>&1 || { echo "FAILED trace $v"; exit 1; }
  tail -1 $O/trace_$v.log
done
echo done
