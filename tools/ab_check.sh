#!/bin/bash
# Same-box A/B of the default bench (config 4): the product library vs a reference build
# (dbslmm_amd/libdbslmm_hip_base.so, built from an earlier commit), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-ab}; mkdir -p $O
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --predict none --no-e2e"
for i in 1 2; do
  for L in base ""; do
    N=${L:-new}
    DBSLMM_LIB_PATH=$PWD/dbslmm_amd/libdbslmm_hip${L:+_$L}.so timeout -k 10 300 $B > $O/bench_${N}_$i.log 2>&1 || { echo "FAILED $N $i"; exit 1; }
    tail -1 $O/bench_${N}_$i.log > $O/bench_${N}_$i.json
  done
done
echo done
