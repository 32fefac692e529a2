#!/bin/bash
# One rocprofv3 --pmc pass per argument group over a short config-N bench:
#   tools/pmc_kern.sh N "CTR_A CTR_B" "CTR_C" ...   -> gpurun_out/pmc_c<N>/<i>_counter_collection.csv
N=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_c$N
i=0
for grp in "$@"; do
  timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_c$N -o p$i -- python3 bench.py --config $N --steps 1 --warmup 0 --no-cpu-baseline --predict none > gpurun_out/pmc_c$N/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/pmc_c$N/p$i.log; exit $rc; }
  i=$((i+1))
done
