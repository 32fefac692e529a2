#!/bin/bash
# Kernel-trace statistics of the default workload (config 4) for profiles/rNN:
#   tools/prof_round.sh OUT   -> OUT/kt_kernel_stats.csv, OUT/kt_kernel_trace.csv, OUT/kt_bench.json
set -u
O=${1:-gpurun_out/prof_round}
export TMPDIR=/tmp
mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-e2e > $O/kt_bench.json 2> $O/kt.log
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/kt.log; exit $rc; }
