#!/bin/bash
# PMC passes over a short config-4 bench (h2f Chebyshev path): per-kernel counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmct; mkdir -p $O
i=0
for grp in "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O -o p$i -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/p$i.log; exit $rc; }
  i=$((i+1))
done
