#!/bin/bash
# PMC evidence of the default workload (config 4): separate rocprofv3 passes (MI355X_MICROARCH.md:
# FETCH_SIZE and WRITE_SIZE in passes of their own) over a short bench.
#   tools/pmc_round.sh OUT   -> OUT/{fetch,write,p0,p1}_counter_collection.csv
set -u
O=${1:-gpurun_out/pmc_round}
export TMPDIR=/tmp
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --predict none --no-isolated --no-e2e"
pass() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --output-format csv -d $O -o $name -- $B > $O/$name.log 2>&1
  local rc=$?; echo "pass $name ($*) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass p0 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES
pass p1 TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
