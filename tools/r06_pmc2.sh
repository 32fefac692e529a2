#!/bin/bash
# round 6: PMC passes over the config-4 kernels -- MFMA busy / wave states (pass 0), HBM traffic
# (passes 1-2) -- one rocprofv3 run per pass, one timed step
set -o pipefail
out=gpurun_out/r06/${1:-pmc2}
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "pcg|gram|unpack" -f csv -d /root/repo/$out -o p$i -- python3 /root/repo/bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/p$i.log 2>&1) || exit 1
  i=$((i+1))
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d /root/repo/$out -o kt -- python3 /root/repo/bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/kt.log 2>&1) || exit 2
