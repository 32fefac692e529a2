#!/bin/bash
# round 6 (final tree): MFMA busy / wave states of the config-4 kernels, one counter pass
set -o pipefail
out=gpurun_out/r06/${1:-pmc4}
mkdir -p $out
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "pcg|gram|unpack" -f csv -d /root/repo/$out -o p0 -- python3 /root/repo/bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/p0.log 2>&1) || exit 1
