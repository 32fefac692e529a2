#!/bin/bash
# A/B of the determinism probe (tools/race_probe.py): the round-3 library vs this tree's
# usage: tools/race_ab.sh CONFIG FRESH
cfg=${1:-3}; fr=${2:-10}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/race_probe.py --config $cfg --fresh $fr --reruns 20 \
    --lib dbslmm_amd/libdbslmm_hip_r03.so --abi 8 > gpurun_out/race${cfg}_old.log 2>&1 &&
timeout -k 10 300 python -u tools/race_probe.py --config $cfg --fresh $fr --reruns 20 --memset-gib 0 \
    > gpurun_out/race${cfg}_new.log 2>&1
rc=$?
cat gpurun_out/race${cfg}_old.log gpurun_out/race${cfg}_new.log
exit $rc
