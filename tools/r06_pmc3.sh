#!/bin/bash
# round 6: wave-state and instruction counters of dbslmm_pcg_block on one small-block device of the
# config-3 N = 8 plan (device 3: 211 blocks of <= 1245 SNPs, one sequence per CU), one pass per group
set -o pipefail
out=gpurun_out/r06/${1:-pmc3}
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA"; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "pcg_block" -f csv -d /root/repo/$out -o p$i -- python3 /root/repo/tools/r06_dev.py /root/repo/$out/dev$i.json 3 8 3 > /root/repo/$out/p$i.log 2>&1) || exit 1
  i=$((i+1))
done
