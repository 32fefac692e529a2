# Gram variant A/B (tools/micro/gram_probe.py) on uniform and config-4 block layouts, one PMC pass
set -u
export TMPDIR=/tmp
O=gpurun_out/g3; mkdir -p $O
for V in 2 1; do
  for M in "2048 64" "600 400" "0"; do
    DBSLMM_GRAM_VARIANT=$V timeout -k 10 200 python -u tools/micro/gram_probe.py $M > "$O/probe_v${V}_${M// /_}.log" 2>&1 || exit $?
  done
done
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o p0 -- python3 tools/micro/gram_probe.py 2048 64 > $O/pmc0.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o p1 -- python3 tools/micro/gram_probe.py 0 > $O/pmc1.log 2>&1
