#!/bin/bash
# Gram phase alone (tools/micro/gram_probe.py) on uniform and config-4 block layouts, the MFMA
# rates (tools/micro/mfma_rate, incl. FP4 on changing operands), and the Gram parity tests.
#   GOUT=name bash tools/gram_probe.sh   -> gpurun_out/name/
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-gram}; mkdir -p $O
timeout -k 10 120 tools/micro/mfma_rate > $O/mfma_rate.txt 2>&1 || exit $?
for M in "4096 16" "2048 64" "600 400" "0"; do
  timeout -k 10 200 python -u tools/micro/gram_probe.py $M > "$O/probe_${M// /_}.log" 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_tiled.py tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
