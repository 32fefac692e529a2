#!/bin/bash
# Gram phase alone at the config-4 layout: kernel trace (per-kernel class: i8 / big / huge) and
# the uniform-block probes (m = 250 / 600 / 4096).
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05gram}; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python tools/micro/gram_probe.py 0 > $O/c4.log 2>&1 || { echo FAILED; exit 1; }
tail -2 $O/c4.log
for M in "250 1600" "600 400" "4096 16"; do
  timeout -k 10 200 python -u tools/micro/gram_probe.py $M > "$O/probe_${M// /_}.log" 2>&1 || { echo FAILED; exit 1; }
  head -1 "$O/probe_${M// /_}.log"
done
echo done
