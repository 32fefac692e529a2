#!/bin/bash
# kernel traces of the N = 8 shard plan's bulk device (7) and of device 6, each alone; then device
# 7 with other lead substitution grids (sub_grid_lead), alternating
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05dev7}; mkdir -p $O
for d in 7 6; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$d -o run -- python tools/micro/units_alone.py 8 $d > $O/dev_$d.log 2>&1 || { echo "FAILED $d"; tail -5 $O/dev_$d.log; exit 1; }
  grep -E "device|ms per run" $O/dev_$d.log
done
for r in 1 2; do
  for g in 0 80 24 56; do
    timeout -k 10 300 python tools/micro/units_alone.py 8 7 5 sub_grid_lead=$g > $O/grid_${g}_$r.log 2>&1 || { echo "FAILED grid $g"; tail -5 $O/grid_${g}_$r.log; exit 1; }
    echo "sub_grid_lead $g: $(grep 'ms per run' $O/grid_${g}_$r.log)"
  done
done
echo done
