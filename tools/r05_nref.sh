#!/bin/bash
# Does the 9.6k block's factorisation time depend on the data?  tchol_alone at n_ref 1000 / 10000
# and region_probe (random unlinked genotypes) at n_ref 10000, each with a kernel trace.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05nref}; mkdir -p $O
for n in 1000 10000; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/alone_$n -o run -- python tools/micro/tchol_alone.py 9600 $n > $O/alone_$n.log 2>&1 || { echo FAILED; exit 1; }
  tail -1 $O/alone_$n.log
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/probe_10000 -o run -- python tools/region_probe.py 9600 10000 > $O/probe_10000.log 2>&1 || { echo FAILED; exit 1; }
tail -1 $O/probe_10000.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/probe_1000 -o run -- python tools/region_probe.py 9600 1000 > $O/probe_1000.log 2>&1 || { echo FAILED; exit 1; }
tail -1 $O/probe_1000.log
echo done
