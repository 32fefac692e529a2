#!/bin/bash
# round 6: PMC passes over the PCG kernels (config 4, one timed step), one rocprofv3 run per pass
#   tools/r06_pmc.sh <outdir> "<counters pass 1>" "<counters pass 2>" ...
out=gpurun_out/r06/$1; shift
mkdir -p $out
export TMPDIR=/tmp
i=0
for grp in "$@"; do
  cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "pcg|gram|unpack" -f csv -d /root/repo/$out -o p$i -- python3 /root/repo/bench.py --config ${PMC_CONFIG:-4} --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/p$i.log 2>&1
  rc=$?; cd /root/repo; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/p$i.log; exit $rc; }
  i=$((i+1))
done
