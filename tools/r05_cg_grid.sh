#!/bin/bash
# With h2f by CG: the lead substitution grid (sub_grid_lead; default 80 of 256 CUs at config 4)
# and the lead threshold (lead_min; default 1536), config 4, alternating, two runs each.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-cggrid}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
for i in 1 2; do
  for opt in "sub_grid_lead=80" "sub_grid_lead=64" "sub_grid_lead=96" "lead_min=2048" "lead_min=1200"; do
    run 300 python bench.py --no-cpu-baseline --predict none --no-e2e --no-check --opt $opt > $O/b.log 2>&1
    tail -1 $O/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=[round(k['ms'],2) for k in d['kernels'] if k['kernel'] in ('dbslmm_trsv','dbslmm_tchol')]; print('$opt run $i', round(d['ms_per_step'],2), 'ms, tchol/trsv span', t)" >> $O/ab.txt
  done
done
cat $O/ab.txt
