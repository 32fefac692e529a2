#!/bin/bash
# CG in chol_cheb too: the GPU suite, then config-4 A/B (h2f_iter 1 vs the default CG) with the
# chol_large phase span.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-cg2b}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t={k['kernel'][7:]: round(k['ms'],2) for k in d['kernels']}; print('$2', round(d['ms_per_step'],2), 'ms', t)" >> $O/ab.txt; }
run 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for i in 1 2; do
  for it in 1 0; do
    run 300 python bench.py --no-cpu-baseline --predict none --no-e2e --no-check --opt h2f_iter=$it > $O/b.log 2>&1
    summ $O/b.log "h2f_iter=$it run $i"
  done
done
cat $O/ab.txt
