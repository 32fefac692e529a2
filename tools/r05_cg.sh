#!/bin/bash
# h2f by CG (h2f_iter = 2) vs Chebyshev: the h2f parity tests, config-4 A/B bench lines, and one
# CG line with the CPU leg (parity against the oracle on the sample and every block >= 2000 SNPs).
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-cg}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
summ() { tail -1 $1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); t=[round(k['ms'],2) for k in d['kernels'] if k['kernel']=='dbslmm_trsv']; print('$2', round(d['ms_per_step'],2), 'ms, trsv span', t, 'dbeta', d.get('max_dbeta_vs_cpu_ref'))" >> $O/ab.txt; }
run 400 python -u -m pytest tests/test_h2f_cheb.py -x -v --timeout 120 --timeout-method thread > $O/pytest_h2f.log 2>&1
for i in 1 2; do
  for it in 1 2; do
    run 300 python bench.py --no-cpu-baseline --predict none --no-e2e --opt h2f_iter=$it > $O/bench_it${it}_$i.log 2>&1
    summ $O/bench_it${it}_$i.log "h2f_iter=$it run $i"
  done
done
run 300 python bench.py --predict none --no-e2e --opt h2f_iter=2 > $O/bench_cg_cpu.log 2>&1
summ $O/bench_cg_cpu.log "h2f_iter=2 with the cpu leg"
cat $O/ab.txt
