#!/bin/bash
# GPU tests, then short benches of configs 3, 4, 5 (kernel times in the JSON line).
# Stops at the first crash / timeout.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for N in ${CFGS:-4 5 3}; do
  timeout -k 10 500 python bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$N.log 2>&1
  rc=$?; echo "config $N rc=$rc"
  [ $rc -eq 0 ] || { tail -5 gpurun_out/cfg_$N.log; exit $rc; }
  tail -1 gpurun_out/cfg_$N.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(' ms/step %.2f  value %.3g' % (d['ms_per_step'], d['value']))
for k in d['kernels']: print('   %-22s %9.3f ms  frac %.3f' % (k['kernel'], k['ms'], k['frac']))"
done
