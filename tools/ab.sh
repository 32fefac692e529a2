#!/bin/bash
# A/B of an environment switch on config N benches: tools/ab.sh N "VAR=a" "VAR=b" ...
N=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -3 gpurun_out/ab.log; exit $rc; }
  tail -1 gpurun_out/ab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('$v', 'ms/step %.2f' % d['ms_per_step'], ' '.join('%s=%.2f' % (k['kernel'][7:], k['ms']) for k in d['kernels']))"
done
