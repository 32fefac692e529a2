#!/bin/bash
# bench.py under several dbslmm_options settings (one line each): VARIANTS="name|args;name|args"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
IFS=';' read -ra VS <<< "$VARIANTS"
for v in "${VS[@]}"; do
    name=${v%%|*}; a=${v#*|}
    echo "== $name: $a"
    timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline $a > gpurun_out/var/$name.log 2>&1
    rc=$?
    [ $rc -eq 0 ] || { echo "stopping: $name rc=$rc"; tail -5 gpurun_out/var/$name.log; exit $rc; }
    tail -1 gpurun_out/var/$name.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('  %.2f ms/step'%d['ms_per_step'], ' '.join('%s=%.2f'%(k['kernel'].replace('dbslmm_',''),k['ms']) for k in d['kernels']))"
done
