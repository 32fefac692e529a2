#!/bin/bash
# step modes: four fresh config-4 bench processes, each under a kernel + HIP runtime trace (host
# call times of the graph launches beside the kernels' start times)
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05modes}; mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --predict none --no-e2e --no-isolated > $O/p$i.log 2>&1 || { echo "FAILED $i"; tail -3 $O/p$i.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/p$i.log').read().strip().splitlines()[-1]);print('p$i', round(d['ms_per_step'],2))"
done
echo done
