#!/bin/bash
# torchrun rehearsal of the 3-GPU strong-scaling bench on ONE GPU (every rank on device 0, gloo
# gather): the ranks' grouped split units (both large blocks split over the three ranks), the
# per-step gather and rank 0's big-block beta check against the oracle's direct solve
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05dist3}; mkdir -p $O
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 3 --dist-backend gloo --rank-device 0 --steps 3 --warmup 1 \
  --no-cpu-baseline --predict none --no-e2e > $O/bench_3rank.log 2>&1 || { echo FAILED; tail -20 $O/bench_3rank.log; exit 1; }
grep '"metric"' $O/bench_3rank.log | tail -1 > $O/bench_3rank.json
python3 -c "
import json; d=json.loads(open('$O/bench_3rank.json').read())
print(round(d['value']/1e6,2), 'M SNPs/s', round(d['ms_per_step'],2), 'ms', d['config'].get('parallelism'))
print(json.dumps(d.get('max_dbeta_vs_cpu_ref'))[:600])"
echo done
