#!/bin/bash
# round 6: kernel traces of single devices of the config-4 N = 8 shard plan (a big-block device and a small-block one)
set -o pipefail
out=gpurun_out/r06/${1:-dev8}
mkdir -p $out
export TMPDIR=/tmp
for d in 0 4; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o d$d -- python3 /root/repo/tools/r06_dev.py /root/repo/$out/dev_$d.json 4 8 $d > /root/repo/$out/dev_$d.log 2>&1) || exit 1
done
