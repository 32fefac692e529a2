#!/bin/bash
# round 6: config 2 (50k x 2k, factorisation route) -- the tiled-path threshold (tiled_min) swept
set -o pipefail
out=gpurun_out/r06/${1:-c2}
mkdir -p $out
export TMPDIR=/tmp
B="--config 2 --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --predict none"
for t in 0 320 400 512 1024; do
  timeout -k 10 200 python -u bench.py $B --opt tiled_min=$t > $out/c2_t$t.json 2> $out/c2_t$t.err || exit 2
done
