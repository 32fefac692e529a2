#!/bin/bash
# round 6: dbslmm_pcg_block with 1 / 2 workgroups per CU (DBSLMM_PCG_FUSED_WG), configs 5 / 3 (one copy) and 4
set -o pipefail
out=gpurun_out/r06/${1:-wg2}
mkdir -p $out
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
for w in 1 2; do for c in 5 3 4; do
  DBSLMM_PCG_FUSED_WG=$w timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_w$w.json 2> $out/c${c}_w$w.err || exit 2
done; done
