#!/bin/bash
# round 6: early result download (the whole-block kernel's blocks' betas come down beside the
# chip-wide iterations; default library) vs the download after the run (ablibs/lib_noearly.so) --
# parity (PCG, GPU, multi-device, full-scale suites), then configs 4 / 5 / 3 alternating, twice
set -o pipefail
out=gpurun_out/r06/${1:-early}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 900 $T tests/test_pcg.py tests/test_gpu.py tests/test_multi.py tests/test_fullscale.py > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_$r.json 2> $out/c${c}_$r.err || exit 2
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_noearly.so timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_late_$r.json 2> $out/c${c}_late_$r.err || exit 3
done
done
