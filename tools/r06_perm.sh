#!/bin/bash
# round 6: permlane16/32 swaps for the xor 16 / 32 exchanges (default library) vs ds_bpermute there (ablibs/lib_noperm.so); permlane semantics probe first
# -- parity, configs 4 / 5 / 3 alternating, and one small-block device of the config-3 N = 8 plan
set -o pipefail
out=gpurun_out/r06/${1:-perm}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 60 ./ablibs/probe_permlane > $out/probe.txt 2>&1 || exit 6
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py > $out/tests.log 2>&1 || exit 1
for c in 4 5 3; do
  timeout -k 10 200 python -u bench.py --config $c $B > $out/c$c.json 2> $out/c$c.err || exit 2
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_noperm.so timeout -k 10 200 python -u bench.py --config $c $B > $out/c${c}_noperm.json 2> $out/c${c}_noperm.err || exit 3
done
timeout -k 10 200 python -u tools/r06_dev.py $out/dev3.json 3 8 3 > $out/dev3.log 2>&1 || exit 4
DBSLMM_LIB_PATH=$PWD/ablibs/lib_noperm.so timeout -k 10 200 python -u tools/r06_dev.py $out/dev3_noperm.json 3 8 3 > $out/dev3_noperm.log 2>&1 || exit 5
