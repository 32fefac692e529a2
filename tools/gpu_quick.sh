#!/bin/bash
# Quick GPU iteration: GPU parity tests, then bench lines of configs 4, 5, 3 (no CPU baseline).
# Every GPU step has its own time limit; the script stops at the first fault / abort / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name" | tee -a gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a gpurun_out/steps.log
    tail -3 "gpurun_out/$name.log" | cut -c1-300
    case $rc in
        0|1|5) return 0 ;;
        *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
    esac
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench_c4 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --predict none
step bench_c5 600 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline --predict none
step bench_c3 600 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --predict none
echo done
