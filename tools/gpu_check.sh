#!/bin/bash
# One gpurun session: smoke, GPU parity tests, a short bench, a rocprofv3 kernel-trace profile.
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
    tail -5 "gpurun_out/$name.log"
    case $rc in
        0|1|5) return 0 ;;          # success / test failures: keep going
        *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
    esac
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 3
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none
echo done
