#!/bin/bash
# Separate rocprofv3 counter passes (FETCH_SIZE, WRITE_SIZE) over a short bench run, then the
# kernel-trace/stats pass; outputs under gpurun_out/pmc/.  No sys/runtime trace with --pmc.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
ARGS="--steps 5 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o fetch -- python3 bench.py $ARGS > gpurun_out/pmc/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o write -- python3 bench.py $ARGS > gpurun_out/pmc/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc -o trace -- python3 bench.py $ARGS > gpurun_out/pmc/trace.log 2>&1 || exit $?
ls -R gpurun_out/pmc | head -30
