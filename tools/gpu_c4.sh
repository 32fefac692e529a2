#!/bin/bash
# Fast GPU iteration: a test subset (TESTS, default the tiled / Gram parity tests), then the
# config-4 bench line (no CPU baseline, no end-to-end leg).  Stops at the first fault / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TESTS=${TESTS:-tests/test_tiled.py tests/test_h2f_cheb.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_sub.log
[ $rc -eq 0 ] || { echo "tests rc=$rc"; exit $rc; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e ${BENCH_ARGS:-} > gpurun_out/bench_c4.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_c4.log; echo "bench rc=$rc"; exit $rc; }
python tools/bench_summary.py gpurun_out/bench_c4.log
