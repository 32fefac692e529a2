#!/bin/bash
# Host-ingest check: the .bed upload / CLI parity tests, then the default bench (config 4) with
# its end-to-end CLI leg.  Outputs under gpurun_out/${GOUT:-u1}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-u1}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest tests/test_cli.py tests/test_gpu.py tests/test_multi.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
run 400 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --predict none > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
echo done
