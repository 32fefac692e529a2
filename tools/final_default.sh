#!/bin/bash
# Round-end check of the tree as the driver runs it: GPU suite, smoke, then the default bench line
# (cpu baseline, multi-GPU rehearsal and end-to-end legs included).  Outputs under gpurun_out/${GOUT:-fin}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-fin}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 600 python -u bench.py > $O/bench_default.log 2>&1
tail -1 $O/bench_default.log > $O/bench_default.json
echo done
