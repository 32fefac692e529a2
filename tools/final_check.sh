#!/bin/bash
# Final tree check: GPU suite, smoke, a 2-device rehearsal of bench --gpus 2 on one GPU, and the
# default bench line.  Outputs under gpurun_out/${GOUT:-fin}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-fin}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 300 python bench.py --gpus 2 --devices 0,0 --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-e2e > $O/bench_2dev.log 2>&1
tail -1 $O/bench_2dev.log > $O/bench_2dev.json
run 300 python bench.py --no-cpu-baseline --predict none --no-e2e > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
for D in "" 0 1; do HIP_ENABLE_DEFERRED_LOADING=$D timeout -k 10 60 tools/micro/hipinit > $O/hipinit_${D:-default}.txt 2>&1 || break; done
echo done
