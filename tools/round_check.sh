#!/bin/bash
# Round evidence, part 1 (config 4 = the metric's workload): GPU parity suite, smoke, the default
# bench line with the CPU baseline, rocprofv3 kernel trace / stats, FETCH_SIZE and WRITE_SIZE
# passes and one MFMA-busy pass.  Outputs under gpurun_out/${GOUT:-r1}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r1}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
run 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
run 400 python bench.py > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-isolated --no-e2e"
run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- $B > $O/c4_prof.log 2>&1
run 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4 -o fetch -- $B > $O/pmc4_fetch.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4 -o write -- $B > $O/pmc4_write.log 2>&1
run 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc4 -o p0 -- $B > $O/pmc4_p0.log 2>&1
echo done
