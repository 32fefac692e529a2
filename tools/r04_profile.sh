#!/bin/bash
# Round-4 evidence of one tree: config-4 bench line, kernel trace, per-dispatch wave-cycle PMC pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python bench.py ${BENCH_ARGS:-} > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
rm -rf $O/c4t
run 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4t -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --predict none --no-e2e --no-isolated > $O/c4t.log 2>&1
run 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d $O/pmcw -o w -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --predict none --no-e2e --no-isolated > $O/pmcw.log 2>&1
echo done
