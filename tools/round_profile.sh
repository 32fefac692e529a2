#!/bin/bash
# Round evidence: default bench line, rocprofv3 kernel stats + PMC traffic passes of the default
# workload, and bench lines + kernel stats of configs 3-5.  Outputs under gpurun_out/round/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python bench.py > $O/bench_c2.log 2>&1
tail -1 $O/bench_c2.log > $O/bench_c2.json
run 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/c2_prof.log 2>&1
run 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc -o fetch -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc -o write -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/pmc_write.log 2>&1
for N in 3 4 5; do
  CPU=""; [ $N -eq 3 ] || CPU="--no-cpu-baseline"
  run 900 python bench.py --config $N --steps 3 --warmup 1 $CPU > $O/bench_c$N.log 2>&1
  tail -1 $O/bench_c$N.log > $O/bench_c$N.json
  run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$N -o run -- python3 bench.py --config $N --steps 2 --warmup 1 --no-cpu-baseline > $O/c${N}_prof.log 2>&1
done
ls -R $O | head -40
