#!/bin/bash
# Round evidence: default bench line (config 4 = the metric's 1M x 10k workload) with the CPU
# baseline, rocprofv3 kernel stats + PMC traffic passes of it, then bench lines + kernel stats of
# configs 2, 3, 5.  Outputs under gpurun_out/round/.
set -u

export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05prof}
mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }


run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-isolated > $O/c4_prof.log 2>&1
run 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc4 -o fetch -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-isolated > $O/pmc4_fetch.log 2>&1
run 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc4 -o write -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --predict none --no-isolated > $O/pmc4_write.log 2>&1
run 300 python bench.py --config 1 > $O/bench_c1.log 2>&1
tail -1 $O/bench_c1.log > $O/bench_c1.json
for N in 2 3 5; do
  CPU=""; [ $N -le 3 ] || CPU="--no-cpu-baseline --predict none"
  STEPS="--steps 5 --warmup 2"; [ $N -eq 2 ] && STEPS="--steps 20 --warmup 3"
  run 900 python bench.py --config $N $STEPS $CPU > $O/bench_c$N.log 2>&1
  tail -1 $O/bench_c$N.log > $O/bench_c$N.json
  run 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$N -o run -- python3 bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline --predict none --no-isolated > $O/c${N}_prof.log 2>&1
done
ls -R $O | head -60
