#!/bin/bash
# Round evidence, part 2: the upload probe (2.5 GB file in the box's page cache), bench lines of
# configs 1, 2, 3, 5 and kernel stats of configs 2, 3, 5.  Outputs under gpurun_out/${GOUT:-r2}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r2}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
head -c 2500000000 /dev/zero | tr '\0' 'U' > /tmp/up_probe.bed
run 120 tools/micro/upload_probe /tmp/up_probe.bed > $O/upload_probe.txt 2>&1
rm -f /tmp/up_probe.bed
run 300 python bench.py --config 1 > $O/bench_c1.log 2>&1
tail -1 $O/bench_c1.log > $O/bench_c1.json
for N in 2 3 5; do
  CPU=""; [ $N -le 3 ] || CPU="--no-cpu-baseline --predict none"
  STEPS="--steps 5 --warmup 2"; [ $N -eq 2 ] && STEPS="--steps 20 --warmup 3"
  run 600 python bench.py --config $N $STEPS $CPU > $O/bench_c$N.log 2>&1
  tail -1 $O/bench_c$N.log > $O/bench_c$N.json
  run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c$N -o run -- python3 bench.py --config $N --steps 3 --warmup 1 --no-cpu-baseline --predict none --no-isolated --no-e2e > $O/c${N}_prof.log 2>&1
done
echo done
