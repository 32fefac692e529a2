#!/bin/bash
# rocprofv3 kernel trace of a short config-N bench (default 3) -> gpurun_out/prof_c<N>/
N=${1:-3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$N -o run --output-format csv -- python3 bench.py --config $N --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c$N.log 2>&1
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/prof_c$N.log
exit $rc
