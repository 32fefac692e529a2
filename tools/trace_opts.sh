#!/bin/bash
# rocprofv3 kernel trace of a short config-4 bench per option set: tools/trace_opts.sh "OPTS_A" "OPTS_B" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
i=0
for o in "$@"; do
  args=""
  for kv in $o; do args="$args --opt $kv"; done
  rm -rf gpurun_out/tr$i
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr$i -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --predict none --no-e2e --no-isolated $args > gpurun_out/tr$i.log 2>&1
  rc=$?; echo "trace $i ($o) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=$((i+1))
done
