#!/bin/bash
# Same-box A/B of bench.py option sets: tools/ab_opts.sh CONFIG "OPTS_A" "OPTS_B" ... (each a list of --opt k=v)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; shift
mkdir -p gpurun_out/ab
i=0
for o in "$@"; do
  args=""
  for kv in $o; do args="$args --opt $kv"; done
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --predict none --no-e2e --no-isolated $args > gpurun_out/ab/c${cfg}_$i.log 2>&1
  rc=$?
  [ $rc -eq 0 ] || { echo "FAILED rc=$rc ($o)"; tail -5 gpurun_out/ab/c${cfg}_$i.log; exit $rc; }
  python - "$o" gpurun_out/ab/c${cfg}_$i.log << 'PY'
import json, sys
p = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {x["kernel"]: x for x in p["kernels"]}
print(f"{sys.argv[1] or 'default':32s} {p['ms_per_step']:7.2f} ms  tchol {k['dbslmm_tchol']['ms']:6.2f}  trsv {k['dbslmm_trsv']['ms']:6.2f}  gram {k['dbslmm_gram_i8']['ms']:5.2f}")
PY
  i=$((i+1))
done
