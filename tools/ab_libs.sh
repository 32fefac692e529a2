#!/bin/bash
# Same-box A/B of library builds on one config: tools/ab_libs.sh CONFIG ROUNDS lib_a.so lib_b.so ...
# (alternating, each a short bench.py line through DBSLMM_LIB_PATH)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; rounds=$2; shift 2
mkdir -p gpurun_out/abl
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    log=gpurun_out/abl/c${cfg}_$(basename $lib .so)_$r.log
    DBSLMM_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --predict none --no-e2e --no-isolated > $log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc ($lib)"; tail -5 $log; exit $rc; }
    python - "$lib" $log << 'PY'
import json, sys
p = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = {x["kernel"]: x for x in p["kernels"]}
print(f"{sys.argv[1]:40s} {p['ms_per_step']:7.2f} ms  tchol {k['dbslmm_tchol']['ms']:6.2f}  trsv {k['dbslmm_trsv']['ms']:6.2f}  unpack {k['dbslmm_unpack_stats']['ms']:5.2f} gram {k['dbslmm_gram_i8']['ms']:5.2f}")
PY
  done
done
