#!/bin/bash
# multi-device download in one pass + the device-scatter RCCL gather (GPU tests), the N = 8 bulk
# device's lead substitution grid sweep, and the config-4 one-GPU rehearsal of N = 2 / 4 / 8
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05mdl}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multi.py tests/test_dist.py > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for g in 0; do
  run 300 python tools/micro/units_alone.py 8 7 5 sub_grid_lead=$g > $O/grid_$g.log 2>&1
  echo "sub_grid_lead $g: $(grep 'ms per run' $O/grid_$g.log)"
done
run 500 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict 2,3,4,8 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
python - $O/bench_c4.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("N=1", round(d["ms_per_step"], 2))
for n, r in d["predicted_multi_gpu"]["results"].items():
    print("N=" + n, round(r["step_ms"], 2), [round(x, 2) for x in r["per_device_ms"]], "model", [round(x, 2) for x in r["model_ms"]])
PY
echo done
