#!/bin/bash
# Gram head / tail split (the first super step overlaps the Gram tail): full GPU suite, the 9.6k
# block alone, the rehearsal, and config 4 / 5 steps
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05ghead}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -1 $O/pytest_gpu.log
run 200 python tools/micro/tchol_alone.py 9600 > $O/alone.log 2>&1
echo "alone $(tail -1 $O/alone.log)"
run 500 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict 4,8 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
python - $O/bench_c4.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("N=1", round(d["ms_per_step"], 2))
for n, r in d["predicted_multi_gpu"]["results"].items():
    print("N=" + n, round(r["step_ms"], 2), [round(x, 2) for x in r["per_device_ms"]])
PY
run 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --predict none --no-e2e --no-isolated > $O/bench_c5.log 2>&1
python3 -c "import json;d=json.loads(open('$O/bench_c5.log').read().strip().splitlines()[-1]);print('c5', round(d['ms_per_step'],2))"
echo done
