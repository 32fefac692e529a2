#!/bin/bash
# ten fresh bench processes of the default config-4 step (CG build), their
# ms_per_step side by side.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-modes10}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
for i in $(seq 1 10); do
  run 300 python bench.py --no-cpu-baseline --predict none --no-e2e --no-check --no-isolated > $O/b$i.log 2>&1
  tail -1 $O/b$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('process $i', round(d['ms_per_step'],3))" >> $O/modes.txt
done
python - $O/modes.txt <<'PY'
import sys
v = [float(l.split()[-1]) for l in open(sys.argv[1])]
print("min %.3f max %.3f spread %.3f ms" % (min(v), max(v), max(v) - min(v)))
PY
