#!/bin/bash
# factorisation chain of one block alone (tools/micro/tchol_alone.py) vs its size
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05chainm}; mkdir -p $O
for m in 1600 2600 4000 5500 7500 9600; do
  timeout -k 10 200 python tools/micro/tchol_alone.py $m > $O/alone_$m.log 2>&1 || { echo FAILED $m; tail -3 $O/alone_$m.log; exit 1; }
  echo "m $m $(tail -1 $O/alone_$m.log)"
done
echo done
