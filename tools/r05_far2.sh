#!/bin/bash
# far1 / far2 split of the bulk trailing (one more super step of lookahead): parity, then A/B.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05far2}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tiled.py tests/test_h2f_cheb.py > $O/pytest.log 2>&1
tail -2 $O/pytest.log
for v in A B; do
  DBSLMM_LIB_PATH=$PWD/ablibs/lib_$v.so run 120 python tools/micro/tchol_alone.py 9600 > $O/alone_$v.log 2>&1
  echo "alone $v: $(tail -1 $O/alone_$v.log)"
done
bash tools/ab_libs.sh 4 3 ablibs/lib_A.so ablibs/lib_B.so
bash tools/ab_libs.sh 5 2 ablibs/lib_A.so ablibs/lib_B.so
echo done
