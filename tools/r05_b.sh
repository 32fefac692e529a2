#!/bin/bash
# Round 5: config-4 four-device parity (split h2f units), the multi-GPU rehearsal with the
# recalibrated shard model, and a kernel trace of the 9.6k block alone.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05b}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread "tests/test_fullscale.py::test_fullscale_blocks_match_oracle[4-multi]" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
run 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --predict none --no-e2e --predict 2,4,8 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
run 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof_alone -o run -- python tools/micro/tchol_alone.py 9600 > $O/prof_alone.log 2>&1
echo done
