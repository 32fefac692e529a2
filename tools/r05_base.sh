#!/bin/bash
# Round-5 check: the new / changed GPU tests, the config-4 bench line (no CPU leg) with the
# one-GPU multi-GPU rehearsal, the 9.6k block alone, and a kernel trace of the block alone.
# Outputs under gpurun_out/${GOUT:-r05base}/.
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-r05base}; mkdir -p $O
run() { local to=$1; shift; timeout -k 10 "$to" "$@"; local rc=$?; [ $rc -eq 0 ] || { echo "FAILED rc=$rc: $*"; exit $rc; }; }
run 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_multi.py tests/test_dist.py \
    "tests/test_tiled.py::test_outputs_refused_after_debug_stop" \
    "tests/test_tiled.py::test_fused_cheb_with_lead_group_matches_unfused" \
    "tests/test_tiled.py::test_split_substitutions_bit_identical" > $O/pytest.log 2>&1
tail -3 $O/pytest.log
run 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict 2,4,8 > $O/bench_c4.log 2>&1
tail -1 $O/bench_c4.log > $O/bench_c4.json
python tools/bench_summary.py $O/bench_c4.json 2>/dev/null | tail -3
run 120 python tools/micro/tchol_alone.py 9600 > $O/alone.log 2>&1
cat $O/alone.log
run 180 rocprofv3 --kernel-trace --stats -d $O/prof_alone -o run -- python tools/micro/tchol_alone.py 9600 > $O/prof_alone.log 2>&1
echo done
