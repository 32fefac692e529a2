#!/bin/bash
# round 6: the driver's round-end sequence on the final tree -- whole GPU suite, smoke, default bench
set -o pipefail
out=gpurun_out/r06/${1:-final}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1 || exit 3
tail -1 $out/bench.log > $out/bench.json
