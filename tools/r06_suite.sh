#!/bin/bash
# round 6: the whole GPU test suite on the final library
set -o pipefail
out=gpurun_out/r06/${1:-suite}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/tests.log 2>&1
