#!/bin/bash
# Capped rest-unpack grid (grid-stride) A/B: 0 = uncapped, 2 / 6 workgroups per CU; fresh
# bench processes alternating, to see how often the slow step mode appears.
set -u
export TMPDIR=/tmp
bash tools/ab_libs.sh 4 4 ablibs/lib_A.so ablibs/lib_B.so ablibs/lib_C.so
echo done
