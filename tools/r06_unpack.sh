#!/bin/bash
# round 6: the dwordx4 unpack + reverted symv order: GPU parity subset, config 4 bench + profile,
# per-device rehearsal breakdown of config 4
set -o pipefail
out=gpurun_out/r06/${1:-unpack}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu.py tests/test_pcg.py tests/test_cli.py tests/test_valid.py > $out/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none > $out/c4.json 2> $out/c4.err || exit 2
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o c4 -- python3 /root/repo/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/prof_c4.json 2> /root/repo/$out/prof_c4.err) || exit 3
timeout -k 10 300 python -u tools/r06_dev.py $out/dev_c4.json 4 1,2,4,8 > $out/dev_c4.log 2>&1 || exit 4
