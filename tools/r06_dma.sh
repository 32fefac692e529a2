#!/bin/bash
# round 6: dwordx4 unpack + LDS-DMA uint16 product (dbslmm_pcg_symv16d) vs the register product
# (DBSLMM_PCG_DMA=0): GPU parity subset, config 4 / 5 A/B, kernel trace, per-device rehearsal
set -o pipefail
out=gpurun_out/r06/${1:-dma}
mkdir -p $out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-e2e --predict none"
timeout -k 10 600 $T tests/test_pcg.py tests/test_gpu.py tests/test_cli.py tests/test_valid.py > $out/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_dma.json 2> $out/c4_dma.err || exit 2
DBSLMM_PCG_DMA=0 timeout -k 10 200 python -u bench.py --config 4 $B > $out/c4_reg.json 2> $out/c4_reg.err || exit 3
timeout -k 10 200 python -u bench.py --config 5 $B > $out/c5_dma.json 2> $out/c5_dma.err || exit 4
DBSLMM_PCG_DMA=0 timeout -k 10 200 python -u bench.py --config 5 $B > $out/c5_reg.json 2> $out/c5_reg.err || exit 5
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d /root/repo/$out/prof -o c4 -- python3 /root/repo/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --predict none --no-isolated > /root/repo/$out/prof_c4.json 2> /root/repo/$out/prof_c4.err) || exit 6
timeout -k 10 300 python -u tools/r06_dev.py $out/dev_c4.json 4 1,2,4,8 > $out/dev_c4.log 2>&1 || exit 7
