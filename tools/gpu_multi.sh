#!/bin/bash
# Multi-device checks on a 1-GPU box: the GPU test suite (incl. tests/test_multi.py: shards of one
# problem on repeated device 0), the default bench, then a 2-rank rehearsal of bench.py's sharded
# (strong-scaling) mode with both ranks on device 0 (gloo: RCCL refuses two ranks on one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout-s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "== $name" | tee -a gpurun_out/steps.log
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a gpurun_out/steps.log
    tail -3 "gpurun_out/$name.log"
    case $rc in
        0|1|5) return 0 ;;
        *) echo "stopping after $name (rc=$rc)"; exit $rc ;;
    esac
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step bench 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --predict none
step rehearse_c3 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config 3 --steps 5 --warmup 2 --dist-backend gloo --rank-device 0
step rehearse_c4 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --rank-device 0
echo done
