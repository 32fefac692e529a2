set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "9596 4 2" "9596 2 2" "9596 2 1" "2047 2 2" "4095 4 2" "800 2 1"; do timeout -k 10 60 tools/micro/trail_bench $a || exit 1; done
