set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "8191 2 2" "8191 2 1" "8191 16 2" "2047 2 2" "4095 2 2" "8191 4 2"; do timeout -k 10 60 tools/micro/trail_bench $a || exit 1; done
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -i -E "mfma|TCC_HIT|TCC_MISS|TCC_EA0_RD|TCP_TCC|SQ_WAIT|SQ_BUSY|LDS_BANK|SQ_INSTS_LDS" gpurun_out/counters.txt | cut -c1-150 | sort -u | head -60
