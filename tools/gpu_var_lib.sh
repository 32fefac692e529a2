set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for lib in s2 s3 s4; do
  for cfg in 4 5; do
    L=dbslmm_amd/libdbslmm_hip.so; [ $lib = s2 ] || L=dbslmm_amd/libdbslmm_hip_$lib.so
    DBSLMM_LIB_PATH=$PWD/$L timeout -k 10 300 python bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/var/${lib}_c$cfg.log 2>&1 || { echo "fail $lib $cfg"; exit 1; }
  done
done
