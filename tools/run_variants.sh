set -u
for t in 256 512; do
  echo "== threads $t"
  DBSLMM_LIB_PATH=dbslmm_amd/libdbslmm_hip_t$t.so timeout -k 10 200 python tools/chol_probe.py || exit 1
  python - <<PY
import os
os.environ["DBSLMM_LIB_PATH"]="dbslmm_amd/libdbslmm_hip_stamps_t$t.so"
PY
  sed "s#libdbslmm_hip_stamps.so#libdbslmm_hip_stamps_t$t.so#" tools/stamp_probe.py > gpurun_out/sp.py && timeout -k 10 100 python gpurun_out/sp.py || exit 1
done
