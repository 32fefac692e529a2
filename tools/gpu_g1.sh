# Gram probe (tools/micro/gram_probe.py): product library vs the diagnostic builds
# (DBSLMM_GRAM_DIAG 1: no FP4 expansion, 2: no operand DMA after the prologue)
set -u
export TMPDIR=/tmp
O=gpurun_out/${GOUT:-g7}; mkdir -p $O
for L in "" _gdiag1 _gdiag2; do
  for M in "4096 16" "0"; do
    DBSLMM_LIB_PATH=$PWD/dbslmm_amd/libdbslmm_hip$L.so timeout -k 10 200 python -u tools/micro/gram_probe.py $M > "$O/probe${L}_${M// /_}.log" 2>&1 || exit $?
  done
done
