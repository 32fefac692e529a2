// Diagnostic variants of dbslmm_tchol_trailing3's main loop (which part costs what).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/dbslmm_hip.h"
#include "../../dbslmm_amd/csrc/chol.hip"
#include "../../dbslmm_amd/csrc/chol_tiled.hip"
using namespace chol;
// mode 0: MFMA + LDS reads only; 1: + barrier per stage; 2: + DMA per stage; 3: + C load/store;
// 4: DMA + C store only; 5: DMA + C load only; 6: as 2 on the triangular tile set; 7: as 3 on it
template <int MODE>
__global__ __launch_bounds__(512, 1) void probe(double* A, int ld, int n_items, int nst) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 2, wc = wave & 3;
    int I = 2 + (blockIdx.x % 60), J = 2 + (blockIdx.x % 50);
    if (MODE >= 6) {   // triangular tile enumeration of a 8192-row block (as the trailing update)
        int e = blockIdx.x % 1953, r = 2;
        while (e >= r - 1) { e -= r - 1; ++r; }
        I = r; J = 2 + e;
    }
    v4d acc[4][2];
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) acc[i][j] = v4d{0, 0, 0, 0};
    if (MODE == 3 || MODE == 5 || MODE == 7) t3_load_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * J + 32 * wc, lane);
    if (MODE >= 2) t3_issue(lds, A, ld, I, J, 0, false, wave, lane);
    for (int g = 0; g < nst; ++g) {
        double* S = lds + (MODE >= 2 ? (g & 1) * 2 * kOp3 : 0);
        if (MODE >= 1) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        if (MODE >= 2 && g + 1 < nst) t3_issue(lds + ((g + 1) & 1) * 2 * kOp3, A, ld, I, J, kK2 * (g + 1), false, wave, lane);
        t3_mfma_stage(acc, S, S + kOp3, wr, wc, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (MODE == 3 || MODE == 4 || MODE == 7) t3_store_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * J + 32 * wc, lane);
    else {
        double t = 0;
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 2; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
        if (t == 12345.0) A[tid] = t;
    }
}
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)
template <int MODE> int run(double* M, int ld, int n, int nst) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe<MODE>), hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(double) * kTrail3Doubles));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(probe<MODE>, dim3(n), dim3(512), sizeof(double) * kTrail3Doubles, 0, M, ld, n, nst);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<MODE>, dim3(n), dim3(512), sizeof(double) * kTrail3Doubles, 0, M, ld, n, nst);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    const double fl = 2.0 * 128 * 128 * 32 * nst * n;
    printf("mode %d nst=%d WGs=%d: %.3f ms %.1f TF/s (%.1f%%)\n", MODE, nst, n, ms, fl / ms * 1e-9, fl / ms * 1e-9 / 78.6 * 100);
    return 0;
}
int main() {
    const int ld = 8192;
    double* M; CK(hipMalloc(&M, sizeof(double) * ld * ld)); CK(hipMemset(M, 0, sizeof(double) * ld * ld));
    for (int nst : {8, 64}) {
        if (run<2>(M, ld, 1953, nst) || run<3>(M, ld, 1953, nst) || run<6>(M, ld, 1953, nst) || run<7>(M, ld, 1953, nst)) return 1;
    }
    return 0;
}
