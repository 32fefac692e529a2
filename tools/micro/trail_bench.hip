// Micro-benchmark of the 128 x 128 trailing-update kernels on one synthetic block (diagnostic).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o trail_bench tools/micro/trail_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
#include "../../include/dbslmm_hip.h"
#include "../../dbslmm_amd/csrc/chol.hip"
#include "../../dbslmm_amd/csrc/chol_tiled.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int m = argc > 1 ? atoi(argv[1]) : 8191;
    const int nk = argc > 2 ? atoi(argv[2]) : 2;
    const int run = argc > 3 ? atoi(argv[3]) : 2;
    const int ld = (m + 1 + 127) / 128 * 128;
    const int T2 = (m + 127) / 128, Tz2 = m / 128;
    const int il = nk, jl = nk;                      // tiles right of the panel columns 0 .. 128 nk
    std::vector<int32_t> items;
    double flops = 0;
    for (int I = il; I <= Tz2; ++I) {
        const int jmax = std::min(I, T2 - 1);
        for (int J = jl; J <= jmax; J += run) {
            items.push_back((0 << 16) | (I << 8) | J);
            items.push_back(nk);                           // (step 0 << 8) | nk
            for (int j = J; j <= std::min(J + run - 1, jmax); ++j) flops += 2.0 * 128 * 128 * 128 * nk * (j == I ? 0.75 : 1.0);
        }
    }
    double* M;
    CK(hipMalloc(&M, sizeof(double) * ld * ld));
    std::vector<double> h(static_cast<size_t>(ld) * ld);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * ((i * 2654435761u) % 1000);
    CK(hipMemcpy(M, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    int32_t *d_items, *d_i32;
    int64_t* d_i64;
    double* d_dbl;
    CK(hipMalloc(&d_items, items.size() * 4));
    CK(hipMemcpy(d_items, items.data(), items.size() * 4, hipMemcpyHostToDevice));
    int32_t hi[8] = {0, m, m, ld, 0, 0, 0, 0};
    CK(hipMalloc(&d_i32, 64));
    CK(hipMemcpy(d_i32, hi, 32, hipMemcpyHostToDevice));
    int64_t z64 = 0;
    CK(hipMalloc(&d_i64, 8));
    CK(hipMemcpy(d_i64, &z64, 8, hipMemcpyHostToDevice));
    CK(hipMalloc(&d_dbl, 64));
    chol::TiledArgs ta{M, d_i32 + 0, d_i32 + 1, d_i32 + 2, d_i32 + 3, d_i64, d_i32 + 4, d_dbl, d_i32 + 4,
                       d_dbl, d_dbl, 1.0, d_dbl, d_dbl, d_dbl, d_i32 + 5, 1, 0, 0, 0, 0, 0};
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(dbslmm_tchol_trailing3),
                           hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(double) * chol::kTrail3Doubles));
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(dbslmm_tchol_trailing3k16),
                           hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(double) * chol::kTrail3k16Doubles));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int n_it = static_cast<int>(items.size() / 2);
    for (int k = 0; k < 2; ++k) {   // 0: K = 32 per stage, one workgroup per CU; 1: K = 16, two
        auto launch = [&] {
            if (k == 0) hipLaunchKernelGGL(dbslmm_tchol_trailing3, dim3(n_it), dim3(512), sizeof(double) * chol::kTrail3Doubles, 0, ta, run, d_items, n_it);
            else hipLaunchKernelGGL(dbslmm_tchol_trailing3k16, dim3(n_it), dim3(512), sizeof(double) * chol::kTrail3k16Doubles, 0, ta, run, d_items, n_it);
        };
        for (int w = 0; w < 2; ++w) launch();
        CK(hipGetLastError());
        CK(hipEventRecord(e0));
        const int reps = 5;
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%s m=%d nk=%d run=%d items=%d  %.3f ms  %.1f TF/s (%.1f%% of 78.6)\n", k ? "trailing3k16" : "trailing3",
               m, nk, run, n_it, ms, flops / ms * 1e-9, flops / ms * 1e-9 / 78.6 * 100);
    }
    // the two variants must agree bit for bit (same K order per element): rerun each once from the
    // same input and compare
    std::vector<double> r0(h.size()), r1(h.size());
    for (int k = 0; k < 2; ++k) {
        CK(hipMemcpy(M, h.data(), h.size() * 8, hipMemcpyHostToDevice));
        if (k == 0) hipLaunchKernelGGL(dbslmm_tchol_trailing3, dim3(n_it), dim3(512), sizeof(double) * chol::kTrail3Doubles, 0, ta, run, d_items, n_it);
        else hipLaunchKernelGGL(dbslmm_tchol_trailing3k16, dim3(n_it), dim3(512), sizeof(double) * chol::kTrail3k16Doubles, 0, ta, run, d_items, n_it);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(k ? r1.data() : r0.data(), M, h.size() * 8, hipMemcpyDeviceToHost));
    }
    size_t ndiff = 0;
    double maxd = 0;
    for (size_t i = 0; i < h.size(); ++i)
        if (r0[i] != r1[i]) { ++ndiff; maxd = std::max(maxd, std::fabs(r0[i] - r1[i])); }
    printf("k16 vs k32: %zu elements differ, max |diff| %.3e\n", ndiff, maxd);
    return 0;
}
