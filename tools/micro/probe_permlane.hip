// gfx950 v_permlane16_swap / v_permlane32_swap semantics probe: every lane holds its lane id; prints
// both results of each swap per lane.  Build: hipcc --offload-arch=gfx950 -o probe_permlane probe_permlane.hip
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* o) {
    const unsigned x = threadIdx.x;
    const auto r32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    const auto r16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    o[4 * x + 0] = r32[0];
    o[4 * x + 1] = r32[1];
    o[4 * x + 2] = r16[0];
    o[4 * x + 3] = r16[1];
}
int main() {
    unsigned* d;
    unsigned h[256];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int ok32 = 1, ok16 = 1;
    for (unsigned l = 0; l < 64; ++l) {
        printf("lane %2u: p32 %2u %2u  p16 %2u %2u\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
        const unsigned x32 = (l & 32) ? h[4 * l] : h[4 * l + 1], x16 = (l & 16) ? h[4 * l + 2] : h[4 * l + 3];
        ok32 &= x32 == (l ^ 32u);
        ok16 &= x16 == (l ^ 16u);
    }
    printf("xor32 = (lane & 32) ? r[0] : r[1]: %s\nxor16 = (lane & 16) ? r[0] : r[1]: %s\n", ok32 ? "yes" : "NO", ok16 ? "yes" : "NO");
    hipFree(d);
    return 0;
}
