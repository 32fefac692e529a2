// Microbenchmark: sustained MFMA rate per dtype on this GPU (diagnostic tool).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
constexpr int ITERS = 4096;

__global__ void k_f64(double* out, double a0) {
    double a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    v4d c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ void k_f32(float* out, float a0) {
    float a = a0 + threadIdx.x, b = a0 - threadIdx.x;
    v4f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
__global__ void k_i8(int* out, int a0) {
    v4i a = {a0, a0 + 1, a0 + 2, (int)threadIdx.x}, b = {a0, a0 - 1, 3, (int)threadIdx.x};
    v16i c0 = {0}, c1 = {0};
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c1, 0, 0, 0);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[5];
}
typedef int v8i __attribute__((ext_vector_type(8)));
// v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 operands (format 4) and unit-ish scales, operand
// nibbles 0..2 like the Gram's dosage codes; 4 independent accumulators
__global__ void k_fp4(float* out, float a0) {
    const int t = threadIdx.x + (int)a0;
    const v8i a = {t & 0x33333333, 0x21021021, 0x12012012, t, 0, 0, 0, 0};
    const v8i b = {0x10210210, t ^ 0x02102102, 0x22112211, 0x11001100, 0, 0, 0, 0};
    v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 4, 4, 0, 0x80808080, 0, 0x80808080);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[5] + c2[9] + c3[15];
}
// the same on operands that change every iteration (random-looking dosage nibbles 0..2): the
// chip's clock under MFMA load depends on the data (DVFS)
__global__ void k_fp4r(float* out, float a0) {
    uint32_t x = 0x9E3779B9u * (threadIdx.x + 1) + (uint32_t)a0;
    v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
    for (int i = 0; i < ITERS; ++i) {
        x = x * 1664525u + 1013904223u;
        const int w = (int)(x & 0x33333333u), y = (int)((x >> 2) & 0x33333333u);
        const v8i a = {w, y, w ^ 0x11111111, y, 0, 0, 0, 0};
        const v8i b = {y, w, y ^ 0x01010101, w, 0, 0, 0, 0};
        c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c1, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c2, 4, 4, 0, 0x80808080, 0, 0x80808080);
        c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, b, c3, 4, 4, 0, 0x80808080, 0, 0x80808080);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[5] + c2[9] + c3[15];
}
__global__ void k_fma64(double* out, double a0) {
    double a = a0 + threadIdx.x, x0 = 1, x1 = 2, x2 = 3, x3 = 4, x4 = 5, x5 = 6, x6 = 7, x7 = 8;
    for (int i = 0; i < ITERS; ++i) {
        x0 = fma(x0, a, a); x1 = fma(x1, a, a); x2 = fma(x2, a, a); x3 = fma(x3, a, a);
        x4 = fma(x4, a, a); x5 = fma(x5, a, a); x6 = fma(x6, a, a); x7 = fma(x7, a, a);
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
template <typename F, typename T>
void run(const char* name, F kern, T* buf, double flops_per_wave_iter, int mfma_per_iter, int wpsimd) {
    const int blocks = 256 * 4, threads = 64 * wpsimd;  // 4 blocks per CU -> wpsimd waves/SIMD
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)1);
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, buf, (T)1);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double waves = (double)blocks * threads / 64 * 5;
    const double fl = waves * ITERS * flops_per_wave_iter;
    const double cyc_per_mfma = (ms * 1e-3) * 2.4e9 / (waves * ITERS * mfma_per_iter / (256.0 * 4));
    printf("%-8s waves/SIMD=%d  %8.1f TFLOP/s  (%.1f SIMD-cycles per instr at 2.4 GHz)\n", name, wpsimd, fl / (ms * 1e-3) / 1e12, cyc_per_mfma);
}
int main() {
    void* buf; hipMalloc(&buf, 1 << 24);
    for (int w = 1; w <= 2; ++w) {
        run("f64mfma", k_f64, (double*)buf, 4 * 2.0 * 16 * 16 * 4, 4, w);
        run("f32mfma", k_f32, (float*)buf, 4 * 2.0 * 16 * 16 * 4, 4, w);
        run("i8mfma", k_i8, (int*)buf, 2 * 2.0 * 32 * 32 * 32, 2, w);
        run("fp4mfma", k_fp4, (float*)buf, 4 * 2.0 * 32 * 32 * 64, 4, w);
        run("fp4rand", k_fp4r, (float*)buf, 4 * 2.0 * 32 * 32 * 64, 4, w);
        run("f64fma", k_fma64, (double*)buf, 8 * 2.0 * 64, 8, w);
    }
    return 0;
}
