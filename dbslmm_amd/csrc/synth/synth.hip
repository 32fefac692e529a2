// Synthetic PLINK panel generator on the GPU (benchmark / scale-test tooling, NOT part of the
// drop-in ABI in include/dbslmm_hip.h).  Same model as dbslmm_amd/synth.py:
// two haplotypes per individual from an AR(1) latent Gaussian along the SNPs of each LD block,
// thresholded at Phi^-1(p); dosage = h1 + h2; optional missing calls.  Random numbers come from a
// counter hash of (seed, snp, individual), so the panel does not depend on the launch shape.
//
// Thread = (block, byte column): it owns 4 individuals (8 haplotypes), walks the block's SNPs in
// order carrying the 8 AR(1) states in registers and writes one packed byte per SNP.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#include "../../../include/dbslmm_synth.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// two N(0,1) from one 64-bit hash (Box-Muller on two 24-bit uniforms)
__device__ __forceinline__ void normal2(uint64_t h, float& a, float& b) {
    const float u1 = ((float)(uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    const float u2 = ((float)(uint32_t)((h >> 8) & 0xFFFFFFu) + 0.5f) * (1.0f / 16777216.0f);
    const float r = __fsqrt_rn(-2.0f * __logf(u1));
    float s, c;
    __sincosf(6.28318530718f * u2, &s, &c);
    a = r * c;
    b = r * s;
}

__global__ __launch_bounds__(256) void synth_panel(const int64_t* __restrict__ blk_ptr,
                                                   const float* __restrict__ thr,
                                                   uint8_t* __restrict__ out, int n_ref,
                                                   int64_t nb, uint64_t seed, float rho,
                                                   float miss_rate) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nb) return;
    const int b = blockIdx.y;
    const int64_t s0 = blk_ptr[b], s1 = blk_ptr[b + 1];
    const float a = sqrtf(1.0f - rho * rho);
    const int nind = min(4, n_ref - (int)(4 * g));
    const uint64_t key = mix64(seed);
    float u[8];
    for (int64_t s = s0; s < s1; ++s) {
        const uint64_t base = mix64(key ^ ((uint64_t)s << 22) ^ (uint64_t)g);
        float e[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) normal2(mix64(base + (uint64_t)k * 0xD1B54A32D192ED03ull), e[2 * k], e[2 * k + 1]);
        if (s == s0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) u[k] = e[k];
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) u[k] = rho * u[k] + a * e[k];
        }
        const float t = thr[s];
        const uint64_t mh = miss_rate > 0.0f ? mix64(base ^ 0x5851F42D4C957F2Dull) : 0;
        uint32_t byte = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t code = 0;                                   // padding individuals: 00
            if (j < nind) {
                const int d = (u[2 * j] < t) + (u[2 * j + 1] < t);
                code = d == 2 ? 0u : (d == 1 ? 2u : 3u);          // 2->00, 1->10, 0->11
                const float um = ((float)((mh >> (16 * j)) & 0xFFFFu) + 0.5f) * (1.0f / 65536.0f);
                if (miss_rate > 0.0f && um < miss_rate) code = 1u;  // missing -> 01
            }
            byte |= code << (2 * j);
        }
        out[s * nb + g] = (uint8_t)byte;
    }
}

thread_local char g_err[256];

int fail(const char* what, hipError_t e) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -2;
}

}  // namespace

extern "C" const char* dbslmm_synth_last_error(void) { return g_err; }

extern "C" int dbslmm_synth_bed(int device, int32_t num_block, const int64_t* blk_ptr,
                                const float* thr, int32_t n_ref, uint64_t seed, float rho,
                                float miss_rate, uint8_t* rows) {
    if (num_block <= 0 || !blk_ptr || !thr || !rows || n_ref <= 0 || !(rho >= 0.0f && rho < 1.0f)) {
        snprintf(g_err, sizeof(g_err), "bad argument");
        return -1;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return fail("hipSetDevice", e);
    const int64_t m = blk_ptr[num_block], nb = (n_ref + 3) / 4;
    for (int b = 0; b < num_block; ++b)
        if (blk_ptr[b + 1] < blk_ptr[b]) { snprintf(g_err, sizeof(g_err), "blk_ptr not monotone"); return -1; }
    int64_t* d_ptr = nullptr;
    float* d_thr = nullptr;
    uint8_t* d_out = nullptr;
    int rc = 0;
    if ((e = hipMalloc(&d_ptr, (num_block + 1) * sizeof(int64_t))) != hipSuccess ||
        (e = hipMalloc(&d_thr, (m > 0 ? m : 1) * sizeof(float))) != hipSuccess ||
        (e = hipMalloc(&d_out, (m * nb > 0 ? m * nb : 1))) != hipSuccess) {
        rc = fail("hipMalloc", e);
    } else if ((e = hipMemcpy(d_ptr, blk_ptr, (num_block + 1) * sizeof(int64_t), hipMemcpyHostToDevice)) != hipSuccess ||
               (e = hipMemcpy(d_thr, thr, m * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess) {
        rc = fail("hipMemcpy H2D", e);
    } else if (m > 0) {
        dim3 grid((unsigned)((nb + 255) / 256), (unsigned)num_block);
        synth_panel<<<grid, 256>>>(d_ptr, d_thr, d_out, n_ref, nb, seed, rho, miss_rate);
        if ((e = hipGetLastError()) != hipSuccess) rc = fail("synth_panel launch", e);
        else if ((e = hipMemcpy(rows, d_out, m * nb, hipMemcpyDeviceToHost)) != hipSuccess) rc = fail("hipMemcpy D2H", e);
    }
    (void)hipFree(d_ptr);
    (void)hipFree(d_thr);
    (void)hipFree(d_out);
    return rc;
}
