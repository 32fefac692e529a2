// Micro-benchmark (diagnostic): latency of one inter-workgroup hand-off hop on MI355X.
// Workgroup i waits for flag[i-1] (one lane polls, sc1), optionally reads a 64-double payload
// with sc1 loads, writes its own payload (sc1 stores), drains, barrier, then sets flag[i] (sc1).
// Reports us per hop for: flag only; flag + payload; flag + payload + an LDS/barrier round.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/micro/chain_bench tools/micro/chain_bench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(512, 1) void chain(int* flags, double* pay, int n, int epoch, int mode, int* ctr) {
    __shared__ int s_t;
    __shared__ double buf[64];
    const int tid = threadIdx.x;
    if (tid == 0) s_t = atomicAdd(ctr, 1);     // ticket order = chain order
    __syncthreads();
    const int i = s_t;
    if (i >= n) return;
    if (i > 0) {
        if (tid == 0)
            while (__hip_atomic_load(flags + i - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch)
                __builtin_amdgcn_s_sleep(1);
        __syncthreads();
        if (mode >= 1 && tid < 64) buf[tid] = __hip_atomic_load(pay + 64 * (i - 1) + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (mode >= 2) __syncthreads();
    }
    if (mode >= 1 && tid < 64) __hip_atomic_store(pay + 64 * i + tid, (mode >= 2 ? buf[tid] : 0.0) + 1.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(flags + i, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int main() {
    const int n = 2048;
    int *flags, *ctr;
    double* pay;
    CK(hipMalloc(&flags, n * 4));
    CK(hipMalloc(&ctr, 4));
    CK(hipMalloc(&pay, n * 64 * 8));
    CK(hipMemset(flags, 0, n * 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int epoch = 0;
    for (int mode = 0; mode < 3; ++mode) {
        for (int grid : {256, 2048}) {
            float best = 1e9;
            for (int rep = 0; rep < 3; ++rep) {
                ++epoch;
                CK(hipMemset(ctr, 0, 4));
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(chain, dim3(grid), dim3(512), 0, 0, flags, pay, grid, epoch, mode, ctr);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("mode %d (0 flag, 1 +payload, 2 +payload via LDS) chain %d: %.3f ms  %.2f us/hop\n", mode, grid, best, best * 1e3 / grid);
        }
    }
    return 0;
}
