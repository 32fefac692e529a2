// Which CUs does a stream created with hipExtStreamCreateWithCUMask run on? (diagnostic)
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o tools/micro/cumask_probe tools/micro/cumask_probe.hip
// Each workgroup records (XCC_ID, HW_ID) of its wave; the host prints the distinct (xcc, se, sh, cu)
// used for several masks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void probe(unsigned* out) {
    if (threadIdx.x == 0) {
        unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
        unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
        // keep the workgroup resident a little so the dispatcher spreads the grid
        for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(10);
    }
}

int main() {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nwg = 4096;
    unsigned* d;
    CK(hipMalloc(&d, nwg * 8));
    std::vector<unsigned> h(2 * nwg);
    const int nw = (ncu + 31) / 32;
    struct M { const char* name; std::vector<uint32_t> m; };
    std::vector<M> masks;
    { std::vector<uint32_t> m(nw, 0); m[0] = 0xFFFFFFFFu; masks.push_back({"bits 0-31", m}); }
    { std::vector<uint32_t> m(nw, 0); for (int i = 0; i < ncu; i += 8) m[i / 32] |= 1u << (i % 32); masks.push_back({"every 8th bit", m}); }
    { std::vector<uint32_t> m(nw, 0); for (int i = 0; i < 8; ++i) m[i / 32] |= 1u << (i % 32); masks.push_back({"bits 0-7", m}); }
    { std::vector<uint32_t> m(nw, 0); m[0] = 1u; masks.push_back({"bit 0", m}); }
    { std::vector<uint32_t> m(nw, 0); m[nw - 1] = 0x80000000u; masks.push_back({"last bit", m}); }
    for (auto& mk : masks) {
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mk.m.size()), mk.m.data()));
        hipLaunchKernelGGL(probe, dim3(nwg), dim3(64), 0, s, d);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d, nwg * 8, hipMemcpyDeviceToHost));
        std::set<std::tuple<int, int, int, int>> cus;
        for (int i = 0; i < nwg; ++i) {
            const unsigned hw = h[2 * i], xcc = h[2 * i + 1] & 0xF;
            cus.insert({static_cast<int>(xcc), static_cast<int>((hw >> 13) & 7), static_cast<int>((hw >> 12) & 1),
                        static_cast<int>((hw >> 8) & 15)});
        }
        printf("%-14s: %zu CUs:", mk.name, cus.size());
        int k = 0;
        for (auto& c : cus) {
            if (k++ < 40) printf(" x%d.se%d.sh%d.cu%d", std::get<0>(c), std::get<1>(c), std::get<2>(c), std::get<3>(c));
        }
        printf("\n");
        CK(hipStreamDestroy(s));
    }
    return 0;
}
