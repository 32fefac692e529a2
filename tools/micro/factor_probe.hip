// factor_probe.hip -- one 32 x 32 tile through chol::factor_tile_lds and a software-pipelined
// variant; outputs compared bit for bit on the host.
#include "../../include/dbslmm_hip.h"
#include "../../dbslmm_amd/csrc/chol.hip"
#include "../../dbslmm_amd/csrc/chol_tiled.hip"
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
namespace chol {
__device__ __forceinline__ bool factor_pipe(double* T, double* Xo, double* colb, int c0, int m,
                                                int ms, double dshift, int lane) {
    const int r = lane & 31;
    const bool xlane = lane >= kT;
    const int jmax = min(kT, m - c0);
    double v[kT];
#pragma unroll
    for (int c = 0; c < kT; ++c) {
        double t = xlane ? (c == r ? 1.0 : 0.0) : (c <= r ? T[r * kTS + c] : 0.0);
        if (!xlane && c == r && c0 + r < ms) t += dshift;
        v[c] = t;
    }
    wave_sync();
    bool fail = false;
    // Software-pipelined steps: step j's column goes out through LDS at the end of step j and is
    // read back at the start of step j + 1, before that step's pivot chain, so the LDS round trip
    // overlaps the pivot's readlane / rsqrt / scale.  Column j + 1 (the next pivot's) takes
    // L[j + 1][j] by readlane instead.  Every column still receives its updates in step order:
    // the same operations as an LDS broadcast per step.
    double vjp = 0.0;     // previous step's scaled column value (0 on a dead step)
#pragma unroll
    for (int j = 0; j < kT; ++j) {
        double col[kT];   // step j - 1's LDS column (entries k > j)
        if (j >= 1 && j + 1 < kT) {
            const double* cb = colb + kT * ((j - 1) & 1);
#pragma unroll
            for (int k0 = (j + 1) & ~1; k0 < kT; k0 += 2) {
                const v2d t = *reinterpret_cast<const v2d*>(cb + k0);
                col[k0] = t[0];
                col[k0 + 1] = t[1];
            }
        }
        double vj = 0.0;                        // dead step: the updates leave v unchanged
        if (j < jmax) {
            const double p = readlane_f64(v[j], j);
            fail |= !(p > 0.0);
            const double rs = rsqrt_f64(p);
            v[j] = (!xlane && r < j) ? 0.0 : v[j] * rs;
            vj = v[j];
        }
        // step j - 1's update of columns j + 1 ..
        if (j >= 1) {
#pragma unroll
            for (int k = j + 1; k < kT; ++k) v[k] -= vjp * col[k];
        }
        // step j's update of column j + 1 (the next pivot's)
        if (j + 1 < kT) v[j + 1] -= vj * readlane_f64(v[j], j + 1);
        // step j's column for columns j + 2 .. into LDS: one wave, so its LDS operations execute
        // in issue order, and the compiler keeps the store / loads (possibly aliasing addresses)
        // in program order
        if (j + 2 < kT) colb[kT * (j & 1) + r + (xlane ? 4 * kT : 0)] = v[j];   // X lanes: spare slots, no divergent store
        vjp = vj;
    }
    if (!xlane) {
#pragma unroll
        for (int c = 0; c < kT; ++c) T[r * kTS + c] = c <= r ? v[c] : 0.0;
    } else {
#pragma unroll
        for (int q = 0; q < kT; ++q) Xo[q * kTS + r] = q >= jmax ? (q == r ? 1.0 : 0.0) : v[q];
    }
    wave_sync();
    return fail;
}

}
__global__ void probe(const double* in, double* outT, double* outX, int* fl, int jmax, int pipe) {
    using namespace chol;
    __shared__ double T[kT * kTS], X[kT * kTS], colb[6 * kT + 8];
    const int lane = threadIdx.x;
    for (int e = lane; e < kT * kTS; e += 64) { T[e] = in[e]; X[e] = 0.0; }
    __syncthreads();
    bool f = pipe ? factor_pipe(T, X, colb, 0, jmax, 0, 0.0, lane) : factor_tile_lds(T, X, colb, 0, jmax, 0, 0.0, lane);
    __syncthreads();
    for (int e = lane; e < kT * kTS; e += 64) { outT[e] = T[e]; outX[e] = X[e]; }
    if (lane == 0) fl[0] = f;
}
int main() {
    using namespace chol;
    const int N = kT * kTS;
    std::vector<double> A(N, 0.0);
    srand(1);
    std::vector<double> G(40 * kT);
    for (auto& g : G) g = (rand() / (double)RAND_MAX) - 0.5;
    for (int r = 0; r < kT; ++r) for (int c = 0; c < kT; ++c) {
        double s = 0; for (int k = 0; k < 40; ++k) s += G[k * kT + r] * G[k * kT + c];
        A[r * kTS + c] = s / 40 + (r == c ? 0.1 : 0.0);
    }
    double *din, *dT, *dX; int* dfl;
    hipMalloc(&din, N * 8); hipMalloc(&dT, 2 * N * 8); hipMalloc(&dX, 2 * N * 8); hipMalloc(&dfl, 8);
    int bad = 0;
    for (int jmax : {32, 20}) {
        std::vector<double> In = A;
        for (int r = jmax + 1; r < kT; ++r) for (int c = 0; c < kTS; ++c) In[r * kTS + c] = 0.0;
        hipMemcpy(din, In.data(), N * 8, hipMemcpyHostToDevice);
        std::vector<double> T0(N), X0(N), T1(N), X1(N); int f0, f1;
        for (int p = 0; p < 2; ++p) {
            probe<<<1, 64>>>(din, dT, dX, dfl, jmax, p);
            hipDeviceSynchronize();
            hipMemcpy(p ? T1.data() : T0.data(), dT, N * 8, hipMemcpyDeviceToHost);
            hipMemcpy(p ? X1.data() : X0.data(), dX, N * 8, hipMemcpyDeviceToHost);
            hipMemcpy(p ? &f1 : &f0, dfl, 4, hipMemcpyDeviceToHost);
        }
        double dt = 0, dx = 0; int nbt = 0, first = -1;
        for (int e = 0; e < N; ++e) {
            if (T0[e] != T1[e] && !(std::isnan(T0[e]) && std::isnan(T1[e]))) { ++nbt; if (first < 0) first = e; dt = fmax(dt, fabs(T0[e] - T1[e])); }
            if (X0[e] != X1[e] && !(std::isnan(X0[e]) && std::isnan(X1[e]))) dx = fmax(dx, fabs(X0[e] - X1[e]));
        }
        printf("jmax %d: fail %d/%d, T differs at %d (first r %d c %d: %g vs %g), max dT %g, max dX %g\n", jmax, f0, f1, nbt,
               first < 0 ? -1 : first / kTS, first < 0 ? -1 : first % kTS, first < 0 ? 0 : T0[first], first < 0 ? 0 : T1[first], dt, dx);
        bad |= nbt != 0 || dx != 0;
    }
    return bad;
}
