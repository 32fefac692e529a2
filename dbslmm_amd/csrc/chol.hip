// chol.hip -- per-LD-block fp64 solve of the joint DBSLMM system (included by plan.hip).
//
// Replaces the reference's PCGm/PCGv calls and the beta assembly of estBlock
// (scr/dbslmmfit.cpp:711-729 large+small, :758-764 small only).  Per block the joint matrix
//     M = [[Sigma_ss + I/(sigma_s n), Sigma_sl], [Sigma_ls, Sigma_ll]]    (m x m, m = m_s + m_l)
// is factored M = L L^T and beta = M^{-1} z / sqrt(n), z = [z_s; z_l].  Block elimination of M
// reproduces the reference's q = A^{-1} z_s, P = A^{-1} Sigma_sl, S = Sigma_ll - Sigma_ls P,
// beta_l = S^{-1}(z_l - Sigma_ls q)/sqrt n and beta_s = sigma_s(sqrt n z_s - n Sigma_sl beta_l
// - Sigma_ss(sqrt n q - n P beta_l)) exactly ("one joint solve").
//
// The forward substitution is folded into the factorisation: z is appended as row m of the
// (row-major, lower-triangular) block matrix, so the Cholesky of the bordered matrix leaves
// y = L^{-1} z in row m.  Only the backward substitution L^T x = y remains.
//
// Two paths in ONE launch (workgroups [0, n_large) take one large block each, the rest take 4
// small blocks, one per wave):
//   small (ld <= 64): one wave per block; the bordered (m+1) x m matrix lives in LDS; Crout
//                     column by column, wave-synchronous (no workgroup barriers).
//   large (ld > 64):  one 256-thread workgroup per block; right-looking blocked Cholesky on
//                     32 x 32 tiles in global memory (L2-resident): wave 0 factors the diagonal
//                     tile (Crout) and inverts it; the panel TRSM is a product with that inverse
//                     and the trailing update C -= L_I L_J^T, both on v_mfma_f64_16x16x4_f64
//                     from LDS-staged tiles.  The inverse of each diagonal tile is kept (in the
//                     tile's upper triangle) for the backward substitution.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chol {

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kT = 32;        // tile edge
constexpr int kTS = 34;       // LDS row stride for MFMA operand tiles (conflict-free 16x4 reads)
constexpr int kSmallLd = 64;  // small path: ld <= 64 (m <= 63)
constexpr int kSS = 65;       // LDS row stride of the small path

// LDS carve (doubles) of the large path
constexpr int kHdr = 2;
constexpr int kOffD = kHdr;
constexpr int kOffX = kOffD + kT * kTS;          // inverse of the diagonal tile
constexpr int kOffRed = kOffX + kT * kTS;        // 8 x 32 partial sums
constexpr int kOffV = kOffRed + 8 * kT;          // 32 (backward substitution vector)
constexpr int kOffStage = kOffV + kT;            // 4 waves x 2 tiles x 32 x 34
constexpr int kLargeDoubles = kOffStage + 4 * 2 * kT * kTS;
constexpr int kSmallDoubles = 4 * kSmallLd * kSS;
constexpr int kLdsDoubles = kLargeDoubles > kSmallDoubles ? kLargeDoubles : kSmallDoubles;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct BlockArgs {
    const int32_t* blk_row0;
    const int32_t* blk_m;
    const int32_t* blk_ms;
    const int32_t* blk_ld;
    const int64_t* blk_matoff;
    const int32_t* blk_id;
    const double* z_slot;
    const int32_t* slot_out;
    const double* rsd;
    double dshift;
    double inv_sqrt_n;
    double* beta_s;
    double* beta_l;
    int32_t* status;
};

__device__ __forceinline__ void scatter_beta(const BlockArgs& a, int b, int row0, int i, double x,
                                             bool fail) {
    const double v = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
    const int o = a.slot_out[row0 + i];
    if (o >= 0) a.beta_s[o] = v;
    else a.beta_l[-1 - o] = v;
}

__device__ __forceinline__ void report_status(const BlockArgs& a, int b, int row0, int m, int lane0,
                                              int stride, bool fail) {
    bool mono = false;
    for (int i = lane0; i < m; i += stride) mono |= !(a.rsd[row0 + i] < INFINITY);
    if (fail || mono) atomicMax(a.status + a.blk_id[b], mono ? 3 : 2);
}

// ------------------------------------------------------------------ small path: one wave
__device__ void small_block(const BlockArgs& a, const double* __restrict__ M, int b, double* L,
                            int lane) {
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ms = a.blk_ms[b], ld = a.blk_ld[b];
    const double* A = M + a.blk_matoff[b];
    // rows 0..m-1: lower triangle of M (+ d shift on small diagonal); row m: z
    for (int r = 0; r < m; ++r) {
        if (lane <= r) {
            double v = A[static_cast<int64_t>(r) * ld + lane];
            if (lane == r && r < ms) v += a.dshift;
            L[r * kSS + lane] = v;
        }
    }
    if (lane < m) L[m * kSS + lane] = a.z_slot[row0 + lane];
    wave_sync();
    bool fail = false;
    for (int j = 0; j < m; ++j) {
        double s = 0.0;
        if (lane >= j && lane <= m) {
            const double* lr = L + lane * kSS;
            const double* lj = L + j * kSS;
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
            int k = 0;
            for (; k + 4 <= j; k += 4) {
                a0 += lr[k] * lj[k];
                a1 += lr[k + 1] * lj[k + 1];
                a2 += lr[k + 2] * lj[k + 2];
                a3 += lr[k + 3] * lj[k + 3];
            }
            for (; k < j; ++k) a0 += lr[k] * lj[k];
            s = lr[j] - ((a0 + a1) + (a2 + a3));
        }
        const double djj = __shfl(s, j, kWave);
        fail |= !(djj > 0.0);
        const double dj = sqrt(djj);
        if (lane > j && lane <= m) L[lane * kSS + j] = s / dj;
        if (lane == j) L[j * kSS + j] = dj;
        wave_sync();
    }
    // backward substitution L^T x = y, y = row m
    double v = lane < m ? L[m * kSS + lane] : 0.0;
    for (int j = m - 1; j >= 0; --j) {
        const double xj = __shfl(v, j, kWave) / L[j * kSS + j];
        if (lane == j) v = xj;
        else if (lane < j) v -= L[j * kSS + lane] * xj;
    }
    if (lane < m) scatter_beta(a, b, row0, lane, v, fail);
    report_status(a, b, row0, m, lane, kWave, fail);
}

// ------------------------------------------------------------------ large path: one workgroup
// Stage a 32x32 tile (rows r0.., cols c0..) of the row-major block matrix into LDS (stride kTS).
__device__ __forceinline__ void stage_tile(double* W, const double* A, int ld, int r0, int c0, int lane) {
    for (int e = lane; e < kT * kT; e += kWave) {
        const int r = e >> 5, c = e & 31;
        W[r * kTS + c] = A[static_cast<int64_t>(r0 + r) * ld + c0 + c];
    }
}

// acc(2x2 subtiles of 16x16) += sign * P Q^T over K = 32, P/Q 32x32 in LDS (stride kTS).
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
// C/D: col = l & 15, row = (l >> 4) + 4 * reg.
__device__ __forceinline__ void mfma_tile(v4d (&acc)[2][2], const double* P, const double* Q,
                                          double sign, int lane) {
    const int ri = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < kT / 4; ++kk) {
        const int k = 4 * kk + kq;
        const double p0 = sign * P[ri * kTS + k];
        const double p1 = sign * P[(16 + ri) * kTS + k];
        const double q0 = Q[ri * kTS + k];
        const double q1 = Q[(16 + ri) * kTS + k];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p0, q1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(p1, q1, acc[1][1], 0, 0, 0);
    }
}

__device__ __forceinline__ void load_acc(v4d (&acc)[2][2], const double* A, int ld, int r0, int c0, int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                acc[si][sj][q] = A[static_cast<int64_t>(r0 + 16 * si + (lane >> 4) + 4 * q) * ld + c0 + 16 * sj + (lane & 15)];
}

__device__ __forceinline__ void store_acc(const v4d (&acc)[2][2], double* A, int ld, int r0, int c0, int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                A[static_cast<int64_t>(r0 + 16 * si + (lane >> 4) + 4 * q) * ld + c0 + 16 * sj + (lane & 15)] = acc[si][sj][q];
}

__device__ void large_block(const BlockArgs& a, double* __restrict__ M, double* __restrict__ y,
                            int b, double* lds) {
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ms = a.blk_ms[b], ld = a.blk_ld[b];
    double* A = M + a.blk_matoff[b];
    int* s_fail = reinterpret_cast<int*>(lds);
    double* D = lds + kOffD;
    double* X = lds + kOffX;
    double* red = lds + kOffRed;
    double* vv = lds + kOffV;
    double* WI = lds + kOffStage + wave * 2 * kT * kTS;
    double* WJ = WI + kT * kTS;
    const int Tm = (m + kT - 1) / kT;   // tiles holding SNP columns
    const int Tz = m / kT;              // tile holding the z row
    if (tid == 0) *s_fail = 0;
    for (int c = tid; c < m; c += 256) A[static_cast<int64_t>(m) * ld + c] = a.z_slot[row0 + c];
    __syncthreads();

    for (int kb = 0; kb < Tm; ++kb) {
        const int c0 = kT * kb;
        const int jmax = min(kT, m - c0);
        // (1) diagonal tile: Crout + inverse by wave 0
        if (wave == 0) {
            for (int e = lane; e < kT * kT; e += kWave) {
                const int r = e >> 5, c = e & 31;
                double v = 0.0;
                if (c <= r && c0 + r <= m) {
                    v = A[static_cast<int64_t>(c0 + r) * ld + c0 + c];
                    if (r == c && c0 + r < ms) v += a.dshift;
                }
                D[r * kTS + c] = v;
            }
            wave_sync();
            bool fail = false;
            for (int j = 0; j < jmax; ++j) {
                double s = 0.0;
                if (lane >= j && lane < kT) {
                    const double* lr = D + lane * kTS;
                    const double* lj = D + j * kTS;
                    double a0 = 0.0, a1 = 0.0;
                    int k = 0;
                    for (; k + 2 <= j; k += 2) { a0 += lr[k] * lj[k]; a1 += lr[k + 1] * lj[k + 1]; }
                    if (k < j) a0 += lr[k] * lj[k];
                    s = lr[j] - (a0 + a1);
                }
                const double djj = __shfl(s, j, kWave);
                fail |= !(djj > 0.0);
                const double dj = sqrt(djj);
                if (lane > j && lane < kT) D[lane * kTS + j] = s / dj;
                if (lane == j) D[j * kTS + j] = dj;
                wave_sync();
            }
            if (fail && lane == 0) *s_fail = 1;
            // X = D^{-1} (lower), identity beyond jmax; lane c owns column c
            if (lane < kT) {
                const int c = lane;
                for (int r = 0; r < kT; ++r) {
                    double v = 0.0;
                    if (r >= c) {
                        if (r < jmax) {
                            double s = (r == c) ? 1.0 : 0.0;
                            for (int k = c; k < r; ++k) s -= D[r * kTS + k] * X[k * kTS + c];
                            v = s / D[r * kTS + r];
                        } else {
                            v = (r == c) ? 1.0 : 0.0;
                        }
                    }
                    X[r * kTS + c] = v;
                }
            }
            wave_sync();
            // write back: lower = L, diagonal = 1/L_cc, upper (c > r) = X[c][r] (= X^T)
            for (int e = lane; e < kT * kT; e += kWave) {
                const int r = e >> 5, c = e & 31;
                if (c0 + r > m) continue;
                double v;
                if (c < r) v = D[r * kTS + c];
                else if (r < jmax) v = X[c * kTS + r];
                else continue;
                A[static_cast<int64_t>(c0 + r) * ld + c0 + c] = v;
            }
        }
        __syncthreads();
        if (*s_fail) break;
        // (2) panel: L_I = A_I X^T for tile rows I = kb+1 .. Tz
        for (int I = kb + 1 + wave; I <= Tz; I += 4) {
            stage_tile(WI, A, ld, kT * I, c0, lane);
            wave_sync();
            v4d acc[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
            mfma_tile(acc, WI, X, 1.0, lane);
            store_acc(acc, A, ld, kT * I, c0, lane);
            wave_sync();
        }
        __syncthreads();
        // (3) trailing update C_IJ -= L_I L_J^T, kb < J <= I <= Tz, J < Tm
        const int nJ = Tm - 1 - kb;
        if (nJ > 0) {
            const int tri = nJ * (nJ + 1) / 2;
            const int npairs = tri + (Tz == Tm ? nJ : 0);
            for (int p = wave; p < npairs; p += 4) {
                int I, J;
                if (p < tri) {
                    int i = static_cast<int>((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
                    while ((i + 1) * (i + 2) / 2 <= p) ++i;
                    while (i * (i + 1) / 2 > p) --i;
                    I = kb + 1 + i;
                    J = kb + 1 + (p - i * (i + 1) / 2);
                } else {
                    I = Tz;
                    J = kb + 1 + (p - tri);
                }
                stage_tile(WI, A, ld, kT * I, c0, lane);
                if (I != J) stage_tile(WJ, A, ld, kT * J, c0, lane);
                wave_sync();
                v4d acc[2][2];
                load_acc(acc, A, ld, kT * I, kT * J, lane);
                mfma_tile(acc, WI, I != J ? WJ : WI, -1.0, lane);
                store_acc(acc, A, ld, kT * I, kT * J, lane);
                wave_sync();
            }
        }
        __syncthreads();
    }
    const bool fail = *s_fail != 0;
    double* x = y + row0;
    if (!fail) {
        // backward substitution L^T x = y (y = row m of the factor), tile by tile
        for (int I = Tm - 1; I >= 0; --I) {
            const int c = tid & 31, g = tid >> 5;
            const int gc = kT * I + c;
            double s = 0.0;
            for (int r = kT * (I + 1) + g; r < m; r += 8) s += A[static_cast<int64_t>(r) * ld + gc] * x[r];
            red[g * kT + c] = s;
            __syncthreads();
            if (tid < kT) {
                const int jmax = min(kT, m - kT * I);
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q) acc += red[q * kT + tid];
                vv[tid] = tid < jmax ? A[static_cast<int64_t>(m) * ld + gc] - acc : 0.0;
                wave_sync();
                // x_c = sum_{k >= c} X[k][c] v_k ; X[k][c] stored at (c, k) of the diagonal tile
                double xc = 0.0;
                if (tid < jmax)
                    for (int k = tid; k < jmax; ++k) xc += A[static_cast<int64_t>(gc) * ld + kT * I + k] * vv[k];
                if (tid < jmax) x[gc] = xc;
            }
            __syncthreads();
        }
    }
    for (int i = tid; i < m; i += 256) scatter_beta(a, b, row0, i, fail ? 0.0 : x[i], fail);
    report_status(a, b, row0, m, tid, 256, fail);
}

}  // namespace chol

// One launch: workgroups [0, n_large) -> large blocks (order_large), the rest -> 4 small blocks
// each (order_small).  Dynamic LDS = chol::kLdsDoubles doubles.
extern "C" __global__ __launch_bounds__(256) void dbslmm_chol_solve(
    double* __restrict__ M, const int32_t* __restrict__ order_large, int32_t n_large,
    const int32_t* __restrict__ order_small, int32_t n_small,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ms, const int32_t* __restrict__ blk_ld,
    const int64_t* __restrict__ blk_matoff, const int32_t* __restrict__ blk_id,
    const double* __restrict__ z_slot, const int32_t* __restrict__ slot_out,
    const double* __restrict__ rsd, double dshift, double inv_sqrt_n, double* __restrict__ y,
    double* __restrict__ beta_s, double* __restrict__ beta_l, int32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const chol::BlockArgs a{blk_row0, blk_m, blk_ms, blk_ld, blk_matoff, blk_id, z_slot, slot_out,
                            rsd, dshift, inv_sqrt_n, beta_s, beta_l, status};
    if (static_cast<int>(blockIdx.x) < n_large) {
        chol::large_block(a, M, y, order_large[blockIdx.x], lds);
        return;
    }
    const int wave = threadIdx.x / chol::kWave, lane = threadIdx.x & (chol::kWave - 1);
    const int idx = (static_cast<int>(blockIdx.x) - n_large) * 4 + wave;
    if (idx >= n_small) return;      // whole wave leaves; the small path has no workgroup barrier
    chol::small_block(a, M, order_small[idx], lds + wave * chol::kSmallLd * chol::kSS, lane);
}
