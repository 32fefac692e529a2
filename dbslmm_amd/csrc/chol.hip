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
// Two kernels, launched concurrently on two streams:
//   dbslmm_chol_small (ld <= 64, m <= 63): one wave per block; the bordered matrix lives in LDS
//       as a packed lower triangle; Crout column by column, wave-synchronous (no barriers).
//   dbslmm_chol_large (ld > 64): one 512-thread workgroup per block; right-looking blocked
//       Cholesky on 32 x 32 tiles of the block matrix in global memory (L2-resident).  Wave 0
//       factors and inverts the diagonal tile; the panel TRSM (product with that inverse) and
//       the trailing update C -= L_I L_J^T run on v_mfma_f64_16x16x4_f64 with the panel kept
//       in LDS.  The inverse of each diagonal tile is kept (in the tile's upper triangle) for
//       the backward substitution.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace chol {

typedef double v4d __attribute__((ext_vector_type(4)));
typedef double v2d __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr int kT = 32;          // tile edge
constexpr int kTS = 34;         // LDS row stride of MFMA operand tiles (conflict-free 16x4 reads)
constexpr int kSmallLd = 64;    // small path: ld <= 64 (m <= 63)
constexpr int kSmallWaves = 2;  // small kernel: 2 waves (blocks) per workgroup
constexpr int kSmallTri = kSmallLd * (kSmallLd + 1) / 2;   // packed bordered triangle
constexpr int kSmallDoublesPerWave = kSmallTri + kSmallLd;  // + reciprocal pivots
constexpr int kLargeThreads = 256;
constexpr int kLargeWaves = kLargeThreads / kWave;

// LDS carve (doubles) of the large kernel
constexpr int kPanelMax = 16;                    // panel tiles kept resident
constexpr int kTileD = kT * kTS;                 // one 32x32 tile, stride 34
constexpr int kOffX = 2;                         // [0,2): flags; X = inverse of the diagonal tile
constexpr int kOffCol = kOffX + kTileD;          // broadcast column buffer (32) + pivots (32)
constexpr int kOffRed = kOffCol + 2 * kT;        // 16 x 32 partial sums
constexpr int kOffLb = kOffRed + 16 * kT;        // diagonal tile being factored (red: <= 16 x 32)
constexpr int kOffPanel = kOffLb + kTileD;       // kPanelMax tiles (also the x / v vector)
constexpr int kLargeDoubles = kOffPanel + kPanelMax * kTileD;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(bits), lane);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), lane);
    return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// 1/sqrt(p) to full fp64 accuracy: v_rsq_f64 + one Newton step
__device__ __forceinline__ double rsqrt_f64(double p) {
    double rs = __builtin_amdgcn_rsq(p);
    return rs * (1.5 - 0.5 * p * rs * rs);
}

#ifdef DBSLMM_STAMPS
// diagnostic build only: accumulated 100 MHz ticks per phase of the large path
__device__ unsigned long long g_stamp[16];
#define STAMP_DECL unsigned long long st_t0 = 0; int st_base = 0;
#define STAMP_BEGIN() do { if (threadIdx.x == 0) st_t0 = __builtin_amdgcn_s_memrealtime(); } while (0)
#define STAMP_END(k) do { if (threadIdx.x == 0) atomicAdd(&g_stamp[(k) + st_base], __builtin_amdgcn_s_memrealtime() - st_t0); } while (0)
#define FSTAMP(k) do { if (lane == 0) { unsigned long long t_ = __builtin_amdgcn_s_memrealtime(); atomicAdd(&g_stamp[k], t_ - fst); fst = t_; } } while (0)
#define FSTAMP_DECL unsigned long long fst = __builtin_amdgcn_s_memrealtime();
#else
#define FSTAMP(k) do {} while (0)
#define FSTAMP_DECL
#define STAMP_DECL
#define STAMP_BEGIN() do {} while (0)
#define STAMP_END(k) do {} while (0)
#endif

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

__device__ __forceinline__ void scatter_beta(const BlockArgs& a, int row0, int i, double x, bool fail) {
    const double v = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
    const int o = a.slot_out[row0 + i];
    if (o >= 0) a.beta_s[o] = v;
    else a.beta_l[-1 - o] = v;
}

__device__ __forceinline__ void report_status(const BlockArgs& a, int b, int row0, int m, int i0,
                                              int stride, bool fail) {
    bool mono = false;
    for (int i = i0; i < m; i += stride) mono |= !(a.rsd[row0 + i] < INFINITY);
    if (fail || mono) atomicMax(a.status + a.blk_id[b], mono ? 3 : 2);
}

// ================================================================== small path: one wave
// Packed bordered lower triangle: element (r, k <= r) at r(r+1)/2 + k, rows 0..m (row m = z).
__device__ __forceinline__ int tri(int r) { return r * (r + 1) / 2; }

__device__ void small_block(const BlockArgs& a, double* __restrict__ M, int b, double* L,
                            double* rdg, int lane) {
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ms = a.blk_ms[b], ld = a.blk_ld[b];
    double* A = M + a.blk_matoff[b];
    for (int r = 0; r < m; ++r) {
        if (lane <= r) {
            double v = A[static_cast<int64_t>(r) * ld + lane];
            if (lane == r && r < ms) v += a.dshift;
            L[tri(r) + lane] = v;
        }
    }
    if (lane < m) L[tri(m) + lane] = a.z_slot[row0 + lane];
    wave_sync();
    bool fail = false;
    const int my = tri(lane);
    for (int j = 0; j < m; ++j) {
        double s = 0.0;
        if (lane >= j && lane <= m) {
            const double* lr = L + my;
            const double* lj = L + tri(j);
            double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, a4 = 0.0, a5 = 0.0, a6 = 0.0, a7 = 0.0;
            int k = 0;
            for (; k + 8 <= j; k += 8) {
                a0 += lr[k] * lj[k];
                a1 += lr[k + 1] * lj[k + 1];
                a2 += lr[k + 2] * lj[k + 2];
                a3 += lr[k + 3] * lj[k + 3];
                a4 += lr[k + 4] * lj[k + 4];
                a5 += lr[k + 5] * lj[k + 5];
                a6 += lr[k + 6] * lj[k + 6];
                a7 += lr[k + 7] * lj[k + 7];
            }
            for (; k < j; ++k) a0 += lr[k] * lj[k];
            s = lr[j] - (((a0 + a1) + (a2 + a3)) + ((a4 + a5) + (a6 + a7)));
        }
        const double p = __shfl(s, j, kWave);
        fail |= !(p > 0.0);
        const double rs = rsqrt_f64(p);
        if (lane > j && lane <= m) L[my + j] = s * rs;
        if (lane == j) { L[my + j] = p * rs; rdg[j] = rs; }
        wave_sync();
    }
    // L back to global (strict lower = L, diagonal = 1/L_jj, the convention of the other solve
    // paths; read by dbslmm_variance)
    for (int r = 0; r < m; ++r)
        if (lane <= r) A[static_cast<int64_t>(r) * ld + lane] = lane == r ? rdg[r] : L[tri(r) + lane];
    // backward substitution L^T x = y, y = row m
    double v = lane < m ? L[tri(m) + lane] : 0.0;
    for (int j = m - 1; j >= 0; --j) {
        const double xj = __shfl(v, j, kWave) * rdg[j];
        const double lj = lane < j ? L[tri(j) + lane] : 0.0;
        if (lane == j) v = xj;
        else if (lane < j) v -= lj * xj;
    }
    if (lane < m) scatter_beta(a, row0, lane, v, fail);
    report_status(a, b, row0, m, lane, kWave, fail);
}

// ================================================================== large path helpers
// Stage a 32x32 tile (rows r0.., cols c0..) of the row-major block matrix into LDS (stride kTS).
__device__ __forceinline__ void stage_tile(double* W, const double* A, int ld, int r0, int c0, int lane) {
    double v[kT * kT / kWave];
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {   // all 16 loads in flight before any write
        const int e = it * kWave + lane;
        v[it] = A[static_cast<int64_t>(r0 + (e >> 5)) * ld + c0 + (e & 31)];
    }
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {
        const int e = it * kWave + lane;
        W[(e >> 5) * kTS + (e & 31)] = v[it];
    }
}

// acc(2x2 subtiles of 16x16) += sign * P Q^T over K = 32, P/Q 32x32 in LDS (stride kTS).
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][k=l>>4], B[k=l>>4][l&15];
// C/D: col = l & 15, row = (l >> 4) + 4 * reg.
__device__ __forceinline__ void mfma_tile(v4d (&acc)[2][2], const double* P, const double* Q,
                                          double sign, int lane) {
    const int ri = lane & 15, kq = lane >> 4;
    // all 32 operand reads first (one LDS latency for the whole tile), then 32 MFMAs
    double p0[kT / 4], p1[kT / 4], q0[kT / 4], q1[kT / 4];
#pragma unroll
    for (int kk = 0; kk < kT / 4; ++kk) {
        const int k = 4 * kk + kq;
        p0[kk] = P[ri * kTS + k];
        p1[kk] = P[(16 + ri) * kTS + k];
        q0[kk] = Q[ri * kTS + k];
        q1[kk] = Q[(16 + ri) * kTS + k];
    }
#pragma unroll
    for (int kk = 0; kk < kT / 4; ++kk) {
        const double a0 = sign * p0[kk], a1 = sign * p1[kk];
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q0[kk], acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, q1[kk], acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, q0[kk], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, q1[kk], acc[1][1], 0, 0, 0);
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

__device__ __forceinline__ void acc_to_lds(const v4d (&acc)[2][2], double* W, int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                W[(16 * si + (lane >> 4) + 4 * q) * kTS + 16 * sj + (lane & 15)] = acc[si][sj][q];
}

// Wave 0: factor the diagonal tile (c0, c0) and invert it, in one pass.
//   Coalesced load into Lb (LDS).  Lane r < 32 keeps ROW r of the tile in v[] and factors it
//   right-looking; lane 32 + c keeps COLUMN c of X = L^{-1} (initially e_c) and runs the
//   column-oriented forward substitution of L X = I alongside.  Both halves apply the same
//   instructions per column j: pivot p = L_jj^2 from lane j (readlane), rs = 1/sqrt(p) (rsq +
//   Newton), v[j] *= rs, then v[i] -= v[j] * L[i][j] for i > j with column j of L broadcast
//   from LDS (written once by the row lanes, read back as ds_read_b128 broadcasts).  So the
//   inverse costs no extra passes.  X is published to Xl (LDS) and the tile is written back:
//   lower = L, diagonal + upper (r, c >= r) = X[c][r].  Returns true on a non-positive pivot.
__device__ __forceinline__ bool factor_diag(double* A, int ld, int c0, int m, int ms, double dshift,
                                            double* Xl, double* Lb, double* colb, int lane,
                                            bool from_lds) {
    FSTAMP_DECL
    const int r = lane & 31;
    const bool xlane = lane >= kT;       // lanes 32..63: columns of X
    const int jmax = min(kT, m - c0);
    // tile -> Lb: from global (coalesced), or already in Lb (lookahead: the updating wave put it
    // there); keep the lower triangle of rows <= m, add 1/(sigma_s n) on the small diagonal
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {
        const int e = it * kWave + lane;
        const int rr = e >> 5, cc = e & 31;
        double v = 0.0;
        if (cc <= rr && c0 + rr <= m)
            v = from_lds ? Lb[rr * kTS + cc] : A[static_cast<int64_t>(c0 + rr) * ld + c0 + cc];
        if (cc == rr && c0 + rr < ms) v += dshift;
        Lb[rr * kTS + cc] = v;
    }
    wave_sync();
    double v[kT];
#pragma unroll
    for (int c = 0; c < kT; ++c) v[c] = xlane ? (c == r ? 1.0 : 0.0) : Lb[r * kTS + c];
    FSTAMP(4);
    bool fail = false;
    double* rdl = colb + kT;           // reciprocal pivots (LDS, 32)
#pragma unroll
    for (int j = 0; j < kT; ++j) {
        if (j < jmax) {
            const double p = readlane_f64(v[j], j);
            fail |= !(p > 0.0);
            const double rs = rsqrt_f64(p);
            v[j] = (!xlane && r < j) ? 0.0 : v[j] * rs;    // row lanes: L[r][j]; X lanes: x[j]
            if (!xlane) {
                colb[r] = v[j];
                Lb[r * kTS + j] = v[j];
            }
            if (lane == 0) rdl[j] = rs;
            wave_sync();
#pragma unroll
            for (int k0 = (j + 1) & ~7; k0 < kT; k0 += 8) {   // broadcast reads, 8 at a time
                double col[8];
#pragma unroll
                for (int k = 0; k < 8; k += 2) {
                    const v2d t = *reinterpret_cast<const v2d*>(colb + k0 + k);
                    col[k] = t[0];
                    col[k + 1] = t[1];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k0 + k > j) v[k0 + k] -= v[j] * col[k];
            }
            wave_sync();
        }
    }
    FSTAMP(5);
    // X columns beyond jmax are identity rows / columns (never used beyond the tile's SNPs)
    if (xlane) {
#pragma unroll
        for (int q = 0; q < kT; ++q) {
            if (q >= jmax) v[q] = (q == r) ? 1.0 : 0.0;
            Xl[q * kTS + r] = v[q];
        }
    }
    wave_sync();
    FSTAMP(6);
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {
        const int e = it * kWave + lane;
        const int rr = e >> 5, cc = e & 31;
        if (c0 + rr > m) continue;
        if (cc < rr) {
            if (cc < jmax) A[static_cast<int64_t>(c0 + rr) * ld + c0 + cc] = Lb[rr * kTS + cc];
        } else if (rr < jmax) {
            A[static_cast<int64_t>(c0 + rr) * ld + c0 + cc] = Xl[cc * kTS + rr];
        }
    }
    FSTAMP(7);
    return fail;
}

__device__ __forceinline__ void decode_pair(int p, int tri_n, int kb, int Tz, int& I, int& J) {
    if (p < tri_n) {
        int i = static_cast<int>((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= p) ++i;
        while (i * (i + 1) / 2 > p) --i;
        I = kb + 1 + i;
        J = kb + 1 + (p - i * (i + 1) / 2);
    } else {
        I = Tz;
        J = kb + 1 + (p - tri_n);
    }
}

__device__ void large_block(const BlockArgs& a, double* __restrict__ M, double* __restrict__ y,
                            int b, double* lds) {
    constexpr int NT = kLargeThreads, NW = kLargeWaves;
    const int tid = threadIdx.x, lane = tid & (kWave - 1), wave = tid / kWave;
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ms = a.blk_ms[b], ld = a.blk_ld[b];
    double* A = M + a.blk_matoff[b];
    int* s_fail = reinterpret_cast<int*>(lds);
    double* Xl = lds + kOffX;
    double* colb = lds + kOffCol;
    double* red = lds + kOffRed;
    double* Lb = lds + kOffLb;
    double* panel = lds + kOffPanel;
    const int Tm = (m + kT - 1) / kT;   // tiles holding SNP columns
    const int Tz = m / kT;              // tile holding the z row
    STAMP_DECL
    if (tid == 0) *s_fail = 0;
    for (int c = tid; c < m; c += NT) A[static_cast<int64_t>(m) * ld + c] = a.z_slot[row0 + c];
    __syncthreads();

    int* s_next = s_fail + 1;   // dynamic pair counter of the trailing update
    // diagonal tile 0; every later diagonal tile is factored by lookahead inside the previous
    // step's trailing update (wave 0 updates it first, then factors it while the other waves
    // finish the remaining pairs)
    STAMP_BEGIN();
    if (wave == 0) {
        const bool f = factor_diag(A, ld, 0, m, ms, a.dshift, Xl, Lb, colb, lane, false);
        if (f && lane == 0) *s_fail = 1;
    }
    __syncthreads();
    STAMP_END(0);
    for (int kb = 0; kb < Tm; ++kb) {
        if (*s_fail) break;
        const int c0 = kT * kb;
        STAMP_BEGIN();
        // (2) panel: L_I = A_I X^T for tile rows I = kb+1 .. Tz; kept in LDS when they fit
        const int P = Tz - kb;
        const bool fits = P <= kPanelMax;
        for (int I = kb + 1 + wave; I <= Tz; I += NW) {
            double* W = fits ? panel + (I - kb - 1) * kTileD : panel + 2 * wave * kTileD;
            stage_tile(W, A, ld, kT * I, c0, lane);
            wave_sync();
            v4d acc[2][2] = {{{0, 0, 0, 0}, {0, 0, 0, 0}}, {{0, 0, 0, 0}, {0, 0, 0, 0}}};
            mfma_tile(acc, W, Xl, 1.0, lane);
            store_acc(acc, A, ld, kT * I, c0, lane);
            wave_sync();
            if (fits) acc_to_lds(acc, W, lane);
        }
        if (tid == 0) *s_next = 1;
        __syncthreads();
        STAMP_END(1);
        STAMP_BEGIN();
        // (3) trailing update C_IJ -= L_I L_J^T, kb < J <= I <= Tz, J < Tm.  Pair 0 is the next
        //     diagonal tile (kb+1, kb+1): wave 0 updates it into LDS and factors it (lookahead);
        //     pairs 1.. are handed out dynamically; the next pair's C tile is prefetched.
        const int nJ = Tm - 1 - kb;
        if (nJ > 0) {
            const int tri_n = nJ * (nJ + 1) / 2;
            const int npairs = tri_n + (Tz == Tm ? nJ : 0);
            auto tile_ptr = [&](int I, double* stage_slot) -> const double* {
                if (fits) return panel + (I - kb - 1) * kTileD;
                stage_tile(stage_slot, A, ld, kT * I, c0, lane);
                return stage_slot;
            };
            if (wave == 0) {
                const int d0 = kT * (kb + 1);
                v4d acc[2][2];
                load_acc(acc, A, ld, d0, d0, lane);
                const double* LI = tile_ptr(kb + 1, panel + 0 * kTileD);
                wave_sync();
                mfma_tile(acc, LI, LI, -1.0, lane);
                wave_sync();
                acc_to_lds(acc, Lb, lane);
                wave_sync();
                const bool f = factor_diag(A, ld, d0, m, ms, a.dshift, Xl, Lb, colb, lane, true);
                if (f && lane == 0) *s_fail = 1;
            }
            auto grab = [&]() -> int {
                int q = 0;
                if (lane == 0) q = atomicAdd(s_next, 1);
                return __shfl(q, 0, kWave);
            };
            int p = grab(), I = 0, J = 0;
            v4d cur[2][2], nxt[2][2];
            if (p < npairs) {
                decode_pair(p, tri_n, kb, Tz, I, J);
                load_acc(cur, A, ld, kT * I, kT * J, lane);
            }
            while (p < npairs) {
                const int pn = grab();
                int In = 0, Jn = 0;
                if (pn < npairs) {
                    decode_pair(pn, tri_n, kb, Tz, In, Jn);
                    load_acc(nxt, A, ld, kT * In, kT * Jn, lane);
                }
                double* WI = panel + 2 * wave * kTileD;
                const double* LI = tile_ptr(I, WI);
                const double* LJ = (I == J) ? LI : tile_ptr(J, WI + kTileD);
                if (!fits) wave_sync();
                mfma_tile(cur, LI, LJ, -1.0, lane);
                store_acc(cur, A, ld, kT * I, kT * J, lane);
                if (!fits) wave_sync();
#pragma unroll
                for (int si = 0; si < 2; ++si)
#pragma unroll
                    for (int sj = 0; sj < 2; ++sj) cur[si][sj] = nxt[si][sj];
                I = In;
                J = Jn;
                p = pn;
            }
        }
        __syncthreads();
        STAMP_END(2);
    }
    STAMP_BEGIN();
    const bool fail = *s_fail != 0;
    double* v = panel;   // v / x vector
    if (m > kPanelMax * kTileD) v = y + row0;
    if (!fail) {
        // backward substitution L^T x = y, right-looking over tile rows J = Tm-1 .. 0.
        // Per step: the strip L[c1.., 0..c1) is loaded into registers up front (overlapping the
        // x_J reduction), the next diagonal tile is prefetched, x_J = X_JJ^T v_J comes from an
        // LDS copy of the stored inverse.
        constexpr int NG = NT / kT;                        // thread groups of 32
        double* D = Lb;                                    // diagonal tile (stride kTS)
        for (int c = tid; c < m; c += NT) v[c] = A[static_cast<int64_t>(m) * ld + c];
        double dg[kT * kT / NT];
        auto load_diag = [&](int J) {
            const int c1 = kT * J, jm = min(kT, m - c1);
#pragma unroll
            for (int it = 0; it < kT * kT / NT; ++it) {
                const int e = it * NT + tid, rr = e >> 5, cc = e & 31;
                dg[it] = (cc >= rr && cc < jm) ? A[static_cast<int64_t>(c1 + rr) * ld + c1 + cc] : 0.0;
            }
        };
        load_diag(Tm - 1);
        for (int J = Tm - 1; J >= 0; --J) {
            const int c1 = kT * J;
            const int jmax = min(kT, m - c1);
            // strip loads for this step (2 columns per thread at most: m < 16 * kTileD)
            double l0[kT], l1[kT];
            const int col0 = tid, col1 = tid + NT;
#pragma unroll
            for (int r = 0; r < kT; ++r) {
                l0[r] = (col0 < c1 && r < jmax) ? A[static_cast<int64_t>(c1 + r) * ld + col0] : 0.0;
                l1[r] = (col1 < c1 && r < jmax) ? A[static_cast<int64_t>(c1 + r) * ld + col1] : 0.0;
            }
#pragma unroll
            for (int it = 0; it < kT * kT / NT; ++it) {
                const int e = it * NT + tid;
                D[(e >> 5) * kTS + (e & 31)] = dg[it];
            }
            __syncthreads();
            if (J > 0) load_diag(J - 1);
            {   // x_J = X_JJ^T v_J: stored (c, k >= c) = X[k][c]
                const int c = tid & 31, g = tid >> 5;
                double sx = 0.0;
                for (int k = c + g; k < jmax; k += NG) sx += D[c * kTS + k] * v[c1 + k];
                red[g * kT + c] = sx;
            }
            __syncthreads();
            if (tid < jmax) {
                double sx = 0.0;
#pragma unroll
                for (int q = 0; q < NG; ++q) sx += red[q * kT + tid];
                v[c1 + tid] = sx;
            }
            __syncthreads();
            // v[col] -= sum_r L[c1 + r][col] x[r] for col < c1
            double s0 = 0.0, s1 = 0.0, t0 = 0.0, t1 = 0.0;
#pragma unroll
            for (int r = 0; r < kT; r += 2) {
                const double x0 = r < jmax ? v[c1 + r] : 0.0, x1 = r + 1 < jmax ? v[c1 + r + 1] : 0.0;
                s0 += l0[r] * x0;
                s1 += l0[r + 1] * x1;
                t0 += l1[r] * x0;
                t1 += l1[r + 1] * x1;
            }
            if (col0 < c1) v[col0] -= s0 + s1;
            if (col1 < c1) v[col1] -= t0 + t1;
            for (int col = tid + 2 * NT; col < c1; col += NT) {      // m > 512: generic tail
                double sg = 0.0;
                for (int r = 0; r < jmax; ++r) sg += A[static_cast<int64_t>(c1 + r) * ld + col] * v[c1 + r];
                v[col] -= sg;
            }
            __syncthreads();
        }
    }
    STAMP_END(3);
    // x = M^{-1} z also into the copy's slot vector: the start of the Chebyshev h2f copies
    // (dbslmm_chol_cheb) when this is the base copy
    if (v != y + row0)
        for (int i = tid; i < m; i += NT) y[row0 + i] = fail ? 0.0 : v[i];
    for (int i = tid; i < m; i += NT) scatter_beta(a, row0, i, fail ? 0.0 : v[i], fail);
    report_status(a, b, row0, m, tid, NT, fail);
}

// ---------------------------------------------------------------- h2f copies by Chebyshev
// The single-workgroup blocks (ld > 64) take part in the h2f Chebyshev iteration of trsv.hip too:
// only the base copy is factored (dbslmm_chol_large), every other copy c iterates
// M_b x = z - delta_c P_s x with the base factor as the preconditioner (the recurrence and the
// coefficients of trsv.hip / cheb_plan: d = alpha d + beta M_b^{-1} r, s = alpha s + beta r,
// x += d, r -= s + delta P_s d; start x = x_b, r = -delta P_s x_b).  One workgroup per block: the
// vectors of up to kChebR copies live in LDS; per iteration a forward substitution (right-looking
// over the 32-row tiles: y_J = X_JJ v_J with the stored inverse, then the strip below it) and a
// backward one (as large_block's), each reading the factor's lower triangle once.  The factor of
// two more copies (2 m^3 / 3 flops, the whole matrix written twice) becomes ~16 triangular
// passes (~8 m^2 flops) with far less LDS per workgroup, so several blocks share a CU.
constexpr int kChebR = 2;                           // copies per launch group (trsv::kMaxR)
constexpr int kChebMaxM = 512;                      // ld > 64 blocks are below the tiled threshold
constexpr int kChebThreads = 512;                   // one strip row / column per thread (m <= 512)
constexpr int kChebLdsDoubles = 5 * kChebR * kChebMaxM + kTileD + kChebR * (kChebThreads / kT) * kT;

// CG instead (dbslmm_options.h2f_iter, the default; trsv.hip dbslmm_cg_update): the same passes,
// then gamma = r.z, zeta = |P_s z|^2, the Chronopoulos-Gear scalars and the update of p (Dv),
// q = M_c p (Sv), x, r; the block stops once every copy has |r| <= tol lambda_min(M_c) |x|
// (lambda_min >= fs[q] = d_c + 1 - tau without large SNPs, fl = 1 - tau with), `iters` the cap.
struct CgStop {
    int32_t on;
    double fs[kChebR];
    double fl;
    double tol;
};
// totals of v[0..4) over the workgroup (8 waves), fixed order: every thread gets the same values
__device__ __forceinline__ void cg_sum4(double (&v)[4], double* red, int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int sft = 32; sft >= 1; sft >>= 1) v[j] += __shfl_xor(v[j], sft);
    if ((tid & 63) == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(tid >> 6) * 4 + j] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double t = 0.0;
        for (int w = 0; w < kChebThreads / 64; ++w) t += red[w * 4 + j];
        v[j] = t;
    }
    __syncthreads();
}

// Returns (CG) the copies still above their bound when the cap ended the loop: bit q = copy q.
__device__ uint32_t cheb_block(const double* __restrict__ A, int ld, int m, int ms, int nr, int iters,
                               const double* __restrict__ coef, double* lds, const CgStop& cgs) {
    constexpr int NT = kChebThreads, NG = NT / kT;
    const int tid = threadIdx.x;
    double* X = lds;                                 // [kChebR][kChebMaxM] each
    double* R = X + kChebR * kChebMaxM;
    double* Dv = R + kChebR * kChebMaxM;
    double* Sv = Dv + kChebR * kChebMaxM;
    double* V = Sv + kChebR * kChebMaxM;             // work vector: r -> y -> z
    double* Dt = V + kChebR * kChebMaxM;             // diagonal tile, stride kTS
    double* red = Dt + kTileD;                       // [kChebR][NG][32] partial sums
    const int T = (m + kT - 1) / kT;
    double gp[kChebR] = {0.0, 0.0}, ap[kChebR] = {0.0, 0.0};   // CG: gamma, alpha of the previous iteration
    uint32_t open = 0;                                   // CG: copies above their bound after the last update
    for (int k = 0; k < iters; ++k) {
        for (int e = tid; e < nr * kChebMaxM; e += NT) V[e] = R[e];
        __syncthreads();
        // forward L y = r: right-looking over the tiles.  Per tile, the diagonal block and the
        // strip below it (rows i0 = c1 + 32 + tid and i0 + 256: m <= 512) are loaded together up
        // front, so a tile step waits for one round of loads
        for (int J = 0; J < T; ++J) {
            const int c1 = kT * J, jmax = min(kT, m - c1);
            v2d l0[kT / 2];
            const int i0 = c1 + kT + tid;                 // m <= 512: one row per thread
#pragma unroll
            for (int c = 0; c < kT / 2; ++c)
                l0[c] = i0 < m ? reinterpret_cast<const v2d*>(A + static_cast<int64_t>(i0) * ld + c1)[c] : v2d{0.0, 0.0};
            for (int e = tid; e < kT * kT; e += NT) {
                const int rr = e >> 5, cc = e & 31;   // stored (rr, cc >= rr) = X[cc][rr]
                Dt[rr * kTS + cc] = (cc >= rr && cc < jmax) ? A[static_cast<int64_t>(c1 + rr) * ld + c1 + cc] : 0.0;
            }
            __syncthreads();
            {   // y_J[kk] = sum_{c <= kk} X[kk][c] v[c1 + c]
                const int kk = tid & 31, g = tid >> 5;
                for (int q = 0; q < nr; ++q) {
                    double sx = 0.0;
                    for (int c = g; c <= kk && c < jmax; c += NG) sx += Dt[c * kTS + kk] * V[q * kChebMaxM + c1 + c];
                    red[(q * NG + g) * kT + kk] = sx;
                }
            }
            __syncthreads();
            if (tid < kT * nr) {
                const int kk = tid & 31, q = tid >> 5;
                double sx = 0.0;
#pragma unroll
                for (int g = 0; g < NG; ++g) sx += red[(q * NG + g) * kT + kk];
                if (kk < jmax) V[q * kChebMaxM + c1 + kk] = sx;
            }
            __syncthreads();
            // v_i -= L[i][c1 ..] y_J for the rows below the tile
            if (i0 < m) {
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int c = 0; c < kT; ++c) {
                    const double y0 = c < jmax ? V[c1 + c] : 0.0;
                    const double y1 = (nr > 1 && c < jmax) ? V[kChebMaxM + c1 + c] : 0.0;
                    s0 += l0[c >> 1][c & 1] * y0;
                    s1 += l0[c >> 1][c & 1] * y1;
                }
                V[i0] -= s0;
                if (nr > 1) V[kChebMaxM + i0] -= s1;
            }
            __syncthreads();
        }
        // backward L^T z = y, right-looking over J = T-1 .. 0 (as large_block); the strip
        // L[c1 + r][col], col < c1 (columns tid and tid + 256), loaded with the diagonal block
        for (int J = T - 1; J >= 0; --J) {
            const int c1 = kT * J, jmax = min(kT, m - c1);
            double l0[kT];
            const int col0 = tid;                          // c1 < 512: one column per thread
#pragma unroll
            for (int r = 0; r < kT; ++r)
                l0[r] = (col0 < c1 && r < jmax) ? A[static_cast<int64_t>(c1 + r) * ld + col0] : 0.0;
            for (int e = tid; e < kT * kT; e += NT) {
                const int rr = e >> 5, cc = e & 31;
                Dt[rr * kTS + cc] = (cc >= rr && cc < jmax) ? A[static_cast<int64_t>(c1 + rr) * ld + c1 + cc] : 0.0;
            }
            __syncthreads();
            {   // x_J[c] = sum_{kk >= c} X[kk][c] v[c1 + kk]
                const int c = tid & 31, g = tid >> 5;
                for (int q = 0; q < nr; ++q) {
                    double sx = 0.0;
                    for (int kk = c + g; kk < jmax; kk += NG) sx += Dt[c * kTS + kk] * V[q * kChebMaxM + c1 + kk];
                    red[(q * NG + g) * kT + c] = sx;
                }
            }
            __syncthreads();
            if (tid < kT * nr) {
                const int c = tid & 31, q = tid >> 5;
                double sx = 0.0;
#pragma unroll
                for (int g = 0; g < NG; ++g) sx += red[(q * NG + g) * kT + c];
                if (c < jmax) V[q * kChebMaxM + c1 + c] = sx;
            }
            __syncthreads();
            // v[col] -= sum_r L[c1 + r][col] x[r] for col < c1
            if (col0 < c1) {
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int r = 0; r < kT; ++r) {
                    const double x0 = r < jmax ? V[c1 + r] : 0.0;
                    const double x1 = (nr > 1 && r < jmax) ? V[kChebMaxM + c1 + r] : 0.0;
                    s0 += l0[r] * x0;
                    s1 += l0[r] * x1;
                }
                V[col0] -= s0;
                if (nr > 1) V[kChebMaxM + col0] -= s1;
            }
            __syncthreads();
        }
        if (cgs.on) {   // CG update (V = z = M_b^{-1} r)
            static_assert(kChebMaxM == NT, "one element per thread and copy");
            const int i = tid;
            double v[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < kChebR; ++q)
                if (q < nr && i < m) {
                    const int e = q * kChebMaxM + i;
                    const double z = V[e];
                    v[2 * q] += R[e] * z;
                    if (i < ms) v[2 * q + 1] += z * z;
                }
            cg_sum4(v, red, tid);
            double al[kChebR], be[kChebR];
#pragma unroll
            for (int q = 0; q < kChebR; ++q) {
                const double gam = v[2 * q], eta = gam + coef[3 * q + 2] * v[2 * q + 1];
                be[q] = 0.0;
                double den = eta;
                if (k > 0) {
                    be[q] = gp[q] > 0.0 ? gam / gp[q] : 0.0;
                    den = eta - (ap[q] != 0.0 ? be[q] * gam / ap[q] : 0.0);
                }
                al[q] = den > 0.0 && gam > 0.0 ? gam / den : 0.0;
                gp[q] = gam;
                ap[q] = al[q];
            }
            double w[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int q = 0; q < kChebR; ++q) {
                if (q >= nr || i >= m) continue;
                const int e = q * kChebMaxM + i;
                const double z = V[e], r = R[e];
                const double pv = z + be[q] * Dv[e];
                const double qv = r + (i < ms ? coef[3 * q + 2] * z : 0.0) + be[q] * Sv[e];
                const double x = X[e] + al[q] * pv;
                const double rn = r - al[q] * qv;
                Dv[e] = pv;
                Sv[e] = qv;
                X[e] = x;
                R[e] = rn;
                w[2 * q] += rn * rn;
                w[2 * q + 1] += x * x;
            }
            cg_sum4(w, red, tid);
            open = 0;
#pragma unroll
            for (int q = 0; q < kChebR; ++q) {
                const double t = cgs.tol * (ms == m ? cgs.fs[q] : cgs.fl);
                if (q < nr && !(w[2 * q] <= t * t * w[2 * q + 1])) open |= 1u << q;   // NaN: not converged
            }
            if (!open) break;   // uniform: every thread holds the same totals
            continue;
        }
        // Chebyshev update (V = M_b^{-1} r)
        const double* cf = coef + static_cast<int64_t>(k) * nr * 3;
        for (int e = tid; e < nr * kChebMaxM; e += NT) {
            const int q = e / kChebMaxM, i = e - q * kChebMaxM;
            if (i >= m) continue;
            const double al = cf[3 * q], be = cf[3 * q + 1], de = cf[3 * q + 2];
            const double d = al * Dv[e] + be * V[e];
            X[e] += d;
            if (k + 1 < iters) {
                const double s2 = al * Sv[e] + be * R[e];
                Dv[e] = d;
                Sv[e] = s2;
                R[e] = R[e] - s2 - (i < ms ? de * d : 0.0);
            }
        }
        __syncthreads();
    }
    return cgs.on ? open : 0u;
}

}  // namespace chol

// Chebyshev h2f copies (cheb_block) of the ld > 64 blocks for one launch group of copies c0 (and
// c1 when nr = 2): workgroup g = block order[g]; M_base = the base copy's factors, x_base its
// solution (slot vector), coef = the group's [iters][nr][3] {alpha, beta, delta}.
extern "C" __global__ __launch_bounds__(chol::kChebThreads) void dbslmm_chol_cheb(
    const double* __restrict__ M_base, const int32_t* __restrict__ order, int32_t n_blocks,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ms, const int32_t* __restrict__ blk_ld,
    const int64_t* __restrict__ blk_matoff, const int32_t* __restrict__ blk_id,
    const int32_t* __restrict__ slot_out, const double* __restrict__ x_base,
    const double* __restrict__ coef, int32_t nr, int32_t iters, double inv_sqrt_n,
    double* __restrict__ beta_s, double* __restrict__ beta_l, int64_t bs_stride, int64_t bl_stride,
    const int32_t* __restrict__ st_base, int32_t* __restrict__ status, int64_t st_stride,
    int32_t c0, int32_t c1, chol::CgStop cgs) {
    using namespace chol;
    const int g = static_cast<int>(blockIdx.x);
    if (g >= n_blocks) return;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int b = order[g];
    const int row0 = blk_row0[b], m = blk_m[b], ms = blk_ms[b], ld = blk_ld[b];
    const int tid = threadIdx.x;
    const int32_t st = st_base[blk_id[b]];
    const bool fail = st >= DBSLMM_BLOCK_NOT_PD;
    if (tid < nr) status[(tid == 0 ? c0 : c1) * st_stride + blk_id[b]] = st;
    double* X = lds;
    double* R = X + kChebR * kChebMaxM;
    double* Dv = R + kChebR * kChebMaxM;
    double* Sv = Dv + kChebR * kChebMaxM;
    if (!fail) {
        for (int e = tid; e < nr * kChebMaxM; e += kChebThreads) {
            const int q = e / kChebMaxM, i = e - q * kChebMaxM;
            const double xb = i < m ? x_base[row0 + i] : 0.0;
            X[e] = xb;
            R[e] = i < ms ? -coef[3 * q + 2] * xb : 0.0;
            Dv[e] = 0.0;
            Sv[e] = 0.0;
        }
        __syncthreads();
        const uint32_t open = cheb_block(M_base + blk_matoff[b], ld, m, ms, nr, iters, coef, lds, cgs);
        // CG reached its cap (the Chebyshev count) above the bound: reported, not silent
        if (tid < nr && (open >> tid & 1u))
            status[(tid == 0 ? c0 : c1) * st_stride + blk_id[b]] = DBSLMM_BLOCK_NOT_CONVERGED;
    }
    for (int e = tid; e < nr * m; e += kChebThreads) {
        const int q = e / m, i = e - q * m;
        const int cq = q == 0 ? c0 : c1;
        const double v = fail ? __builtin_nan("") : X[q * kChebMaxM + i] * inv_sqrt_n;
        const int o = slot_out[row0 + i];
        if (o >= 0) beta_s[cq * bs_stride + o] = v;
        else beta_l[cq * bl_stride - 1 - o] = v;
    }
}

// Blocks with ld <= 64: one wave each, kSmallWaves per workgroup.
extern "C" __global__ __launch_bounds__(chol::kSmallWaves * chol::kWave) void dbslmm_chol_small(
    double* __restrict__ M, const int32_t* __restrict__ order, int32_t n_blocks,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ms, const int32_t* __restrict__ blk_ld,
    const int64_t* __restrict__ blk_matoff, const int32_t* __restrict__ blk_id,
    const double* __restrict__ z_slot, const int32_t* __restrict__ slot_out,
    const double* __restrict__ rsd, const double* __restrict__ dshift_p, double inv_sqrt_n,
    double* __restrict__ beta_s, double* __restrict__ beta_l, int32_t* __restrict__ status) {
    const double dshift = *dshift_p;   // 1/(sigma_s n): a device scalar so one launch list serves every sigma
    __shared__ __attribute__((aligned(16))) double lds[chol::kSmallWaves * chol::kSmallDoublesPerWave];
    const chol::BlockArgs a{blk_row0, blk_m, blk_ms, blk_ld, blk_matoff, blk_id, z_slot, slot_out,
                            rsd, dshift, inv_sqrt_n, beta_s, beta_l, status};
    const int wave = threadIdx.x / chol::kWave, lane = threadIdx.x & (chol::kWave - 1);
    const int idx = blockIdx.x * chol::kSmallWaves + wave;
    if (idx >= n_blocks) return;     // whole wave leaves; this kernel has no workgroup barrier
    double* L = lds + wave * chol::kSmallDoublesPerWave;
    chol::small_block(a, M, order[idx], L, L + chol::kSmallTri, lane);
}

// Blocks with ld > 64: one 512-thread workgroup each.  Dynamic LDS = kLargeDoubles doubles.
extern "C" __global__ __launch_bounds__(chol::kLargeThreads) void dbslmm_chol_large(
    double* __restrict__ M, const int32_t* __restrict__ order, int32_t n_blocks,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ms, const int32_t* __restrict__ blk_ld,
    const int64_t* __restrict__ blk_matoff, const int32_t* __restrict__ blk_id,
    const double* __restrict__ z_slot, const int32_t* __restrict__ slot_out,
    const double* __restrict__ rsd, const double* __restrict__ dshift_p, double inv_sqrt_n,
    double* __restrict__ y, double* __restrict__ beta_s, double* __restrict__ beta_l,
    int32_t* __restrict__ status, int32_t n_copies, int64_t m_stride, int64_t y_stride,
    int64_t bs_stride, int64_t bl_stride, int64_t st_stride) {
    // workgroup g: block order[g / n_copies] of factorisation copy g % n_copies (h2f tuning: all
    // copies in one launch, each block's copies next to each other, largest blocks first)
    const int g = static_cast<int>(blockIdx.x);
    if (g >= n_blocks * n_copies) return;
    const int c = g % n_copies;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const chol::BlockArgs a{blk_row0, blk_m, blk_ms, blk_ld, blk_matoff, blk_id, z_slot, slot_out,
                            rsd, dshift_p[c], inv_sqrt_n, beta_s + c * bs_stride,
                            beta_l + c * bl_stride, status + c * st_stride};
    chol::large_block(a, M + c * m_stride, y + c * y_stride, order[g / n_copies], lds);
}
