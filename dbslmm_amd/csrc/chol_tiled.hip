// chol_tiled.hip -- multi-workgroup Cholesky + solves for the big LD blocks (included by plan.hip
// after chol.hip).  Same bordered system as chol.hip (z appended as row m, y = L^{-1} z left in
// row m, beta = L^{-T} y / sqrt n), but every block with m >= the tiled threshold is spread over
// many workgroups, batched across blocks, one launch per phase (schedule: build_tiled in plan.hip):
//
//   tchol_region        factor + invert a 128 x 128 diagonal region in LDS (+ pending updates)
//   tchol_panel         L_i = A_i L_RR^{-T} per 64-row tile below the region (+ pending update)
//   tchol_trailing3     C_IJ -= L_I L_J^T on 128 x 128 tiles, K = 128 x regions per super step
// followed by one persistent backward substitution over all tiled blocks (trsv.hip,
// dbslmm_trsv_bwd, plain mode).
//
// A 64 x 64 diagonal tile is factored as 2 x 2 tiles of 32 by chol::factor_diag:
//   L00, X00 = L00^{-1};  L10 = A10 X00^T;  A11 -= L10 L10^T;  L11, X11;  X10 = -X11 L10 X00
// and stored as: strict lower = L, diagonal + upper (r, c >= r) = X[c][r] (X = L_kk^{-1}).  The
// panel and region kernels also store every off-diagonal 64 x 64 tile of L transposed into the
// upper triangle (rows < m only), for the row-streaming backward substitution of trsv.hip.
//
// Work items of the region / panel / trailing launches are int32 pairs [block or tile,
// (local step << 8) | count]: every block runs at its own step inside a shared launch.
namespace chol {

constexpr int kBT = 64;                          // tiled-path tile edge (half the panel width)
constexpr int kSub = kT * kTS;                   // one 32x32 LDS sub-tile (stride 34)
// LDS carve of the tiled kernels (doubles): 8 sub-tiles = two 64x64 operands
constexpr int kTiledDoubles = 8 * kSub + 2 * kT + 8;

struct TiledArgs {
    double* M;
    const int32_t* blk_row0;
    const int32_t* blk_m;
    const int32_t* blk_ms;
    const int32_t* blk_ld;
    const int64_t* blk_matoff;
    const int32_t* blk_id;
    const double* z_slot;
    const int32_t* slot_out;
    const double* rsd;
    const double* dshift;   // device scalar 1/(sigma_s n)
    double inv_sqrt_n;
    double* y;
    double* beta_s;
    double* beta_l;
    int32_t* status;
    // replicated factorisations (h2f tuning): item block id bq = b + c * nb is copy c, whose
    // matrices, sigma scalar, scratch, betas and status sit at these strides
    int32_t nb;
    int64_t m_stride, y_stride, bs_stride, bl_stride, st_stride;

    __device__ __forceinline__ TiledArgs view(int bq, int& b) const {
        const int c = bq / nb;
        b = bq - c * nb;
        TiledArgs v = *this;
        v.M += c * m_stride;
        v.dshift += c;
        v.y += c * y_stride;
        v.beta_s += c * bs_stride;
        v.beta_l += c * bl_stride;
        v.status += c * st_stride;
        return v;
    }
};

__device__ __forceinline__ void acc_to_lds_t(const v4d (&acc)[2][2], double* W, int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                W[(16 * sj + (lane & 15)) * kTS + 16 * si + (lane >> 4) + 4 * q] = acc[si][sj][q];
}

__device__ __forceinline__ void zero_acc(v4d (&acc)[2][2]) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj) acc[si][sj] = v4d{0.0, 0.0, 0.0, 0.0};
}

// 64x64 tile (r0, c0) -> 4 LDS sub-tiles: S[2a + b] = rows 32a.., cols 32b..
__device__ __forceinline__ void stage64(double* S, const double* A, int ld, int r0, int c0, int tid) {
    constexpr int NT = kLargeThreads;
    double v[kBT * kBT / NT];
#pragma unroll
    for (int it = 0; it < kBT * kBT / NT; ++it) {
        const int e = it * NT + tid;
        v[it] = A[static_cast<int64_t>(r0 + (e >> 6)) * ld + c0 + (e & 63)];
    }
#pragma unroll
    for (int it = 0; it < kBT * kBT / NT; ++it) {
        const int e = it * NT + tid;
        const int r = e >> 6, c = e & 63;
        S[(2 * (r >> 5) + (c >> 5)) * kSub + (r & 31) * kTS + (c & 31)] = v[it];
    }
}

// stage_tile split into its loads (registers) and its LDS stores, so the next slice of a
// pending update is in flight while the current one is multiplied
__device__ __forceinline__ void tile32_load(double (&v)[kT * kT / kWave], const double* A, int ld, int r0, int c0,
                                            int lane) {
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {
        const int e = it * kWave + lane;
        v[it] = A[static_cast<int64_t>(r0 + (e >> 5)) * ld + c0 + (e & 31)];
    }
}
__device__ __forceinline__ void tile32_store(const double (&v)[kT * kT / kWave], double* W, int lane) {
#pragma unroll
    for (int it = 0; it < kT * kT / kWave; ++it) {
        const int e = it * kWave + lane;
        W[(e >> 5) * kTS + (e & 31)] = v[it];
    }
}

}  // namespace chol

// ---------------------------------------------------------------- 128-column regions
// Region r (columns c0 = 128 r ..) is factored by dbslmm_tchol_region and holds, after it: strict
// lower = L, each 64 x 64 diagonal tile's diagonal + upper (r, c >= r) = X[c][r] of its own
// inverse (what the panel and the backward solve read).
namespace chol {

// X block (64 x 64) in row-major form from the stored upper triangle: X[q][r] = A(rr0 + r,
// cc0 + q); on a diagonal block only q >= r (else 0).  S: 4 sub-tiles (q >> 5, r >> 5).
__device__ __forceinline__ void stage_x(double* S, const double* A, int ld, int rr0, int cc0,
                                        bool diag, int tid) {
    double v[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, q = e & 63;
        v[it] = (!diag || q >= r) ? A[static_cast<int64_t>(rr0 + r) * ld + cc0 + q] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, q = e & 63;
        S[(2 * (q >> 5) + (r >> 5)) * kSub + (q & 31) * kTS + (r & 31)] = v[it];
    }
}

// stage_x split into its loads (registers) and its LDS stores, so loads can be issued early
__device__ __forceinline__ void xregs_load(double (&v)[16], const double* A, int ld, int rr0, int cc0,
                                           bool diag, int tid) {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, q = e & 63;
        v[it] = (!diag || q >= r) ? A[static_cast<int64_t>(rr0 + r) * ld + cc0 + q] : 0.0;
    }
}
__device__ __forceinline__ void xregs_store(const double (&v)[16], double* S, int tid) {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, q = e & 63;
        S[(2 * (q >> 5) + (r >> 5)) * kSub + (q & 31) * kTS + (r & 31)] = v[it];
    }
}

// upper triangle (incl. diagonal) of a 64 x 64 block as-is (= X^T of a diagonal block), 0 below
__device__ __forceinline__ void stage_upper(double* S, const double* A, int ld, int r0, int c0, int tid) {
    double v[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, c = e & 63;
        v[it] = c >= r ? A[static_cast<int64_t>(r0 + r) * ld + c0 + c] : 0.0;
    }
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid, r = e >> 6, c = e & 63;
        S[(2 * (r >> 5) + (c >> 5)) * kSub + (r & 31) * kTS + (c & 31)] = v[it];
    }
}

// this thread's 16 elements of a 64x64 tile (coalesced rows), and their LDS sub-tile slots
__device__ __forceinline__ void tile_regs_load(double (&v)[16], const double* A, int ld, int r0, int c0, int tid) {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid;
        v[it] = A[static_cast<int64_t>(r0 + (e >> 6)) * ld + c0 + (e & 63)];
    }
}
__device__ __forceinline__ void tile_regs_store(const double (&v)[16], double* S, int tid) {
#pragma unroll
    for (int it = 0; it < 16; ++it) {
        const int e = it * kLargeThreads + tid;
        const int r = e >> 6, c = e & 63;
        S[(2 * (r >> 5) + (c >> 5)) * kSub + (r & 31) * kTS + (c & 31)] = v[it];
    }
}

// 32 x 32 tile in LDS (stride kTS, lower triangle valid, rows beyond m zero): factor and invert
// it in one pass (the scheme of factor_diag: row lanes factor, lanes 32..63 carry the columns of
// X = L^{-1}).  Both go back into T in the layout of the stored matrix: strict lower = L, diagonal
// + upper (r, c >= r) = X[c][r] (L's diagonal is not kept: nothing reads it), so the region needs
// no LDS of its own for the inverses.
__device__ __forceinline__ bool factor_tile_lds(double* T, double* colb, int c0, int m, int ms, double dshift,
                                                int lane) {
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
#pragma unroll
    for (int j = 0; j < kT; ++j) {
        if (j < jmax) {
            const double p = readlane_f64(v[j], j);
            fail |= !(p > 0.0);
            const double rs = rsqrt_f64(p);
            v[j] = (!xlane && r < j) ? 0.0 : v[j] * rs;
            // column j through LDS: one wave, so its LDS operations execute in issue order, and
            // the compiler keeps the store / loads (possibly aliasing addresses) in program order
            // -- no wave barrier between the steps, so step j + 1's pivot overlaps step j's FMAs
            double* cb = colb + kT * (j & 1);   // alternate buffers: no write-after-read on reuse
            if (!xlane) cb[r] = v[j];
#pragma unroll
            for (int k0 = (j + 1) & ~7; k0 < kT; k0 += 8) {
                double col[8];
#pragma unroll
                for (int k = 0; k < 8; k += 2) {
                    const v2d t = *reinterpret_cast<const v2d*>(cb + k0 + k);
                    col[k] = t[0];
                    col[k + 1] = t[1];
                }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if (k0 + k > j) v[k0 + k] -= v[j] * col[k];
            }
        }
    }
    // row lane r: L[r][c < r]; inverse lane r (column r of X): X[q][r] for q >= r at (r, q)
#pragma unroll
    for (int c = 0; c < kT; ++c) {
        if (!xlane && c < r) T[r * kTS + c] = v[c];
        if (xlane && c >= r) T[r * kTS + c] = c >= jmax ? (c == r ? 1.0 : 0.0) : v[c];
    }
    wave_sync();
    return fail;
}

// X[a][b] of a diagonal sub-tile factored by factor_tile_lds (lower triangular: 0 above)
__device__ __forceinline__ double x_at(const double* T, int a, int b) {
    return b <= a ? T[b * kTS + a] : 0.0;
}

// acc (2 x 2 of 16 x 16) += sign * P Q^T over K = 32, operand elements P(row, k), Q(row, k) from
// the accessors (the reads and MFMA order of mfma_tile)
template <class PF, class QF>
__device__ __forceinline__ void mfma_tile_f(v4d (&acc)[2][2], PF pget, QF qget, double sign, int lane) {
    const int ri = lane & 15, kq = lane >> 4;
    double p0[kT / 4], p1[kT / 4], q0[kT / 4], q1[kT / 4];
#pragma unroll
    for (int kk = 0; kk < kT / 4; ++kk) {
        const int k = 4 * kk + kq;
        p0[kk] = pget(ri, k);
        p1[kk] = pget(16 + ri, k);
        q0[kk] = qget(ri, k);
        q1[kk] = qget(16 + ri, k);
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

__device__ __forceinline__ void lds_to_acc(v4d (&acc)[2][2], const double* W, int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                acc[si][sj][q] = W[(16 * si + (lane >> 4) + 4 * q) * kTS + 16 * sj + (lane & 15)];
}

// acc (a 32 x 32 piece of L at rows r0.., columns c0..) also stored transposed into the upper
// triangle (rows c0.., columns r0..) for the row-streaming backward substitution (trsv.hip);
// rows >= m (the bordered z row, padding) are not copied
__device__ __forceinline__ void store_acc_t(const v4d (&acc)[2][2], double* A, int ld, int r0, int c0, int m,
                                            int lane) {
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int r = r0 + 16 * si + (lane >> 4) + 4 * q;
                if (r < m) A[static_cast<int64_t>(c0 + 16 * sj + (lane & 15)) * ld + r] = acc[si][sj][q];
            }
}

// A 64 x 64 tile of L held in 4 LDS sub-tiles (S[2a + b] = rows 32 a.., cols 32 b..) -> A at
// (r0, c0), and transposed into the upper triangle at (c0, r0) for the row-streaming backward
// substitution (rows >= m not copied).  Both writes in whole 512-B row segments (the per-lane
// MFMA layout would scatter 32-B pieces over 16 rows per instruction).
__device__ __forceinline__ void store64_both(const double* S, double* A, int ld, int r0, int c0, int m, int tid) {
    constexpr int NT = kLargeThreads;
#pragma unroll 4
    for (int it = 0; it < kBT * kBT / NT; ++it) {
        const int e = it * NT + tid, r = e >> 6, c = e & 63;
        A[static_cast<int64_t>(r0 + r) * ld + c0 + c] = S[(2 * (r >> 5) + (c >> 5)) * kSub + (r & 31) * kTS + (c & 31)];
    }
#pragma unroll 4
    for (int it = 0; it < kBT * kBT / NT; ++it) {
        const int e = it * NT + tid, c = e >> 6, r = e & 63;
        if (r0 + r < m)
            A[static_cast<int64_t>(c0 + c) * ld + r0 + r] = S[(2 * (r >> 5) + (c >> 5)) * kSub + (r & 31) * kTS + (c & 31)];
    }
}

// lower sub-tiles (a >= b) of a 128 x 128 region, 4 x 4 of 32
__device__ __forceinline__ int rsub(int a, int b) { return a * (a + 1) / 2 + b; }
// LDS of the region kernel: R (10 sub-tiles; the diagonal ones also hold their inverses, the
// pending-update staging and the 64-level inverse temporaries reuse R) + colb + flag = 87.6 KiB,
// so a region workgroup fits on a CU beside one trailing workgroup (64 KiB)
constexpr int kRegionDoubles = 10 * kSub + 2 * kT + 8;

}  // namespace chol

// ---------------------------------------------------------------- kernels
// Factor region r (128 x 128 at c0 = 128 r) of each listed block, entirely in LDS (one workgroup
// per block, 4 waves): load the region's lower sub-tiles -- applying the pending K = 128 update
// C -= P P^T from the panels of regions r-update .. r-1 (update = 0, 1, 2; P staged one 32-column
// slice at a time) --
// then four 32-column steps (wave 0: factor_tile_lds; all waves: MFMA panel and trailing updates
// inside the region), the 64-level inverse blocks X10 = -X11 L10 X00 of its two 64 x 64
// diagonal tiles, and the write-back: strict lower = L, each 64 x 64 diagonal tile's diagonal +
// upper = its X^T (what the panel and the backward solve read).  Region 0 without update also
// writes the z row and flags monomorphic SNPs.  87.6 KiB of LDS and <= 256 registers per lane
// (2 waves per SIMD), so the workgroup needs half a CU, not a whole one: the lead chain's region
// launches start beside the bulk trailing workgroups instead of waiting for a CU to drain.
extern "C" __global__ __launch_bounds__(chol::kLargeThreads, 2) void dbslmm_tchol_region(
    chol::TiledArgs a0, const int32_t* __restrict__ blocks, int32_t n) {
    using namespace chol;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= n) return;
    int b;
    const TiledArgs a = a0.view(blocks[2 * blockIdx.x], b);
    const int32_t meta = blocks[2 * blockIdx.x + 1];
    const int reg = meta >> 8, update = meta & 255;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ld = a.blk_ld[b], ms = a.blk_ms[b];
    double* A = a.M + a.blk_matoff[b];
    const double dshift = *a.dshift;
    const int c0 = 2 * kBT * reg;
    STAMP_DECL
#ifdef DBSLMM_STAMPS
    st_base = (update == 0 && reg > 0) ? 8 : 0;   // the first region of a super step: its own counters
#endif
    STAMP_BEGIN();
    double* R = lds;
    double* colb = lds + 10 * kSub;
    int* fflag = reinterpret_cast<int*>(colb + 2 * kT);
    if (tid == 0) *fflag = 0;
    if (reg == 0 && !update) {
        for (int c = tid; c < m; c += kLargeThreads)
            A[static_cast<int64_t>(m) * ld + c] = a.z_slot[row0 + c];   // z row
        __syncthreads();
    }
    // 1) region -> registers (wave w owns sub-tiles w, w + 4, w + 8), pending update, -> LDS
    v4d acc[3][2][2];
    int qa[3], qb[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int q = wave + 4 * u;
        int aa = 0;
        while ((aa + 1) * (aa + 2) / 2 <= q) ++aa;
        qa[u] = aa;
        qb[u] = q - aa * (aa + 1) / 2;
        if (q < 10) load_acc(acc[u], A, ld, c0 + kT * qa[u], c0 + kT * qb[u], lane);
    }
    if (update) {
        double* P = R;     // staging of one 32-column slice of the panel rows (4 sub-tiles; R is
                           // not populated before the accumulators are stored below)
        const int cp = c0 - 2 * kBT * update, nk = 4 * update;
        double nv[kT * kT / chol::kWave];
        tile32_load(nv, A, ld, c0 + kT * wave, cp, lane);
        for (int k = 0; k < nk; ++k) {
            __syncthreads();                  // every wave is done with the previous slice
            tile32_store(nv, P + wave * kSub, lane);
            if (k + 1 < nk) tile32_load(nv, A, ld, c0 + kT * wave, cp + kT * (k + 1), lane);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 3; ++u)
                if (wave + 4 * u < 10) mfma_tile(acc[u], P + qa[u] * kSub, P + qb[u] * kSub, -1.0, lane);
        }
        __syncthreads();                      // every wave is done with the staging (= R)
    }
#pragma unroll
    for (int u = 0; u < 3; ++u)
        if (wave + 4 * u < 10) acc_to_lds(acc[u], R + (wave + 4 * u) * kSub, lane);
    __syncthreads();
    STAMP_END(0);
    STAMP_BEGIN();
    // 2) four 32-column steps inside the region
    for (int t = 0; t < 4; ++t) {
        if (c0 + kT * t >= m) break;
        if (wave == 0) {
            const bool f = factor_tile_lds(R + rsub(t, t) * kSub, colb, c0 + kT * t, m, ms, dshift, lane);
            if (f && lane == 0) *fflag = 1;
        }
        __syncthreads();
        if (t == 0) STAMP_END(7);
        else STAMP_END(4);
        STAMP_BEGIN();
        {   // panel: R[i][t] <- R[i][t] X_t^T
            const int i = t + 1 + wave;
            if (i <= 3 && c0 + kT * i <= m) {
                v4d pc[2][2];
                zero_acc(pc);
                const double* P = R + rsub(i, t) * kSub;
                const double* X = R + rsub(t, t) * kSub;
                mfma_tile_f(pc, [&](int r, int k) { return P[r * kTS + k]; },
                            [&](int r, int k) { return x_at(X, r, k); }, 1.0, lane);
                acc_to_lds(pc, R + rsub(i, t) * kSub, lane);
            }
        }
        __syncthreads();
        STAMP_END(5);
        STAMP_BEGIN();
        {   // trailing: R[i][j] -= R[i][t] R[j][t]^T, t < j <= i <= 3
            const int nt = 3 - t, np = nt * (nt + 1) / 2;
            for (int pq = wave; pq < np; pq += 4) {
                int ii = 0;
                while ((ii + 1) * (ii + 2) / 2 <= pq) ++ii;
                const int i = t + 1 + ii, j = t + 1 + (pq - ii * (ii + 1) / 2);
                if (c0 + kT * i > m) continue;
                v4d tc[2][2];
                lds_to_acc(tc, R + rsub(i, j) * kSub, lane);
                mfma_tile(tc, R + rsub(i, t) * kSub, R + rsub(j, t) * kSub, -1.0, lane);
                acc_to_lds(tc, R + rsub(i, j) * kSub, lane);
            }
        }
        __syncthreads();
        STAMP_END(6);
        STAMP_BEGIN();
    }
    STAMP_END(1);
    STAMP_BEGIN();
    // 3a) write-back of the region's off-diagonal 64 x 64 tile L10 (sub-tiles (2|3, 0|1)), as-is and
    //     transposed: its LDS then holds the 64-level inverse temporaries
    for (int u = 0; u < 4; ++u) {
        const int aa = 2 + (u >> 1), bb = u & 1;
        const double* S = R + rsub(aa, bb) * kSub;
        for (int e = tid; e < kT * kT; e += kLargeThreads) {
            const int rr = e >> 5, cc = e & 31;
            const int gr = c0 + kT * aa + rr, gc = c0 + kT * bb + cc;
            if (gr <= m && gc < m) A[static_cast<int64_t>(gr) * ld + gc] = S[rr * kTS + cc];
        }
        for (int e = tid; e < kT * kT; e += kLargeThreads) {
            const int rr = e & 31, cc = e >> 5;
            const int gr = c0 + kT * aa + rr, gc = c0 + kT * bb + cc;
            if (gr < m && gc < m) A[static_cast<int64_t>(gc) * ld + gr] = S[rr * kTS + cc];
        }
    }
    __syncthreads();
    STAMP_END(2);
    STAMP_BEGIN();
    // 3b) 64-level inverse blocks: X10_p = -X_{2p+1} (L_{2p+1,2p} X_{2p}), p = wave (0, 1), in the
    //     LDS of sub-tile (2, p)
    double* X10 = R + rsub(2, 0) * kSub;   // X10 + p * kSub = sub-tile (2, p)
    if (wave < 2 && c0 + kBT * wave + kT <= m) {
        const int p = wave;
        const double* L10 = R + rsub(2 * p + 1, 2 * p) * kSub;
        const double* X0 = R + rsub(2 * p, 2 * p) * kSub;
        const double* X1 = R + rsub(2 * p + 1, 2 * p + 1) * kSub;
        double* W = X10 + p * kSub;
        v4d tt[2][2];
        zero_acc(tt);
        mfma_tile_f(tt, [&](int r, int k) { return L10[r * kTS + k]; },
                    [&](int r, int k) { return x_at(X0, k, r); }, 1.0, lane);              // T = L10 X00
        acc_to_lds(tt, W, lane);
        chol::wave_sync();
        zero_acc(tt);
        mfma_tile_f(tt, [&](int r, int k) { return x_at(X1, r, k); },
                    [&](int r, int k) { return W[k * kTS + r]; }, -1.0, lane);               // -X11 T
        chol::wave_sync();
        acc_to_lds(tt, W, lane);
    }
    __syncthreads();
    // 4) write-back of the rest: the other lower sub-tiles, the diagonal sub-tiles (strict lower =
    //    L, diagonal + upper = X^T, both already in place), and X10^T
    for (int q = 0; q < 10; ++q) {
        int aa = 0;
        while ((aa + 1) * (aa + 2) / 2 <= q) ++aa;
        const int bb = q - aa * (aa + 1) / 2;
        if (aa >= 2 && bb <= 1) continue;      // L10: written above
        const double* S = R + q * kSub;
        const int jm = min(kT, m - (c0 + kT * aa));
        for (int e = tid; e < kT * kT; e += kLargeThreads) {
            const int rr = e >> 5, cc = e & 31;
            const int gr = c0 + kT * aa + rr, gc = c0 + kT * bb + cc;
            if (aa == bb && cc >= rr) {
                if (rr < jm) A[static_cast<int64_t>(gr) * ld + gc] = S[rr * kTS + cc];
                continue;
            }
            if (gr > m || gc >= m) continue;
            A[static_cast<int64_t>(gr) * ld + gc] = S[rr * kTS + cc];
        }
    }
    for (int p = 0; p < 2; ++p) {      // upper-right sub-tile of each 64 x 64 diagonal tile: X10^T
        if (c0 + kBT * p + kT > m) break;
        const double* X = X10 + p * kSub;
        for (int e = tid; e < kT * kT; e += kLargeThreads) {
            const int rr = e >> 5, cc = e & 31;
            A[static_cast<int64_t>(c0 + kBT * p + rr) * ld + c0 + kBT * p + kT + cc] = X[cc * kTS + rr];
        }
    }
    STAMP_END(3);
    const bool fail = *fflag != 0;
    if (reg == 0 && !update) {
        chol::BlockArgs ba{a.blk_row0, a.blk_m, a.blk_ms, a.blk_ld, a.blk_matoff, a.blk_id, a.z_slot,
                           a.slot_out, a.rsd, dshift, a.inv_sqrt_n, a.beta_s, a.beta_l, a.status};
        chol::report_status(ba, b, row0, m, tid, chol::kLargeThreads, fail && tid == 0);
    } else if (fail && tid == 0) {
        atomicMax(a.status + a.blk_id[b], DBSLMM_BLOCK_NOT_PD);
    }
}

// panel of outer step s, one workgroup per 64-row tile i below region s (item (block << 16) | i):
// L_i0 = A_i0 X00^T, then L_i1 = (A_i1 - L_i0 L10^T) X11^T (X00, X11: the inverses of the
// region's two 64 x 64 diagonal tiles; L10 its off-diagonal 64 x 64 block).  upd: first apply
// the pending update of A_i from the panels of regions s-upd .. s-1.
extern "C" __global__ __launch_bounds__(chol::kLargeThreads, 2) void dbslmm_tchol_panel(
    chol::TiledArgs a0, const int32_t* __restrict__ items, int32_t n_items) {
    using namespace chol;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= n_items) return;
    const int32_t it = items[2 * blockIdx.x];
    const int32_t meta = items[2 * blockIdx.x + 1];
    const int s = meta >> 8, upd = meta & 255;
    const int i = it & 0xFFFF;
    int b;
    const TiledArgs a = a0.view(it >> 16, b);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qi = wave >> 1, qj = wave & 1;
    const int m = a.blk_m[b], ld = a.blk_ld[b];
    const int T = (m + kBT - 1) / kBT;
    double* A = a.M + a.blk_matoff[b];
    const int c0 = 2 * kBT * s;
    double* XS = lds;
    double* W = lds + 4 * kSub;
    const bool two = 2 * s + 1 <= T - 1;            // the region has a second column tile
    // every global load of the workgroup first (one latency), then the three products
    double x00[16], ai0[16], l10[16], x11[16];
    v4d cc[2][2];
    v4d u0[2][2];
    if (upd) {
        // pending K = 128 upd update from the panels of regions s-upd .. s-1 (what a trailing
        // launch of region s's columns would do): A_i -= L_{i,.} L_{R,.}^T, R = region s's 128
        // rows; wave (qi, qj) updates its quadrant of both 64-column halves, operands staged 32
        // columns at a time (sub-tiles 0-1: rows of tile i, 2-5: rows of the region)
        const int cp = c0 - 2 * kBT * upd, nk = 4 * upd;
        load_acc(u0, A, ld, kBT * i + kT * qi, c0 + kT * qj, lane);
        if (two) load_acc(cc, A, ld, kBT * i + kT * qi, c0 + kBT + kT * qj, lane);
        // sub-tile q of a slice: rows of tile i (q < 2) or of the region (q >= 2); wave w stages
        // q = w and (waves 0, 1) q = w + 4, the next slice in flight during the current MFMAs
        const int qa = wave, qb = wave + 4;
        const int ra = qa < 2 ? kBT * i + kT * qa : c0 + kT * (qa - 2), rb = c0 + kT * (qb - 2);
        double na[kT * kT / chol::kWave], nb[kT * kT / chol::kWave];
        tile32_load(na, A, ld, ra, cp, lane);
        if (qb < 6) tile32_load(nb, A, ld, rb, cp, lane);
        for (int kc = 0; kc < nk; ++kc) {
            tile32_store(na, lds + qa * kSub, lane);
            if (qb < 6) tile32_store(nb, lds + qb * kSub, lane);
            if (kc + 1 < nk) {
                tile32_load(na, A, ld, ra, cp + kT * (kc + 1), lane);
                if (qb < 6) tile32_load(nb, A, ld, rb, cp + kT * (kc + 1), lane);
            }
            __syncthreads();
            mfma_tile(u0, lds + qi * kSub, lds + (2 + qj) * kSub, -1.0, lane);
            if (two) mfma_tile(cc, lds + qi * kSub, lds + (4 + qj) * kSub, -1.0, lane);
            __syncthreads();
        }
    }
    xregs_load(x00, A, ld, c0, c0, true, tid);
    if (!upd) tile_regs_load(ai0, A, ld, kBT * i, c0, tid);
    if (two) {
        tile_regs_load(l10, A, ld, c0 + kBT, c0, tid);
        xregs_load(x11, A, ld, c0 + kBT, c0 + kBT, true, tid);
        if (!upd) load_acc(cc, A, ld, kBT * i + kT * qi, c0 + kBT + kT * qj, lane);   // A_i1
    }
    xregs_store(x00, XS, tid);
    if (upd) acc_to_lds(u0, W + (2 * qi + qj) * kSub, lane);
    else tile_regs_store(ai0, W, tid);
    __syncthreads();
    v4d acc[2][2];
    zero_acc(acc);
    for (int kc = 0; kc <= qj; ++kc) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    __syncthreads();
    acc_to_lds(acc, W + (2 * qi + qj) * kSub, lane);                        // L_i0
    __syncthreads();
    store64_both(W, A, ld, kBT * i, c0, m, tid);
    if (!two) return;
    tile_regs_store(l10, XS, tid);
    __syncthreads();
    for (int kc = 0; kc < 2; ++kc) mfma_tile(cc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, -1.0, lane);
    __syncthreads();
    acc_to_lds(cc, W + (2 * qi + qj) * kSub, lane);                          // A_i1 - L_i0 L10^T
    xregs_store(x11, XS, tid);
    __syncthreads();
    zero_acc(acc);
    for (int kc = 0; kc <= qj; ++kc) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    __syncthreads();
    acc_to_lds(acc, W + (2 * qi + qj) * kSub, lane);                        // L_i1
    __syncthreads();
    store64_both(W, A, ld, kBT * i, c0 + kBT, m, tid);
}

// ---------------------------------------------------------------- 128 x 128 trailing update
// C(I, J) -= L_I L_J^T on 128 x 128 tiles (I, J in units of 128 rows), K = 128 nk from column
// c0, one 512-thread workgroup per run of tiles J0..J1 of tile row I.  A 64 x 64 tile does 8 flops
// per operand byte loaded, which at the f64 MFMA rate needs ~10 TB/s of L2/HBM operand traffic;
// a 128 x 128 tile halves that (the bulk of the factorisation is bound by it).  Wave w (8 waves)
// owns rows 64 (w >> 2) .., columns 32 (w & 3) .. of the tile: 4 x 2 accumulators of
// v_mfma_f64_16x16x4_f64; on a diagonal tile (I == J) the two waves wholly above the diagonal
// skip their MFMAs and stores; the next tile's C is prefetched during the last stage of the
// current one.  (A register-staged twin and a 64 x 64-tile version were measured slower in
// round 1 and dropped.)
namespace chol {
constexpr int kT2 = 128;                 // tile edge
constexpr int kK2 = 32;                  // K per stage
constexpr int kRun2 = 1;                 // tiles per run (2 measured slower with two workgroups per CU:
                                         // trail_bench m 9596 K 512, 63.5 vs 73.5 % of the f64 peak)
}  // namespace chol

// The same update fed by LDS-DMA (global_load_lds_dwordx4): no staging registers, no LDS store
// instructions.  Operand rows are unpadded in LDS (32 doubles = 16 chunks of 16 B); the DMA image
// is lane-linear, so the swizzle goes through the SOURCE address: LDS position p of row r holds
// K chunk p ^ (r & 15), which puts the 16 rows of every ds_read_b128 lane group on 16 distinct
// bank groups.  Two slots; per stage: wait for this wave's DMA, barrier, issue the next stage's
// DMA into the other slot (every wave has left it), multiply.  acc holds -C (negated on load and
// store), so the MFMAs add L_I L_J^T.
#ifndef DBSLMM_T3_DIAG
#define DBSLMM_T3_DIAG 0
#endif
namespace chol {
// KS = K per stage: 32 (two 64 KiB slots, one workgroup per CU) or 16 (two 32 KiB slots, two
// workgroups per CU, so one's barrier / DMA wait hides under the other's MFMAs)
template <int KS> struct T3 {
    static constexpr int kOp = kT2 * KS;              // one operand stage, unpadded
    static constexpr int kDoubles = 4 * kOp;          // A, B x 2 slots
    static constexpr int kChunks = KS / 2;            // 16-B chunks per operand row
    static constexpr int kRowsPerInst = 64 / kChunks; // rows one DMA instruction covers
    // LDS position of K chunk c in row r: conflict-free ds_read_b128 for 16 consecutive rows
    __device__ static __forceinline__ int swz(int c, int r) { return KS == 32 ? c ^ (r & 15) : c ^ ((r >> 1) & 7); }
};
constexpr int kOp3 = T3<kK2>::kOp;                   // (K = 32: 32 KiB per operand stage)
constexpr int kTrail3Doubles = T3<kK2>::kDoubles;    // 128 KiB
constexpr int kTrail3k16Doubles = T3<16>::kDoubles;  // 64 KiB
typedef __attribute__((address_space(1))) const void* gptr_f;
typedef __attribute__((address_space(3))) void* lptr_f;

// (32-bit element offsets from the block's base -- tiled blocks have m < 32640, so ld <= 32768 and
// ld * ld <= 2^30 (plan_create) --
// so the loads take a scalar base + one VGPR offset each instead of 64-bit addresses)
__device__ __forceinline__ void t3_load_c(v4d (&c)[4][2], const double* A, int ld, int r0, int c0, int lane) {
    const int o = (r0 + (lane >> 4)) * ld + c0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) c[i][j][q] = -A[o + (16 * i + 4 * q) * ld + 16 * j];
}
__device__ __forceinline__ void t3_store_c(const v4d (&c)[4][2], double* A, int ld, int r0, int c0, int lane) {
    const int o = (r0 + (lane >> 4)) * ld + c0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) A[o + (16 * i + 4 * q) * ld + 16 * j] = -c[i][j][q];
}
// DMA of one stage (rows 16 w .. 16 w + 15 of each operand)
template <int KS>
__device__ __forceinline__ void t3_issue(double* slot, const double* A, int ld, int I, int J, int col,
                                         bool diag, int wave, int lane) {
    using P = T3<KS>;
    const int rr = lane / P::kChunks, p = lane % P::kChunks;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
        if (op == 1 && diag) break;
        const int rb = kT2 * (op ? J : I);
#pragma unroll
        for (int q = 0; q < 16 / P::kRowsPerInst; ++q) {
            const int r = 16 * wave + P::kRowsPerInst * q + rr;
            const int c = P::swz(p, r);   // (the swizzle is an involution: position p holds chunk c)
            __builtin_amdgcn_global_load_lds((gptr_f)(A + ((rb + r) * ld + col + 2 * c)),
                                             (lptr_f)(slot + op * P::kOp + (16 * wave + P::kRowsPerInst * q) * KS), 16, 0, 0);
        }
    }
}
template <int KS>
__device__ __forceinline__ void t3_mfma_stage(v4d (&acc)[4][2], const double* SA, const double* SB,
                                              int wr, int wc, int lane) {
    using P = T3<KS>;
    const int ri = lane & 15, kq = lane >> 4;
    // operand reads one 8-deep group ahead of the MFMAs that consume them
    v2d a[2][4], b[2][2];
    auto load = [&](int j8, int u) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int r = 64 * wr + 16 * i + ri;
            a[u][i] = *reinterpret_cast<const v2d*>(SA + r * KS + 2 * P::swz(4 * j8 + kq, r));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int r = 32 * wc + 16 * j + ri;
            b[u][j] = *reinterpret_cast<const v2d*>(SB + r * KS + 2 * P::swz(4 * j8 + kq, r));
        }
    };
    load(0, 0);
#pragma unroll
    for (int j8 = 0; j8 < KS / 8; ++j8) {
        const int u = j8 & 1;
        if (j8 + 1 < KS / 8) load(j8 + 1, u ^ 1);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][i][h], b[u][j][h], acc[i][j], 0, 0, 0);
    }
}

template <int KS>
__device__ __forceinline__ void trailing3_item(const TiledArgs& a0, int32_t run, const int32_t* __restrict__ items,
                                               int e, double* lds) {
    using P = T3<KS>;
    // K = 32: the next tile's C is prefetched during the current tile's last stage; K = 16 (two
    // workgroups per CU, 128 VGPRs) loads it at the tile's first stage -- the other workgroup's
    // MFMAs cover that wait
    constexpr bool kPrefetchC = KS == 32;
    const int32_t it = items[2 * e];
    if (it < 0) return;
    const int32_t meta = items[2 * e + 1];
    const int s = meta >> 8, nk = meta & 255;
    const int I = (it >> 8) & 255, J0 = it & 255;
    int b;
    const TiledArgs a = a0.view(it >> 16, b);
    const int m = a.blk_m[b], ld = a.blk_ld[b];
    const int T2 = (m + kT2 - 1) / kT2;
    const int J1 = min(J0 + run - 1, min(I, T2 - 1));
    double* A = a.M + a.blk_matoff[b];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 2, wc = wave & 3;
    const int c0 = 2 * kBT * s;
    const int nst = (kT2 / KS) * nk;
    const int total = nst * (J1 - J0 + 1);
    v4d acc[4][2], nxt[4][2];
    t3_issue<KS>(lds, A, ld, I, J0, c0, I == J0, wave, lane);
    t3_load_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * J0 + 32 * wc, lane);
    // tile j's C store is issued at the start of tile j+1's first stage (after that stage's DMA),
    // so it drains under that stage's MFMAs instead of in front of the next vmcnt wait
    for (int g = 0; g < total; ++g) {
        const int J = J0 + g / nst, t = g % nst;
        const bool diag = I == J;
        double* S = lds + (g & 1) * 2 * P::kOp;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA (and C traffic)
        __builtin_amdgcn_s_barrier();                        // stage g is in LDS; slot g+1 free
        if (g + 1 < total) {
            const int Jn = J0 + (g + 1) / nst, tn = (g + 1) % nst;
#if DBSLMM_T3_DIAG != 2
            t3_issue<KS>(lds + ((g + 1) & 1) * 2 * P::kOp, A, ld, I, Jn, c0 + KS * tn, I == Jn, wave, lane);
#endif
            if (kPrefetchC && tn == 0) t3_load_c(nxt, A, ld, kT2 * I + 64 * wr, kT2 * Jn + 32 * wc, lane);
        }
        if (t == 0 && g > 0) {
            const int Jp = J - 1;
            if (!(Jp == I && 32 * wc > 64 * wr + 63)) t3_store_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * Jp + 32 * wc, lane);
            if (kPrefetchC) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = nxt[i][j];
            } else {
                t3_load_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * J + 32 * wc, lane);
            }
        }
        const bool skip = diag && 32 * wc > 64 * wr + 63;
#if DBSLMM_T3_DIAG != 1   // diagnostic builds only (1: no MFMAs, 2: no operand DMA)
        if (!skip) t3_mfma_stage<KS>(acc, S, diag ? S : S + P::kOp, wr, wc, lane);
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    {
        const int J = J1;
        if (!(J == I && 32 * wc > 64 * wr + 63)) t3_store_c(acc, A, ld, kT2 * I + 64 * wr, kT2 * J + 32 * wc, lane);
    }
}
}  // namespace chol

// Work item e of the launch's list, for e = blockIdx.x, + gridDim.x, ... (a grid capped to a
// multiple of 8 keeps item e on XCD e % 8; the plan launches one workgroup per item -- capped
// grids that left 16 / 32 CUs to the chain kernels measured no faster)
extern "C" __global__ __launch_bounds__(512, 1) void dbslmm_tchol_trailing3(
    chol::TiledArgs a0, int32_t run, const int32_t* __restrict__ items, int32_t n_items) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    for (int e = blockIdx.x; e < n_items; e += gridDim.x) {
        chol::trailing3_item<chol::kK2>(a0, run, items, e, lds);
        __syncthreads();   // every wave is done with the LDS slots before the next item's DMA
    }
}
extern "C" __global__ __launch_bounds__(512, 4) void dbslmm_tchol_trailing3k16(   // 4 waves per SIMD: two workgroups per CU
    chol::TiledArgs a0, int32_t run, const int32_t* __restrict__ items, int32_t n_items) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    for (int e = blockIdx.x; e < n_items; e += gridDim.x) {
        chol::trailing3_item<16>(a0, run, items, e, lds);
        __syncthreads();
    }
}

