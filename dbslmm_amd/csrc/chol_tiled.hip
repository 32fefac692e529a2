// chol_tiled.hip -- multi-workgroup Cholesky + solves for the big LD blocks (included by plan.hip
// after chol.hip).  Same bordered system as chol.hip (z appended as row m, y = L^{-1} z left in
// row m, beta = L^{-T} y / sqrt n), but every block with m >= the tiled threshold is spread over
// many workgroups, batched across blocks, one launch per phase of a 64-wide panel step:
//
//   tchol_diag0          step 0 only: factor + invert diagonal tile (0, 0)
//   tchol_panel(k)       L_ik = A_ik X_kk^T for every tile row i > k     (one workgroup per tile)
//   tchol_trailing(k)    C_ij -= L_ik L_jk^T, k < j <= i                 (one workgroup per tile)
//                        -- the first workgroups take tile (k+1, k+1): update, then factor +
//                           invert it (lookahead), overlapping the rest of the update
//   tchol_backward(J)    x_J = X_JJ^T v_J, v_{<J} -= L_{J,<J}^T x_J        (one workgroup per
//                        256 columns; x_J recomputed per workgroup, v_J is read-only in a launch)
//
// A 64 x 64 diagonal tile is factored as 2 x 2 tiles of 32 by chol::factor_diag:
//   L00, X00 = L00^{-1};  L10 = A10 X00^T;  A11 -= L10 L10^T;  L11, X11;  X10 = -X11 L10 X00
// and stored as: strict lower = L, diagonal + upper (r, c >= r) = X[c][r] (X = L_kk^{-1}).
//
// Work lists are per step: the blocks active at that step and the prefix of their work-item
// counts; a workgroup finds its block by binary search (no per-item tables).
namespace chol {

constexpr int kBT = 64;                          // tiled-path tile edge (half the panel width)
constexpr int kJRun = 4;                         // trailing tiles per workgroup run
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
};

// work list of one launch: act[0..n) = plan block indices, pfx[0..n] = prefix of item counts
__device__ __forceinline__ int find_item(const int32_t* pfx, int n, int item) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (pfx[mid] <= item) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

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

// Wave-level factorisation + inversion of the 64x64 diagonal tile at (c0, c0) (rows <= m).
// lds: >= 6 sub-tiles + 2*kT.  Returns true when a pivot was not positive.
__device__ __forceinline__ bool factor_diag64(double* A, int ld, int c0, int m, int ms, double dshift,
                              double* lds, int lane) {
    double* Xl = lds;                 // X00, later X11
    double* Lb = lds + kSub;
    double* L10 = lds + 2 * kSub;
    double* XT = lds + 3 * kSub;      // X00^T
    double* TT = lds + 4 * kSub;      // (L10 X00)^T
    double* W = lds + 5 * kSub;
    double* colb = lds + 6 * kSub;
    bool fail = factor_diag(A, ld, c0, m, ms, dshift, Xl, Lb, colb, lane, false);
    if (c0 + kT > m) return fail;     // the tile ends inside its first half
    // X00^T, A10 -> LDS
    for (int e = lane; e < kT * kT; e += kWave) {
        const int q = e >> 5, r = e & 31;
        XT[r * kTS + q] = Xl[q * kTS + r];
    }
    stage_tile(W, A, ld, c0 + kT, c0, lane);
    wave_sync();
    v4d acc[2][2];
    zero_acc(acc);
    mfma_tile(acc, W, Xl, 1.0, lane);                  // L10 = A10 X00^T
    store_acc(acc, A, ld, c0 + kT, c0, lane);
    acc_to_lds(acc, L10, lane);
    wave_sync();
    v4d c11[2][2];
    load_acc(c11, A, ld, c0 + kT, c0 + kT, lane);
    mfma_tile(c11, L10, L10, -1.0, lane);              // A11 -= L10 L10^T
    acc_to_lds(c11, Lb, lane);
    wave_sync();
    fail |= factor_diag(A, ld, c0 + kT, m, ms, dshift, Xl, Lb, colb, lane, true);   // Xl = X11
    zero_acc(acc);
    mfma_tile(acc, L10, XT, 1.0, lane);                // T = L10 X00
    acc_to_lds_t(acc, TT, lane);
    wave_sync();
    zero_acc(acc);
    mfma_tile(acc, Xl, TT, -1.0, lane);                // X10 = -X11 T
    // X10^T -> sub-tile (0, 1): element (r, 32 + c) = X10[c][r]
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int R = 16 * si + (lane >> 4) + 4 * q, Cc = 16 * sj + (lane & 15);
                A[static_cast<int64_t>(c0 + Cc) * ld + c0 + kT + R] = acc[si][sj][q];
            }
    return fail;
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

}  // namespace chol

// ---------------------------------------------------------------- 128-column outer steps
// Outer step s covers tile columns k0 = 2s, k1 = 2s + 1 (columns c0 = 128 s ..).  Its 128 x 128
// diagonal region R is factored by diag128 (two factor_diag64 + MFMA glue) and holds, after it:
// strict lower = L_RR, diagonal + upper (r, c >= r) = X[c][r], X = L_RR^{-1} (so each 64 x 64
// diagonal tile keeps its own inverse for the backward solve, and tile (k0, k1) holds X10^T).
// panel128(s):    L_i = A_i X^T for 64-row tiles i below R; workgroup = (i, column half h)
// trailing128(s): C_IJ -= L_{I,s} L_{J,s}^T with K = 128 (two 64-deep phases, C in registers)
//                 for J >= k1 + 1; the first workgroups update region s+1 and run diag128 on it.
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

// Factor + invert the 128 x 128 diagonal region at (c0, c0), rows <= m (whole workgroup).
// LDS: 8 sub-tiles + 2 kT + 8 doubles.  Returns true (on every thread) on a non-positive pivot.
__device__ __forceinline__ bool diag128(double* A, int ld, int c0, int m, int ms, double dshift, double* lds, int tid) {
    const int lane = tid & 63, wave = tid >> 6, qi = wave >> 1, qj = wave & 1;
    int* fflag = reinterpret_cast<int*>(lds + 8 * kSub + 2 * kT);
    if (tid == 0) *fflag = 0;
    __syncthreads();
    if (wave == 0) {
        const bool f = factor_diag64(A, ld, c0, m, ms, dshift, lds, lane);
        if (f && lane == 0) *fflag = 1;
    }
    __syncthreads();
    if (c0 + kBT > m) return *fflag != 0;          // no rows in the second half
    double* XS = lds;
    double* W = lds + 4 * kSub;
    stage_x(XS, A, ld, c0, c0, true, tid);          // X00
    stage64(W, A, ld, c0 + kBT, c0, tid);           // A10
    __syncthreads();
    v4d acc[2][2];
    zero_acc(acc);
    for (int kc = 0; kc <= qj; ++kc) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    __syncthreads();
    store_acc(acc, A, ld, c0 + kBT + kT * qi, c0 + kT * qj, lane);   // L10
    acc_to_lds(acc, W + (2 * qi + qj) * kSub, lane);
    stage_upper(XS, A, ld, c0, c0, tid);            // X00^T
    __syncthreads();
    if (qj <= qi) {                                 // A11 -= L10 L10^T
        v4d c11[2][2];
        load_acc(c11, A, ld, c0 + kBT + kT * qi, c0 + kBT + kT * qj, lane);
        for (int kc = 0; kc < 2; ++kc) mfma_tile(c11, W + (2 * qi + kc) * kSub, W + (2 * qj + kc) * kSub, -1.0, lane);
        store_acc(c11, A, ld, c0 + kBT + kT * qi, c0 + kBT + kT * qj, lane);
    }
    zero_acc(acc);                                  // T = L10 X00, parked in tile (k0, k1)
    for (int kc = qj; kc < 2; ++kc) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    store_acc(acc, A, ld, c0 + kT * qi, c0 + kBT + kT * qj, lane);
    __syncthreads();
    if (wave == 0) {
        const bool f = factor_diag64(A, ld, c0 + kBT, m, ms, dshift, lds, lane);
        if (f && lane == 0) *fflag = 1;
    }
    __syncthreads();
    stage_x(XS, A, ld, c0 + kBT, c0 + kBT, true, tid);   // X11
    stage_x(W, A, ld, c0, c0 + kBT, false, tid);          // T^T (row-major transpose of T)
    __syncthreads();
    zero_acc(acc);                                  // X10 = -X11 T
    for (int kc = 0; kc <= qi; ++kc) mfma_tile(acc, XS + (2 * qi + kc) * kSub, W + (2 * qj + kc) * kSub, -1.0, lane);
    // X10^T over T: element (r, 64 + c) = X10[c][r]
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
        for (int sj = 0; sj < 2; ++sj)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int R = kT * qi + 16 * si + (lane >> 4) + 4 * q, Cc = kT * qj + 16 * sj + (lane & 15);
                A[static_cast<int64_t>(c0 + Cc) * ld + c0 + kBT + R] = acc[si][sj][q];
            }
    __syncthreads();
    return *fflag != 0;
}

// C(I, J..) -= L_{I,s} L_{J,s}^T, K = 128 as two 64-deep phases, over a run of tiles J0..J1 of
// tile row I (skips the strictly-upper quadrant of a diagonal tile).  Next phase's operands and
// the next tile's C are prefetched into registers while the current phase's MFMAs run.
__device__ __forceinline__ void update_run(double* A, int ld, int I, int J0, int J1, int c0,
                                           double* lds, int tid) {
    const int lane = tid & 63, wave = tid >> 6, qi = wave >> 1, qj = wave & 1;
    double* LI = lds;
    double* LJ = lds + 4 * kSub;
    double li[16], lj[16];
    v4d acc[2][2], nxt[2][2];
    const int nph = 2 * (J1 - J0 + 1);
    tile_regs_load(li, A, ld, kBT * I, c0, tid);
    if (I != J0) tile_regs_load(lj, A, ld, kBT * J0, c0, tid);
    load_acc(acc, A, ld, kBT * I + kT * qi, kBT * J0 + kT * qj, lane);
    for (int p = 0; p < nph; ++p) {
        const int J = J0 + (p >> 1);
        tile_regs_store(li, LI, tid);
        if (I != J) tile_regs_store(lj, LJ, tid);
        __syncthreads();
        if (p + 1 < nph) {
            const int Jn = J0 + ((p + 1) >> 1), kcn = (p + 1) & 1;
            tile_regs_load(li, A, ld, kBT * I, c0 + kBT * kcn, tid);
            if (I != Jn) tile_regs_load(lj, A, ld, kBT * Jn, c0 + kBT * kcn, tid);
            if (kcn == 0) load_acc(nxt, A, ld, kBT * I + kT * qi, kBT * Jn + kT * qj, lane);
        }
        const double* LJp = I == J ? LI : LJ;
        const bool skip = I == J && qj > qi;
        if (!skip) {
            mfma_tile(acc, LI + (2 * qi) * kSub, LJp + (2 * qj) * kSub, -1.0, lane);
            mfma_tile(acc, LI + (2 * qi + 1) * kSub, LJp + (2 * qj + 1) * kSub, -1.0, lane);
        }
        if (p & 1) {
            if (!skip) store_acc(acc, A, ld, kBT * I + kT * qi, kBT * J + kT * qj, lane);
#pragma unroll
            for (int si = 0; si < 2; ++si)
#pragma unroll
                for (int sj = 0; sj < 2; ++sj) acc[si][sj] = nxt[si][sj];
        }
        __syncthreads();
    }
}

}  // namespace chol

// ---------------------------------------------------------------- kernels
// step 0: z row, factor + invert region 0 of each tiled block; flag monomorphic SNPs
extern "C" __global__ __launch_bounds__(chol::kLargeThreads) void dbslmm_tchol_diag0(
    chol::TiledArgs a, const int32_t* __restrict__ blocks, int32_t n) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= n) return;
    const int b = blocks[blockIdx.x];
    const int tid = threadIdx.x;
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ld = a.blk_ld[b];
    double* A = a.M + a.blk_matoff[b];
    for (int c = tid; c < m; c += chol::kLargeThreads)
        A[static_cast<int64_t>(m) * ld + c] = a.z_slot[row0 + c];   // z row of the bordered matrix
    chol::BlockArgs ba{a.blk_row0, a.blk_m, a.blk_ms, a.blk_ld, a.blk_matoff, a.blk_id, a.z_slot,
                       a.slot_out, a.rsd, *a.dshift, a.inv_sqrt_n, a.beta_s, a.beta_l, a.status};
    __syncthreads();
    const bool fail = chol::diag128(A, ld, 0, m, a.blk_ms[b], *a.dshift, lds, tid);
    chol::report_status(ba, b, row0, m, tid, chol::kLargeThreads, fail && tid == 0);
}

// panel of outer step s: items (block << 16) | (i << 8) | h -> L(i, column half h)
extern "C" __global__ __launch_bounds__(chol::kLargeThreads) void dbslmm_tchol_panel(
    chol::TiledArgs a, int32_t s, const int32_t* __restrict__ items, int32_t n_items) {
    using namespace chol;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= n_items) return;
    const int32_t it = items[blockIdx.x];
    const int b = it >> 16, i = (it >> 8) & 255, h = it & 255;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, qi = wave >> 1, qj = wave & 1;
    const int ld = a.blk_ld[b];
    double* A = a.M + a.blk_matoff[b];
    const int c0 = 2 * kBT * s;
    double* XS = lds;
    double* W = lds + 4 * kSub;
    v4d acc[2][2];
    zero_acc(acc);
    // h = 0: A_{i,0} X00^T;  h = 1: A_{i,0} X10^T + A_{i,1} X11^T
    stage_x(XS, A, ld, c0, c0 + kBT * h, h == 0, tid);
    stage64(W, A, ld, kBT * i, c0, tid);
    __syncthreads();
    for (int kc = 0; kc < 2; ++kc)
        if (h == 1 || kc <= qj) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    if (h == 1) {
        __syncthreads();
        stage_x(XS, A, ld, c0 + kBT, c0 + kBT, true, tid);
        stage64(W, A, ld, kBT * i, c0 + kBT, tid);
        __syncthreads();
        for (int kc = 0; kc <= qj; ++kc) mfma_tile(acc, W + (2 * qi + kc) * kSub, XS + (2 * qj + kc) * kSub, 1.0, lane);
    }
    store_acc(acc, A, ld, kBT * i + kT * qi, c0 + kBT * h + kT * qj, lane);
}

// trailing update of outer step s.  Items (block << 16) | (I << 8) | J0, -1 = padding: a run of
// tiles (I, J0 .. J0 + kJRun - 1) (clipped to the lower triangle).  The list starts with one
// item per active block for region s+1 (I = J0 = 2s + 2): that workgroup updates the region's
// tiles and factors it (lookahead); then per-XCD queues (item e runs on XCD e % 8; the runs of
// one tile row I of a block share an XCD, so L_I is served by its L2).
extern "C" __global__ __launch_bounds__(chol::kLargeThreads, 2) void dbslmm_tchol_trailing(
    chol::TiledArgs a, int32_t s, const int32_t* __restrict__ items, int32_t n_items) {
    using namespace chol;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= n_items) return;
    const int32_t it = items[blockIdx.x];
    if (it < 0) return;
    const int b = it >> 16, I = (it >> 8) & 255, J0 = it & 255;
    const int tid = threadIdx.x;
    const int m = a.blk_m[b], ld = a.blk_ld[b];
    const int T = (m + kBT - 1) / kBT, Tz = m / kBT;
    double* A = a.M + a.blk_matoff[b];
    const int c0 = 2 * kBT * s;
    const int k0n = 2 * s + 2;
    if (I == k0n && J0 == k0n) {          // region s+1: its tiles, then factor it
        update_run(A, ld, k0n, k0n, k0n, c0, lds, tid);
        if (k0n + 1 <= Tz) update_run(A, ld, k0n + 1, k0n, min(k0n + 1, T - 1), c0, lds, tid);
        const bool fail = diag128(A, ld, kBT * k0n, m, a.blk_ms[b], *a.dshift, lds, tid);
        if (fail && tid == 0) atomicMax(a.status + a.blk_id[b], DBSLMM_BLOCK_NOT_PD);
        return;
    }
    update_run(A, ld, I, J0, min(J0 + kJRun - 1, min(I, T - 1)), c0, lds, tid);
}

// backward step J (launches J = Kmax-1 .. 0).  v lives in y[row0 ..]; x_J overwrites v_J once
// it is known.  Workgroup = (block, 256 columns of [0, 64 J)):
//   x_J: read from y (written by the previous launch) -- or, at a block's first backward step
//        (J = T-1), computed by every workgroup from the z row;
//   v[c] -= sum_r L[64 J + r][c] x_J[r]   (column per thread, 64 independent loads);
//   the workgroup holding tile J-1 then has the final v_{J-1}: it forms x_{J-1} = X^T v_{J-1}
//   from the stored inverse, writes it over v_{J-1} and scatters beta for tile J-1.
namespace chol {
__device__ __forceinline__ void tile_x(const double* A, int ld, int c1, int jmax, const double* vsrc,
                                       double* D, double* vl, double* red, double* xs, int tid) {
    // D = stored rows c1.. of the diagonal tile (diagonal + upper = X^T), vl = v_J
    for (int e = tid; e < kBT * kBT; e += kLargeThreads) {
        const int r = e >> 6, c = e & 63;
        D[r * (kBT + 1) + c] = (r < jmax && c < jmax) ? A[static_cast<int64_t>(c1 + r) * ld + c1 + c] : 0.0;
    }
    if (tid < kBT) vl[tid] = tid < jmax ? vsrc[c1 + tid] : 0.0;
    __syncthreads();
    const int r = tid & 63, g = tid >> 6;
    double acc = 0.0;
    for (int c = r + g; c < kBT; c += 4) acc += D[r * (kBT + 1) + c] * vl[c];
    red[g * kBT + r] = acc;
    __syncthreads();
    if (tid < kBT) xs[tid] = (red[tid] + red[kBT + tid]) + (red[2 * kBT + tid] + red[3 * kBT + tid]);
    __syncthreads();
}
}  // namespace chol

extern "C" __global__ __launch_bounds__(chol::kLargeThreads) void dbslmm_tchol_backward(
    chol::TiledArgs a, int32_t J, const int32_t* __restrict__ act, const int32_t* __restrict__ pfx,
    int32_t n) {
    using namespace chol;
    __shared__ double D[kBT * (kBT + 1)];
    __shared__ double vl[kBT];
    __shared__ double red[4 * kBT];
    __shared__ double xs[kBT];
    const int item = blockIdx.x;
    if (item >= pfx[n]) return;
    const int s = find_item(pfx, n, item);
    const int b = act[s];
    const int chunk = item - pfx[s];
    const int tid = threadIdx.x;
    const int row0 = a.blk_row0[b], m = a.blk_m[b], ld = a.blk_ld[b];
    const double* A = a.M + a.blk_matoff[b];
    const int T = (m + kBT - 1) / kBT;
    const bool first = J == T - 1;
    const double* zrow = A + static_cast<int64_t>(m) * ld;
    double* v = a.y + row0;
    const int c1 = kBT * J, jmax = min(kBT, m - c1);
    const bool fail = a.status[a.blk_id[b]] >= DBSLMM_BLOCK_NOT_PD;
    auto put_beta = [&](int c0, int i, double x) {
        const double val = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
        const int o = a.slot_out[row0 + c0 + i];
        if (o >= 0) a.beta_s[o] = val;
        else a.beta_l[-1 - o] = val;
    };
    if (first) {
        tile_x(A, ld, c1, jmax, zrow, D, vl, red, xs, tid);
        if (chunk == 0 && tid < jmax) put_beta(c1, tid, xs[tid]);
    } else {
        if (tid < kBT) xs[tid] = tid < jmax ? v[c1 + tid] : 0.0;
        __syncthreads();
    }
    const int c = chunk * kLargeThreads + tid;
    if (c < c1) {
        const double* Lc = A + static_cast<int64_t>(c1) * ld + c;
        double part[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (jmax == kBT) {
#pragma unroll
            for (int r = 0; r < kBT; ++r) part[r & 7] += Lc[static_cast<int64_t>(r) * ld] * xs[r];
        } else {
            for (int r = 0; r < jmax; ++r) part[r & 7] += Lc[static_cast<int64_t>(r) * ld] * xs[r];
        }
        const double sum = ((part[0] + part[1]) + (part[2] + part[3])) + ((part[4] + part[5]) + (part[6] + part[7]));
        v[c] = (first ? zrow[c] : v[c]) - sum;
    }
    // the workgroup holding tile J-1 finishes it: x_{J-1} over v_{J-1}, beta
    if (J >= 1 && (c1 - 1) / kLargeThreads == chunk) {
        __syncthreads();
        __threadfence_block();
        const int c0 = c1 - kBT;
        tile_x(A, ld, c0, kBT, v, D, vl, red, xs, tid);
        if (tid < kBT) {
            v[c0 + tid] = xs[tid];
            put_beta(c0, tid, xs[tid]);
        }
    }
}
