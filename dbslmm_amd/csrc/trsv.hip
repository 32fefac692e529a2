// trsv.hip -- persistent blocked triangular solves with the tiled factors, and the Chebyshev
// iteration of h2f tuning built on them (included by plan.hip after chol_tiled.hip).
//
// h2f tuning (software/DBSLMM.R:205-219 runs dbslmm once per h2 factor) solves, per block,
// M_c x = z for several sigma_c, where M_c = Sigma + d_c P_s (d_c = 1/(sigma_c n), P_s = the
// small-SNP diagonal; scr/dbslmmfit.cpp:705-712).  For the tiled (big) blocks only one copy, the
// base M_b, is factored; every other copy iterates on
//     M_b x = z - delta P_s x,      delta = d_c - d_b,
// accelerated by Chebyshev with M_b as the preconditioner.  Sigma = tau X^T X / n_ref +
// (1 - tau) I >= (1 - tau) I, so the Schur complement of M_b on the small SNPs is
// >= (d_b + 1 - tau) I and the spectrum of M_b^{-1} M_c lies in [1, 1 + delta / (d_b + 1 - tau)]
// (delta > 0) or [1 + delta / (d_b + 1 - tau), 1] (delta < 0) -- an interval that does not
// depend on the data, so the iteration count is fixed on the host (8 for h2f = 0.8 / 1 / 1.2
// at a relative error of 1e-10) and no inner products are needed.  M_b d is carried by the recurrence
// s = alpha s + beta r (M_b z = r), so one iteration is one forward and one backward
// substitution; the Chebyshev update is the backward kernel's epilogue.
//
// The substitutions are persistent kernels: one workgroup per CU takes work items (64-row tiles of
// all tiled blocks) from a ticket counter in dependency order.  A tile's result is handed to the
// workgroups of the later tiles of its block inside the launch.  A workgroup only waits for
// tiles with smaller tickets, held by running workgroups: no deadlock for any residency.
// Hand-off: payload stored sc1 (agent-scope relaxed atomic stores), every storing wave drained, a
// workgroup barrier, one lane's sc1 flag store (the launch's epoch); the consumer polls the flag
// (sc1 load) and reads the payload with sc1 loads only (MI355X_MICROARCH.md, inter-workgroup
// visibility, first row of the sc1 table: one workgroup per CU, which the > 80 KiB LDS request
// enforces).  (Measured: "data is the flag" granules, R2, were slower here.)  Flags are never
// cleared (epochs grow with every launch) and the ticket counter is reset by its last drawer, so
// a launch needs no memset.  Ticket order: the tile's position relative to its block's
// length, so the long dependency chains of the biggest blocks advance with the bulk.
//
// Wave roles: 8 streaming waves read L with a deep prefetch and never touch the hand-offs; one
// control wave takes the handed-off granules and stages the values into an LDS ring (ready
// counter in LDS).  vmcnt counts in order per wave, so a hand-off load in a streaming wave would
// drain its whole L prefetch; split this way the streaming waves keep ~128 KiB per CU in flight
// and the hand-off latency overlaps the stream.  A launch is bound by the dependency chain of the
// longest block (about 3.8 us per 64-row tile alone, 5.7 us under the bulk streaming: drain +
// flag + poll + payload round trips and the tile's reductions) and by the streaming bandwidth.
//
// Factor layout (chol_tiled.hip): strict lower = L; each 64 x 64 diagonal tile holds, on and
// above its diagonal, X^T with X = L_kk^{-1}; every other 64 x 64 tile of the upper triangle holds
// the transposed L tile (L^T), so the backward substitution streams rows like the forward one.
namespace trsv {

constexpr int kT = 64;                       // tile rows = the stored diagonal inverse blocks
constexpr int kSW = 8;                       // streaming waves (rows 8 w .. 8 w + 7 of a tile)
constexpr int kThreads = (kSW + 1) * 64;     // + the control wave
constexpr int kPF = 4;                       // column tiles of L in flight per streaming wave
constexpr int kMaxR = 2;                     // right-hand sides per launch
constexpr int kNS = 16;                      // LDS ring slots (tiles) of handed-off vectors
constexpr int kGrp = 8;                      // tiles the control wave stages per round trip
constexpr size_t kLdsBytes = 96 * 1024;      // one workgroup per CU (sc1 hand-off condition)
// the larger carve (backward): ring + w + z + transpose + ring words
static_assert((kNS * kT * kMaxR + 2 * kT * kMaxR + kSW * 8 * kMaxR * (kT + 1)) * sizeof(double) + 64 <= kLdsBytes,
              "TRSV LDS carve");

struct Args {
    const double* M;             // the factored base copy
    const int64_t* matoff;
    const int32_t* ld;
    const int32_t* m;
    const int32_t* ms;
    const int32_t* row0;
    const int32_t* blk_id;
    const int32_t* slot_out;
    const int32_t* items;        // (plan block, tile) pairs in dependency order
    int32_t n_items;
    int32_t grid;                // workgroups of the launch (the last ticket drawer resets ctr)
    const int32_t* foff;         // plan block -> its first tile flag
    int32_t* flags;              // tile t of this launch is done when flags[t] == epoch
    int32_t epoch;               // grows with every launch (flags are never cleared)
    int32_t* ctr;                // ticket counter: 0 at launch, reset to 0 by its last drawer
    int32_t* err;                // set when a bounded wait gives up
    int64_t vs;                  // per right-hand-side stride of the vectors (n_slots)
    const double* src;           // forward: r, backward: y
    double* dst;                 // forward: y, backward: z (handed off inside the launch)
    // Chebyshev epilogue (backward)
    double* X;
    double* R;
    double* D;
    double* S;
    const double* coef;          // [NR][3] {alpha, beta, delta} of this iteration
    int32_t last;                // last iteration: write beta, skip the state update
    double inv_sqrt_n;
    double* beta_s;              // copy c's betas at beta_s + cix[c] * ns_stride
    double* beta_l;
    int64_t ns_stride, nl_stride;
    int32_t cix[kMaxR];
    const int32_t* status;       // the base copy's block status
    int32_t mode;                // backward: 0 Chebyshev epilogue; 1 plain solve of the factored
                                 // system (y = the matrix's z row, x -> X, beta of copy cix[0])
    unsigned long long* stamps;  // diagnostic build (DBSLMM_DIAG, env DBSLMM_TRSV_STAMPS): per tile of block stamp_b,
    int32_t stamp_b;             // 100 MHz times [claim, last hand-off staged, stream done, publish]
};
__device__ __forceinline__ void stamp(const Args& a, int b, int I, int k) {
#ifdef DBSLMM_DIAG
    if (a.stamps && b == a.stamp_b) a.stamps[8 * I + k] = __builtin_amdgcn_s_memrealtime();
#endif
}

// LDS control words of the ring
struct Ring {
    int ticket;
    int ready;                   // tiles staged so far (control wave -> streaming waves)
    int done[kSW];               // tiles consumed so far, per streaming wave
};

__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool flag_set(const int32_t* f, int32_t epoch) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
}
__device__ __forceinline__ void publish(int32_t* f, int32_t epoch, int tid) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
    __syncthreads();
    if (tid == 0) __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int lds_get(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_put(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ double red8(double v) {   // sum over an aligned group of 8 lanes
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    return v + __shfl_xor(v, 4);
}
// every workgroup draws tickets until one is past the list; the last of those resets the counter.
// Also resets the ring words for the next item.
__device__ __forceinline__ int take_ticket(const Args& a, Ring* rg, int tid) {
    if (tid == 0) {
        const int t = atomicAdd(a.ctr, 1);
        if (t == a.n_items + a.grid - 1) __hip_atomic_store(a.ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rg->ticket = t;
        rg->ready = 0;
#pragma unroll
        for (int w = 0; w < kSW; ++w) rg->done[w] = 0;
    }
    __syncthreads();
    const int t = rg->ticket;
    __syncthreads();
    return t;
}
// Control wave: stage the handed-off vectors of tiles j_0, j_0 + dj, ... (n tiles, rows of 64,
// values past m zero) into ring slots (position % kNS), in rounds of up to kGrp tiles: lane u
// polls tile p + u's flag, the round takes the done prefix (at least tile p), then one sc1 load
// per lane (= row) and right-hand side per tile, and publishes the new ready count.  A slot is
// reused only when every streaming wave has consumed the tile that held it.
template <int NR>
__device__ __forceinline__ void control(const Args& a, Ring* rg, double* ring, const int32_t* flag, int g0,
                                        int m, int j0, int dj, int n, int lane) {
    for (int p = 0; p < n;) {
        for (;;) {   // slot reuse: position p + kGrp - 1 must not overrun the slowest streaming wave
            int mn = n;
#pragma unroll
            for (int w = 0; w < kSW; ++w) mn = min(mn, lds_get(&rg->done[w]));
            if (p + kGrp - 1 < mn + kNS) break;
            __builtin_amdgcn_s_sleep(1);
        }
        int cnt = 0;
        for (long spins = 0;; ++spins) {
            bool ok = false;
            if (lane < kGrp && p + lane < n) ok = flag_set(flag + j0 + (p + lane) * dj, a.epoch);
            cnt = __builtin_ctzll(~__ballot(ok));   // length of the done prefix
            if (cnt > 0) break;
            __builtin_amdgcn_s_sleep(1);
            if (spins > (1L << 25)) {   // bounded (about a second): report and proceed
                if (lane == 0) atomicOr(a.err, 1);
                cnt = 1;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // hand-off loads stay behind the poll
        double v[kGrp][NR];
#pragma unroll
        for (int u = 0; u < kGrp; ++u)
            if (u < cnt) {
                const int gr = kT * (j0 + (p + u) * dj) + lane;
#pragma unroll
                for (int c = 0; c < NR; ++c) v[u][c] = gr < m ? ld_sc1(a.dst + c * a.vs + g0 + gr) : 0.0;
            }
#pragma unroll
        for (int u = 0; u < kGrp; ++u)
            if (u < cnt) {
#pragma unroll
                for (int c = 0; c < NR; ++c) ring[(((p + u) % kNS) * kT + lane) * NR + c] = v[u][c];
            }
        p += cnt;
        if (lane == 0) lds_put(&rg->ready, p);   // release: the ring writes land first
    }
}
// streaming wave: wait until position p is staged
__device__ __forceinline__ void wait_ready(Ring* rg, int p) {
    while (lds_get(&rg->ready) <= p) __builtin_amdgcn_s_sleep(1);
}

}  // namespace trsv

// Forward substitution L y = r (NR right-hand sides), one 64-row tile per work item.  Streaming
// wave w owns rows 8 w .. 8 w + 7, lane = column of L_IJ (512-B coalesced rows, kPF tiles in
// flight); y_J comes from the control wave's LDS ring.  Diagonal: y_I = X_I v with X_I^T stored
// on and above the diagonal tile's diagonal.
template <int NR>
__global__ __launch_bounds__(trsv::kThreads, 1) void dbslmm_trsv_fwd(trsv::Args a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* ring = lds;                       // [kNS][64][NR]
    double* vs = ring + kNS * kT * NR;        // [64][NR]: r_I - sum_J L_IJ y_J
    double* rt = vs + kT * NR;                // [8 waves][8 NR][65]: lane partial sums (transpose)
    Ring* rg = reinterpret_cast<Ring*>(rt + kSW * 8 * NR * (kT + 1));
    const int tid = threadIdx.x, row = tid >> 3, part = tid & 7, lane = tid & 63, wave = tid >> 6;
    constexpr int kV = 8 * NR, kG = kT / kV;  // row sums per wave; lanes per row sum
    for (;;) {
        const int it = take_ticket(a, rg, tid);
        if (it >= a.n_items) break;
        const int b = a.items[2 * it], I = a.items[2 * it + 1];
        const int m = a.m[b], ld = a.ld[b], g0 = a.row0[b];
        const double* A = a.M + a.matoff[b];
        const int r0 = kT * I, jmax = min(kT, m - r0);
        const int32_t* flag = a.flags + a.foff[b];
        double xd[8];
        if (tid == 0) stamp(a, b, I, 0);
        if (wave == kSW) {
            control<NR>(a, rg, ring, flag, g0, m, 0, 1, I, lane);
            if (lane == 0) stamp(a, b, I, 1);
        } else {
            // xd[k] = X[row][8 part + k] = A(r0 + 8 part + k, r0 + row) (8 part + k <= row)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int rr = 8 * part + k;
                const double x = A[static_cast<int64_t>(r0 + rr) * ld + r0 + row];   // inside ld x ld
                xd[k] = (rr <= row && row < jmax) ? x : 0.0;
            }
            // this lane's share of r_I, read now (off the dependency chain): value v = lane / kG
            const int vv = lane / kG, vk = vv / NR, vc = vv - vk * NR, vr = 8 * wave + vk;
            const double rsrc = vr < jmax ? a.src[vc * a.vs + g0 + r0 + vr] : 0.0;
            const double* Lw = A + static_cast<int64_t>(r0 + 8 * wave) * ld + lane;
            double acc[8][NR];
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) acc[k][c] = 0.0;
            double lr[kPF][8];
#pragma unroll
            for (int u = 0; u < kPF; ++u)
                if (u < I) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) lr[u][k] = Lw[static_cast<int64_t>(k) * ld + kT * u];
                }
            for (int J = 0; J < I; J += kPF) {
#pragma unroll
                for (int u = 0; u < kPF; ++u) {
                    const int j = J + u;
                    if (j < I) {
                        wait_ready(rg, j);
                        const double* y = ring + ((j % kNS) * kT + lane) * NR;
#pragma unroll
                        for (int k = 0; k < 8; ++k)
#pragma unroll
                            for (int c = 0; c < NR; ++c) acc[k][c] += lr[u][k] * y[c];
                        if (lane == 0) lds_put(&rg->done[wave], j + 1);
                        if (j + kPF < I) {
#pragma unroll
                            for (int k = 0; k < 8; ++k) lr[u][k] = Lw[static_cast<int64_t>(k) * ld + kT * (j + kPF)];
                        }
                    }
                }
            }
            if (tid == 0) stamp(a, b, I, 2);
            // row sums over the 64 lanes: transpose through LDS (wave-private region), then lane
            // group g of kG lanes sums value v = lane / kG over 64 / kG lanes each
            double* rw = rt + wave * kV * (kT + 1);
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) rw[(k * NR + c) * (kT + 1) + lane] = acc[k][c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double sum = 0.0;
            const int q0 = (lane % kG) * (kT / kG);
#pragma unroll
            for (int q = 0; q < kT / kG; ++q) sum += rw[vv * (kT + 1) + q0 + q];
#pragma unroll
            for (int sft = 1; sft < kG; sft <<= 1) sum += __shfl_xor(sum, sft);
            if (tid == 0) stamp(a, b, I, 4);
            if (lane % kG == 0) vs[vr * NR + vc] = vr < jmax ? rsrc - sum : 0.0;
        }
        __syncthreads();
        if (tid == 0) stamp(a, b, I, 5);
        if (wave < kSW) {
            double y[NR];
#pragma unroll
            for (int c = 0; c < NR; ++c) y[c] = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) y[c] += xd[k] * vs[(8 * part + k) * NR + c];
#pragma unroll
            for (int c = 0; c < NR; ++c) y[c] = red8(y[c]);
            if (part == 0 && row < jmax) {
#pragma unroll
                for (int c = 0; c < NR; ++c) st_sc1(a.dst + c * a.vs + g0 + r0 + row, y[c]);
            }
        }
        if (tid == 0) stamp(a, b, I, 6);
        publish(a.flags + a.foff[b] + I, a.epoch, tid);   // (its barrier also frees vs)
        if (tid == 0) stamp(a, b, I, 3);
    }
}

// Backward substitution L^T z = y, then the Chebyshev update of the tile's rows.  It reads L^T
// from the upper triangle (the panel / region kernels store each off-diagonal 64 x 64 tile of L
// transposed there too), so it streams rows exactly like the forward kernel: wave w owns rows
// 8 w .. 8 w + 7 of tile I, lane = column of the later tile J (J = T - 1 down to I + 1),
// acc += (L^T)_IJ z_J with z_J from the control wave's LDS ring, then row sums through the
// wave-private LDS transpose.
template <int NR>
__global__ __launch_bounds__(trsv::kThreads, 1) void dbslmm_trsv_bwd(trsv::Args a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* ring = lds;                       // [kNS][64][NR]
    double* ws = ring + kNS * kT * NR;        // [64][NR]: y_I - sum_J (L^T)_IJ z_J
    double* zt = ws + kT * NR;                // [64][NR] this tile's z
    double* rt = zt + kT * NR;                // [8 waves][8 NR][65]: lane partial sums (transpose)
    Ring* rg = reinterpret_cast<Ring*>(rt + kSW * 8 * NR * (kT + 1));
    const int tid = threadIdx.x, row = tid >> 3, part = tid & 7, wave = tid >> 6, lane = tid & 63;
    constexpr int kV = 8 * NR, kG = kT / kV;  // row sums per wave; lanes per row sum
    for (;;) {
        const int it = take_ticket(a, rg, tid);
        if (it >= a.n_items) break;
        const int b = a.items[2 * it], I = a.items[2 * it + 1];
        const int m = a.m[b], ld = a.ld[b], g0 = a.row0[b];
        const int T = (m + kT - 1) / kT;
        const double* A = a.M + a.matoff[b];
        const int r0 = kT * I, jmax = min(kT, m - r0);
        const int32_t* flag = a.flags + a.foff[b];
        const int cnt = T - 1 - I;                // later tiles, taken from the last one down
        double xd[8];
        if (wave == kSW) {
            control<NR>(a, rg, ring, flag, g0, m, T - 1, -1, cnt, lane);
        } else {
            // xd[k] = X^T[row][8 part + k] = A(r0 + row, r0 + 8 part + k), on and above the diagonal
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int q = 8 * part + k;
                const double x = A[static_cast<int64_t>(r0 + row) * ld + r0 + q];
                xd[k] = (q >= row && q < jmax) ? x : 0.0;
            }
            // this lane's share of y_I (value v = lane / kG), read now (off the dependency chain)
            const int vv = lane / kG, vk = vv / NR, vc = vv - vk * NR, vr = 8 * wave + vk;
            const double ysrc = vr >= jmax ? 0.0
                                : a.mode ? A[static_cast<int64_t>(m) * ld + r0 + vr]   // bordered row m: y = L^-1 z
                                         : a.src[vc * a.vs + g0 + r0 + vr];
            const double* Uw = A + static_cast<int64_t>(r0 + 8 * wave) * ld + lane;   // rows of tile I
            double acc[8][NR];
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) acc[k][c] = 0.0;
            double lr[kPF][8];
            auto issue = [&](int u, int t) {
                const int cj = kT * (T - 1 - t);          // columns of tile J: cj + lane < 64 T <= ld
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const double x = Uw[static_cast<int64_t>(k) * ld + cj];
                    lr[u][k] = cj + lane < m ? x : 0.0;   // past m: bordered row / padding
                }
            };
#pragma unroll
            for (int u = 0; u < kPF; ++u)
                if (u < cnt) issue(u, u);
            for (int t0 = 0; t0 < cnt; t0 += kPF) {
#pragma unroll
                for (int u = 0; u < kPF; ++u) {
                    const int t = t0 + u;
                    if (t < cnt) {
                        wait_ready(rg, t);
                        const double* z = ring + ((t % kNS) * kT + lane) * NR;
#pragma unroll
                        for (int k = 0; k < 8; ++k)
#pragma unroll
                            for (int c = 0; c < NR; ++c) acc[k][c] += lr[u][k] * z[c];
                        if (lane == 0) lds_put(&rg->done[wave], t + 1);
                        if (t + kPF < cnt) issue(u, t + kPF);
                    }
                }
            }
            double* rw = rt + wave * kV * (kT + 1);
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) rw[(k * NR + c) * (kT + 1) + lane] = acc[k][c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double sum = 0.0;
            const int q0 = (lane % kG) * (kT / kG);
#pragma unroll
            for (int q = 0; q < kT / kG; ++q) sum += rw[vv * (kT + 1) + q0 + q];
#pragma unroll
            for (int sft = 1; sft < kG; sft <<= 1) sum += __shfl_xor(sum, sft);
            if (lane % kG == 0) ws[vr * NR + vc] = vr < jmax ? ysrc - sum : 0.0;
        }
        __syncthreads();
        if (wave < kSW) {
            double z[NR];
#pragma unroll
            for (int c = 0; c < NR; ++c) z[c] = 0.0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < NR; ++c) z[c] += xd[k] * ws[(8 * part + k) * NR + c];
#pragma unroll
            for (int c = 0; c < NR; ++c) z[c] = red8(z[c]);
            if (part == 0 && row < jmax) {
#pragma unroll
                for (int c = 0; c < NR; ++c) {
                    st_sc1(a.dst + c * a.vs + g0 + r0 + row, z[c]);
                    zt[row * NR + c] = z[c];
                }
            }
        }
        publish(a.flags + a.foff[b] + I, a.epoch, tid);
        // Chebyshev epilogue: d = alpha d + beta z; s = alpha s + beta r; x += d;
        // r -= s + delta P_s d  (this tile's rows; read and written only here in this launch)
        if (tid < kT * NR) {
            const int rr = tid / NR, c = tid - rr * NR;
            if (rr < jmax) {
                const int i = r0 + rr;
                const int64_t gi = g0 + i;
                const bool small = i < a.ms[b];
                const bool fail = a.status[a.blk_id[b]] >= DBSLMM_BLOCK_NOT_PD;
                if (a.mode) {   // plain solve: x and beta (NR = 1)
                    const double x = zt[tid];
                    a.X[gi] = x;
                    const double v = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
                    const int so = a.slot_out[gi];
                    if (so >= 0) a.beta_s[a.cix[0] * a.ns_stride + so] = v;
                    else a.beta_l[a.cix[0] * a.nl_stride - 1 - so] = v;
                    continue;
                }
                const double al = a.coef[3 * c], be = a.coef[3 * c + 1], de = a.coef[3 * c + 2];
                const int64_t o = c * a.vs + gi;
                const double d = al * a.D[o] + be * zt[tid];
                const double x = a.X[o] + d;
                if (a.last) {
                    const double v = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
                    const int so = a.slot_out[gi];
                    if (so >= 0) a.beta_s[a.cix[c] * a.ns_stride + so] = v;
                    else a.beta_l[a.cix[c] * a.nl_stride - 1 - so] = v;
                } else {
                    const double r = a.R[o];
                    const double s2 = al * a.S[o] + be * r;
                    a.D[o] = d;
                    a.S[o] = s2;
                    a.X[o] = x;
                    a.R[o] = r - s2 - (small ? de * d : 0.0);
                }
            }
        }
    }
}

// Chebyshev start for a copy group (coef0 = its iteration-0 {alpha, beta, delta}): x = x_b (the
// base copy's solution), r = z - M_c x_b = -delta P_s x_b, d = s = 0; the copies' block status =
// the base's.  One workgroup per tiled block.
extern "C" __global__ __launch_bounds__(256) void dbslmm_cheb_init(
    const int32_t* __restrict__ tb, const int32_t* __restrict__ row0, const int32_t* __restrict__ mv,
    const int32_t* __restrict__ msv, const int32_t* __restrict__ blk_id, const double* __restrict__ xbase,
    const double* __restrict__ coef0, int nr, int64_t vs, double* X, double* R, double* D, double* S,
    const int32_t* __restrict__ st_base, int32_t* st, int64_t st_stride, int c0, int c1) {
    const int b = tb[blockIdx.x];
    const int g0 = row0[b], m = mv[b], ms = msv[b];
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const double xb = xbase[g0 + i];
        for (int c = 0; c < nr; ++c) {
            const int64_t o = c * vs + g0 + i;
            X[o] = xb;
            R[o] = i < ms ? -coef0[3 * c + 2] * xb : 0.0;
            D[o] = 0.0;
            S[o] = 0.0;
        }
    }
    if (threadIdx.x < nr) st[(threadIdx.x == 0 ? c0 : c1) * st_stride + blk_id[b]] = st_base[blk_id[b]];
}
