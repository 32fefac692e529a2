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
                                 // system (y = the matrix's z row, x -> X, beta of copy cix[0]);
                                 // 2 CG: z only (dbslmm_cg_update does the block's update)
    const int32_t* conv;         // CG: per plan block, nonzero once every copy has converged (its
                                 // items are skipped); nullptr otherwise
    unsigned long long* stamps;  // diagnostic build (DBSLMM_DIAG, env DBSLMM_TRSV_STAMPS): per tile of block stamp_b,
    int32_t stamp_b;             // 100 MHz times [claim, last hand-off staged, stream done, publish]
    // all passes of a Chebyshev group in one launch (dbslmm_trsv_cheb): pass p = 2 k (+1 for the
    // backward substitution) of iteration k runs at epoch + p; the vectors live in Y (forward
    // result), Z (backward result) and X / R / D / S; `epi` flags a tile's Chebyshev update
    int32_t fused;               // 1: the item waits for its own inputs (no launch boundary) and
                                 // reads the per-pass vectors with sc1 loads
    int32_t iters;               // K
    int32_t* epi;                // per tile: epoch of the backward pass whose update is stored
    double* Y;
    double* Z;
};
// the per-pass inputs of an item (the separate forward / backward launches take them from Args)
struct Pass {
    int32_t epoch;
    const double* src;
    double* dst;
    const double* coef;
    int32_t last;
};
__device__ __forceinline__ Pass pass_of(const Args& a) { return Pass{a.epoch, a.src, a.dst, a.coef, a.last}; }

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
// flags only grow (epochs), and a tile's hand-off data of pass p is overwritten only at pass p + 2,
// after every consumer of pass p: ">=" serves consumers that run late
__device__ __forceinline__ bool flag_set(const int32_t* f, int32_t epoch) {
    return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= epoch;
}
// the calling wave waits for flag f >= epoch (bounded; every lane polls the same word: one
// request per poll), then an acquire fence for the wave's later loads
__device__ __forceinline__ void wave_wait_flag(const Args& a, const int32_t* f, int32_t epoch) {
    for (long spins = 0; !flag_set(f, epoch); ++spins) {
        __builtin_amdgcn_s_sleep(1);
        if (spins > (1L << 25) ||
            ((spins & 1023) == 1023 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            atomicOr(a.err, 1);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
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
    // tid made opaque per call: a loop-invariant "tid == 0" at the loop head was jump-threaded
    // into a lane-divergent inner loop around the barriers below (a deadlock)
    asm volatile("" : "+v"(tid));
    if (tid == 0) {
        const int t = atomicAdd(a.ctr, 1);
        if (t == a.n_items + a.grid - 1) __hip_atomic_store(a.ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        rg->ticket = t;
        rg->ready = 0;
#pragma unroll
        for (int w = 0; w < kSW; ++w) rg->done[w] = 0;
    }
    __syncthreads();
    // uniform by construction; readfirstlane makes it so for the compiler too (scalar loop exit
    // and item branches -- a "divergent" exit around the barriers of the fused kernel's two item
    // kinds was structurised into a loop that deadlocked)
    const int t = __builtin_amdgcn_readfirstlane(rg->ticket);
    __syncthreads();
    return t;
}
// Control wave: stage the handed-off vectors of tiles j_0, j_0 + dj, ... (n tiles, rows of 64,
// values past m zero) into ring slots (position % kNS), in rounds of up to kGrp tiles: lane u
// polls tile p + u's flag, the round takes the done prefix (at least tile p), then one sc1 load
// per lane (= row) and right-hand side per tile, and publishes the new ready count.  A slot is
// reused only when every streaming wave has consumed the tile that held it.
template <int NR>
__device__ __forceinline__ void control(const Args& a, int32_t epoch, const double* dst, Ring* rg, double* ring,
                                        const int32_t* flag, int g0, int m, int j0, int dj, int n, int lane) {
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
            if (lane < kGrp && p + lane < n) ok = flag_set(flag + j0 + (p + lane) * dj, epoch);
            cnt = __builtin_ctzll(~__ballot(ok));   // length of the done prefix
            if (cnt > 0) break;
            __builtin_amdgcn_s_sleep(1);
            // bounded (about a second): report and proceed; once any wait has given up, every
            // later wait of the launch gives up at once (the launch ends promptly, results invalid)
            if (spins > (1L << 25) ||
                ((spins & 1023) == 1023 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
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
                for (int c = 0; c < NR; ++c) v[u][c] = gr < m ? ld_sc1(dst + c * a.vs + g0 + gr) : 0.0;
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

// One 64-row tile of a substitution (NR right-hand sides).  Forward (L y = r): the later rows
// of tile I against the earlier tiles J < I of L.  Backward (L^T z = y): rows of tile I of L^T,
// read from the upper triangle (the panel / region kernels store each off-diagonal 64 x 64 tile
// of L transposed there too), against the later tiles J = T - 1 down to I + 1 -- so both stream
// rows the same way: wave w owns rows 8 w .. 8 w + 7 of tile I, lane = column of tile J
// (512-B coalesced rows, kPF tiles in flight), acc += tile_IJ v_J with v_J from the control
// wave's LDS ring, row sums through a wave-private LDS transpose, then the diagonal: v_I = X_I w
// (forward; X_I^T stored on and above the diagonal tile's diagonal) or X_I^T w (backward).
// One body for both directions: the fused Chebyshev kernel runs both kinds of item in one ticket
// loop, and two inlined bodies there were structurised into a lane-divergent loop around their
// barriers (deadlock); the direction is a uniform runtime branch here.
//   wait_f / wait_e: (fused passes) the item's own input is ready when *wait_f >= wait_e
//   (forward: the previous backward pass's Chebyshev update of r_I, in a.epi; backward: y_I)
//   epi: (backward) the Chebyshev update of the tile's rows after the hand-off
template <int NR>
__device__ __forceinline__ void tile_item(const trsv::Args& a, const trsv::Pass& ps, trsv::Ring* rg, double* lds,
                                          int b, int I, bool bwd, const int32_t* wait_f, int32_t wait_e, int tid) {
    using namespace trsv;
    double* ring = lds;                       // [kNS][64][NR]
    double* ws = ring + kNS * kT * NR;        // [64][NR]: v_I's source minus sum_J tile_IJ v_J
    double* zt = ws + kT * NR;                // [64][NR]: this tile's result (backward epilogue)
    double* rt = zt + kT * NR;                // [8 waves][8 NR][65]: lane partial sums (transpose)
    const int row = tid >> 3, part = tid & 7, wave = tid >> 6, lane = tid & 63;
    constexpr int kV = 8 * NR, kG = kT / kV;  // row sums per wave; lanes per row sum
    const int m = a.m[b], ld = a.ld[b], g0 = a.row0[b];
    const int T = (m + kT - 1) / kT;
    const double* A = a.M + a.matoff[b];
    const int r0 = kT * I, jmax = min(kT, m - r0);
    const int32_t* flag = a.flags + a.foff[b];
    const int cnt = bwd ? T - 1 - I : I;      // tiles streamed (backward: from the last one down)
    if (tid == 0) stamp(a, b, I, 0);
    double xd[8];
    if (wave == kSW) {
        control<NR>(a, ps.epoch, ps.dst, rg, ring, flag, g0, m, bwd ? T - 1 : 0, bwd ? -1 : 1, cnt, lane);
        if (lane == 0) stamp(a, b, I, 1);
    } else {
        // forward: xd[k] = X[row][8 part + k] = A(r0 + 8 part + k, r0 + row) (8 part + k <= row);
        // backward: xd[k] = X^T[row][8 part + k] = A(r0 + row, r0 + 8 part + k) (on and above)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int q = 8 * part + k;
            const int64_t o = bwd ? static_cast<int64_t>(r0 + row) * ld + r0 + q
                                  : static_cast<int64_t>(r0 + q) * ld + r0 + row;   // inside ld x ld
            const double x = A[o];
            xd[k] = (bwd ? (q >= row && q < jmax) : (q <= row && row < jmax)) ? x : 0.0;
        }
        // this lane's share of the source (value v = lane / kG), read now (off the dependency
        // chain: the control wave meanwhile polls the hand-offs; fused passes wait for it here)
        if (wait_e > 0) wave_wait_flag(a, wait_f, wait_e);
        const int vv = lane / kG, vk = vv / NR, vc = vv - vk * NR, vr = 8 * wave + vk;
        const double* sp = ps.src + vc * a.vs + g0 + r0 + vr;
        const double src = vr >= jmax ? 0.0
                           : (bwd && a.mode == 1) ? A[static_cast<int64_t>(m) * ld + r0 + vr]   // bordered row m: y = L^-1 z
                                             : a.fused ? ld_sc1(sp) : *sp;
        const double* Lw = A + static_cast<int64_t>(r0 + 8 * wave) * ld + lane;   // rows of tile I
        double acc[8][NR];
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int c = 0; c < NR; ++c) acc[k][c] = 0.0;
        double lr[kPF][8];
        auto issue = [&](int u, int t) {
            const int cj = kT * (bwd ? T - 1 - t : t);   // columns of tile J: cj + lane < 64 T <= ld
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double x = Lw[static_cast<int64_t>(k) * ld + cj];
                lr[u][k] = cj + lane < m ? x : 0.0;      // past m: bordered row / padding
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
                    const double* v = ring + ((t % kNS) * kT + lane) * NR;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
#pragma unroll
                        for (int c = 0; c < NR; ++c) acc[k][c] += lr[u][k] * v[c];
                    if (lane == 0) lds_put(&rg->done[wave], t + 1);
                    if (t + kPF < cnt) issue(u, t + kPF);
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
        if (lane % kG == 0) ws[vr * NR + vc] = vr < jmax ? src - sum : 0.0;
    }
    __syncthreads();
    if (tid == 0) stamp(a, b, I, 5);
    if (wave < kSW) {
        double v[NR];
#pragma unroll
        for (int c = 0; c < NR; ++c) v[c] = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int c = 0; c < NR; ++c) v[c] += xd[k] * ws[(8 * part + k) * NR + c];
#pragma unroll
        for (int c = 0; c < NR; ++c) v[c] = red8(v[c]);
        if (part == 0 && row < jmax) {
#pragma unroll
            for (int c = 0; c < NR; ++c) {
                st_sc1(ps.dst + c * a.vs + g0 + r0 + row, v[c]);
                zt[row * NR + c] = v[c];
            }
        }
    }
    if (tid == 0) stamp(a, b, I, 6);
    publish(a.flags + a.foff[b] + I, ps.epoch, tid);   // (its barrier also frees ws and orders zt)
    if (tid == 0) stamp(a, b, I, 3);
    if (!bwd || a.mode == 2) return;
    // Chebyshev epilogue: d = alpha d + beta z; s = alpha s + beta r; x += d;
    // r -= s + delta P_s d  (this tile's rows; read and written only here in this pass)
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
            } else {
                const double al = ps.coef[3 * c], be = ps.coef[3 * c + 1], de = ps.coef[3 * c + 2];
                const int64_t o = c * a.vs + gi;
                // fused passes: the state of this tile was written by another workgroup's update
                // in the previous pass (sc1 both ways); separate launches: plain accesses
                auto ld_v = [&](const double* q) { return a.fused ? ld_sc1(q) : *q; };
                auto st_v = [&](double* q, double v) { if (a.fused) st_sc1(q, v); else *q = v; };
                const double d = al * ld_v(a.D + o) + be * zt[tid];
                const double x = ld_v(a.X + o) + d;
                if (ps.last) {
                    const double v = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
                    const int so = a.slot_out[gi];
                    if (so >= 0) a.beta_s[a.cix[c] * a.ns_stride + so] = v;
                    else a.beta_l[a.cix[c] * a.nl_stride - 1 - so] = v;
                } else {
                    const double r = ld_v(a.R + o);
                    const double s2 = al * ld_v(a.S + o) + be * r;
                    st_v(a.D + o, d);
                    st_v(a.S + o, s2);
                    st_v(a.X + o, x);
                    st_v(a.R + o, r - s2 - (small ? de * d : 0.0));
                }
            }
        }
    }
    if (a.fused && !ps.last) publish(a.epi + a.foff[b] + I, ps.epoch, tid);   // the update is stored
}

template <int NR>
__global__ __launch_bounds__(trsv::kThreads, 1) void dbslmm_trsv_fwd(trsv::Args a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Ring* rg = reinterpret_cast<Ring*>(lds + kNS * kT * NR + 2 * kT * NR + kSW * 8 * NR * (kT + 1));
    const int tid = threadIdx.x;
    for (;;) {
        const int it = take_ticket(a, rg, tid);
        if (it >= a.n_items) break;
        const int b = __builtin_amdgcn_readfirstlane(a.items[2 * it]);
        const int I = __builtin_amdgcn_readfirstlane(a.items[2 * it + 1]);
        if (a.conv && __builtin_amdgcn_readfirstlane(a.conv[b]) != 0) continue;   // CG: converged block
        tile_item<NR>(a, pass_of(a), rg, lds, b, I, false, nullptr, 0, tid);
    }
}

template <int NR>
__global__ __launch_bounds__(trsv::kThreads, 1) void dbslmm_trsv_bwd(trsv::Args a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Ring* rg = reinterpret_cast<Ring*>(lds + kNS * kT * NR + 2 * kT * NR + kSW * 8 * NR * (kT + 1));
    const int tid = threadIdx.x;
    for (;;) {
        const int it = take_ticket(a, rg, tid);
        if (it >= a.n_items) break;
        const int b = __builtin_amdgcn_readfirstlane(a.items[2 * it]);
        const int I = __builtin_amdgcn_readfirstlane(a.items[2 * it + 1]);
        if (a.conv && __builtin_amdgcn_readfirstlane(a.conv[b]) != 0) continue;   // CG: converged block
        tile_item<NR>(a, pass_of(a), rg, lds, b, I, true, nullptr, 0, tid);
    }
}

// Every pass of a Chebyshev group in one persistent launch: items (block | pass << 16, tile) in
// an order where each block's items follow its own dependency order (passes in sequence, tiles
// in their substitution order) -- so every wait is on a smaller ticket (deadlock-free) -- while
// the blocks are interleaved by a timing model: the small blocks' many iterations stream at the
// memory bandwidth while the largest blocks' long chains advance beside them, instead of every
// block waiting for the largest one at the end of each pass (plan.hip, build_cheb_items).
template <int NR>
__global__ __launch_bounds__(trsv::kThreads, 1) void dbslmm_trsv_cheb(trsv::Args a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Ring* rg = reinterpret_cast<Ring*>(lds + kNS * kT * NR + 2 * kT * NR + kSW * 8 * NR * (kT + 1));
    const int tid = threadIdx.x;
    for (;;) {
        const int it = take_ticket(a, rg, tid);
        if (it >= a.n_items) break;
        const int32_t w = __builtin_amdgcn_readfirstlane(a.items[2 * it]);
        const int32_t I = __builtin_amdgcn_readfirstlane(a.items[2 * it + 1]);
        const int b = w & 0xFFFF, p = w >> 16, k = p >> 1;
        const bool bwd = p & 1;
        // backward: y_I of this iteration's forward pass; forward k > 0: the previous backward
        // pass's update of r_I
        const Pass ps{a.epoch + p, bwd ? a.Y : a.R, bwd ? a.Z : a.Y,
                      a.coef + static_cast<int64_t>(k) * NR * 3, bwd && k == a.iters - 1};
        const int32_t* wf = (bwd ? a.flags : a.epi) + a.foff[b] + I;
        tile_item<NR>(a, ps, rg, lds, b, I, bwd, wf, (bwd || k > 0) ? a.epoch + p - 1 : 0, tid);
    }
}

// Chebyshev start for a copy group (coef0 = its iteration-0 {alpha, beta, delta}): x = x_b (the
// base copy's solution), r = z - M_c x_b = -delta P_s x_b, d = s = 0; the copies' block status =
// the base's.  One workgroup per tiled block.
extern "C" __global__ __launch_bounds__(256) void dbslmm_cheb_init(
    const int32_t* __restrict__ tb, const int32_t* __restrict__ row0, const int32_t* __restrict__ mv,
    const int32_t* __restrict__ msv, const int32_t* __restrict__ blk_id, const double* __restrict__ xbase,
    const double* __restrict__ coef0, int nr, int64_t vs, double* X, double* R, double* D, double* S,
    const int32_t* __restrict__ st_base, int32_t* st, int64_t st_stride, int c0, int c1, int32_t* conv, int32_t* iters) {
    const int b = tb[blockIdx.x];
    const int g0 = row0[b], m = mv[b], ms = msv[b];
    if (conv && threadIdx.x == 0) conv[b] = 0;   // CG (dbslmm_cg_update): the block iterates
    if (iters && threadIdx.x == 0) iters[b] = 0;  // CG: the run's first copy group
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

// ---------------------------------------------------------------- h2f by conjugate gradients
// The copies' iteration as preconditioned CG (dbslmm_options.h2f_iter = 2, the default) instead of Chebyshev:
// same operator M_c = M_b + delta P_s, same preconditioner (the base factor: one forward and one
// backward pass per iteration), same state vectors (D = p, S = q = M_c p), and no product with
// M_b either -- the Chronopoulos-Gear form takes both inner products from r and z = M_b^{-1} r:
//     gamma = r.z,  eta = z.M_c z = gamma + delta |P_s z|^2   (M_b z = r)
//     beta = gamma / gamma_prev,  alpha = gamma / (eta - beta gamma / alpha_prev)
//     p = z + beta p,  q = r + delta P_s z + beta q,  x += alpha p,  r -= alpha q.
// CG adapts to the block's actual spectrum (M_b^{-1} M_c within [1 + delta / lambda_max(M_b),
// 1 + delta / (d_b + 1 - tau)], not the a priori [1, ...] the Chebyshev coefficients must cover),
// so it stops early: after each update a copy has converged when |r| <= cheb_tol lambda_min(M_c)
// |x| (a bound on the relative error, lambda_min(M_c) >= d_c + 1 - tau, or 1 - tau for a block
// with large SNPs).  A block whose copies have all converged writes its betas and sets conv[b]:
// the later passes skip its items (tools/cheb_vs_cg.py: 5 iterations on config 4's blocks of
// 544 - 9667 SNPs where Chebyshev needs 7; the a priori Chebyshev count stays the cap).
// One workgroup per tiled block of the group, after each backward pass; reductions in a fixed
// order (deterministic).
namespace trsv {
constexpr int kCGThreads = 512;
struct CGArgs {
    const int32_t* tb;           // the group's tiled blocks (plan block ids)
    const int32_t* row0;
    const int32_t* m;
    const int32_t* ms;
    const int32_t* blk_id;
    const int32_t* slot_out;
    const int32_t* st_base;      // the base copy's block status
    int32_t nr, k, last;
    int64_t vs;
    const double* Z;             // z = M_b^{-1} r (the backward pass's result)
    double* X;
    double* R;
    double* D;                   // p
    double* S;                   // q = M_c p
    double delta[kMaxR];
    double floor_s[kMaxR];       // lambda_min(M_c) bound of a block without large SNPs: d_c + 1 - tau
    double floor_l;              // ... with large SNPs: 1 - tau
    double tol;
    double* rec;                 // per plan block and copy: {gamma, alpha} of the previous iteration
    int32_t* conv;
    int32_t* iters;              // per plan block: iterations run, summed over the copy groups
    double inv_sqrt_n;
    double* beta_s;
    double* beta_l;
    int64_t ns_stride, nl_stride;
    int32_t cix[kMaxR];
    int32_t* status;             // per copy (cix) and original block: NOT_CONVERGED at the cap
    int64_t st_stride;
};
// sums of v[0..4) over the workgroup, in a fixed order; every thread gets the totals
__device__ __forceinline__ void cg_sum4(double (&v)[4], double (*red)[4], int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int sft = 32; sft >= 1; sft >>= 1) v[j] += __shfl_xor(v[j], sft);
    if ((tid & 63) == 0)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[tid >> 6][j] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double t = 0.0;
        for (int w = 0; w < kCGThreads / 64; ++w) t += red[w][j];
        v[j] = t;
    }
    __syncthreads();
}
}  // namespace trsv

extern "C" __global__ __launch_bounds__(trsv::kCGThreads) void dbslmm_cg_update(trsv::CGArgs a) {
    using namespace trsv;
    __shared__ double red[kCGThreads / 64][4];
    __shared__ double sc[2 * kMaxR];
    const int b = a.tb[blockIdx.x];
    if (a.conv[b]) return;
    const int tid = threadIdx.x;
    const int g0 = a.row0[b], m = a.m[b], ms = a.ms[b];
    const bool fail = a.st_base[a.blk_id[b]] >= DBSLMM_BLOCK_NOT_PD;
    // gamma_c = r.z, zeta_c = |P_s z|^2
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = tid; i < m; i += kCGThreads)
#pragma unroll
        for (int c = 0; c < kMaxR; ++c) if (c < a.nr) {
            const int64_t o = c * a.vs + g0 + i;
            const double z = a.Z[o];
            v[2 * c] += a.R[o] * z;
            if (i < ms) v[2 * c + 1] += z * z;
        }
    cg_sum4(v, red, tid);
    if (tid == 0)
#pragma unroll
        for (int c = 0; c < kMaxR; ++c) if (c < a.nr) {
            double* rc = a.rec + (static_cast<int64_t>(b) * kMaxR + c) * 2;
            const double gam = v[2 * c], eta = gam + a.delta[c] * v[2 * c + 1];
            double be = 0.0, den = eta;
            if (a.k > 0) {
                be = rc[0] > 0.0 ? gam / rc[0] : 0.0;
                den = eta - (rc[1] != 0.0 ? be * gam / rc[1] : 0.0);
            }
            const double al = den > 0.0 && gam > 0.0 ? gam / den : 0.0;
            sc[2 * c] = al;
            sc[2 * c + 1] = be;
            rc[0] = gam;
            rc[1] = al;
        }
    __syncthreads();
    // the update; |r|^2 and |x|^2 of the new iterate
    double w[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = tid; i < m; i += kCGThreads)
#pragma unroll
        for (int c = 0; c < kMaxR; ++c) if (c < a.nr) {
            const int64_t o = c * a.vs + g0 + i;
            const double al = sc[2 * c], be = sc[2 * c + 1];
            const double z = a.Z[o], r = a.R[o];
            const double p = z + be * a.D[o];
            const double q = r + (i < ms ? a.delta[c] * z : 0.0) + be * a.S[o];
            const double x = a.X[o] + al * p;
            const double rn = r - al * q;
            a.D[o] = p;
            a.S[o] = q;
            a.X[o] = x;
            a.R[o] = rn;
            w[2 * c] += rn * rn;
            w[2 * c + 1] += x * x;
        }
    cg_sum4(w, red, tid);
    bool conv = true;
#pragma unroll
    for (int c = 0; c < kMaxR; ++c) if (c < a.nr) {
        const double t = a.tol * (ms == m ? a.floor_s[c] : a.floor_l);
        const bool cc = w[2 * c] <= t * t * w[2 * c + 1];   // NaN: not converged
        conv = conv && cc;
        // the cap (the Chebyshev count) reached without the bound: the copy keeps this iterate and
        // reports it (the cap was silent); a failed base factor keeps its own status
        if (a.last && !cc && !fail && tid == 0 && a.status)
            a.status[a.cix[c] * a.st_stride + a.blk_id[b]] = DBSLMM_BLOCK_NOT_CONVERGED;
    }
    const bool done = a.last || fail || conv;
    if (!done) return;
    for (int i = tid; i < m; i += kCGThreads) {   // this thread's own x entries
        const int so = a.slot_out[g0 + i];
#pragma unroll
        for (int c = 0; c < kMaxR; ++c) if (c < a.nr) {
            const double x = a.X[c * a.vs + g0 + i];
            const double bv = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
            if (so >= 0) a.beta_s[a.cix[c] * a.ns_stride + so] = bv;
            else a.beta_l[a.cix[c] * a.nl_stride - 1 - so] = bv;
        }
    }
    if (tid == 0) {
        a.conv[b] = 1;
        a.iters[b] += a.k + 1;
    }
}

// ---------------------------------------------------------------- whole-block Chebyshev passes
// The rest group's tiled blocks (m < the lead threshold, at most ~40 tiles of 64) iterate with one
// workgroup per block and every pass of the Chebyshev group in ONE launch: no ticket, flag or
// hand-off per 64-row tile -- the tile item's fixed cost (ticket, drain, flag, poll, about as long
// as streaming a small block's tile row) is what held those blocks' per-pass launches to ~14 GB/s
// per CU.  The block's substitutions stream its factor row by row (the layout of trsv.hip's tile
// items: 8 waves x 8 rows of a 64-row tile, lane = column) as one flat sequence of (row tile,
// column tile) pairs with kPF pairs in flight per wave across row-tile boundaries; a row tile ends
// with a butterfly reduction of the 8 x NR lane partial sums (no LDS transpose), the diagonal
// inverse block product and a workgroup barrier.  The vectors: the work vector v in LDS, the
// Chebyshev state x / r / d / s in the group's slot vectors (as dbslmm_cheb_init / the tile items'
// epilogue, same recurrence and coefficients).
namespace trsv {
constexpr int kBThreads = kSW * 64;          // 8 streaming waves, no control wave
constexpr int kBPF = 4;                      // column tiles in flight per wave

// sum of a[0 .. NV) over the wave's 64 lanes; lane l ends with value l >> (6 - log2 NV)
// (fixed order: deterministic)
template <int NV>
__device__ __forceinline__ double wave_sums(double (&a)[NV], int lane) {
    constexpr int kSteps = NV == 16 ? 4 : NV == 8 ? 3 : NV == 4 ? 2 : 1;
#pragma unroll
    for (int st = 0; st < kSteps; ++st) {
        const int h = NV >> (st + 1), bit = 5 - st;
        const bool hi = (lane >> bit) & 1;
#pragma unroll
        for (int j = 0; j < h; ++j) {
            const double send = hi ? a[j] : a[j + h];
            const double keep = hi ? a[j + h] : a[j];
            a[j] = keep + __shfl_xor(send, 1 << bit);
        }
    }
    double s = a[0];
#pragma unroll
    for (int bit = 5 - kSteps; bit >= 0; --bit) s += __shfl_xor(s, 1 << bit);
    return s;
}

// one substitution pass of a block (forward L y = v or backward L^T z = v, in place on v).  Row
// tiles in substitution order; row tile I streams its column tiles (forward J = 0 .. I-1, backward
// J = T-1 .. I+1) kBPF in flight per wave, and issues the next row tile's first kBPF column tiles
// before its own reduction, so the stream does not restart at the row-tile boundary.
template <int NR, bool BWD>
__device__ __forceinline__ void block_pass(const double* __restrict__ A, int ld, int m, int T, double* v, int vld,
                                           double* ws, int tid) {
    const int wave = tid >> 6, lane = tid & 63, row = tid >> 3, part = tid & 7;
    constexpr int NV = 8 * NR;
    const double* Lw = A + static_cast<int64_t>(8 * wave) * ld + lane;
    auto cnt_of = [&](int I) { return BWD ? T - 1 - I : I; };
    auto col_of = [&](int I, int t) { return BWD ? T - 1 - t : t; };
    double lr[kBPF][8];
    auto issue = [&](int u, int I, int t) {
        const int cj = kT * col_of(I, t);
        const double* p = Lw + static_cast<int64_t>(kT * I) * ld + cj;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double x = p[static_cast<int64_t>(k) * ld];
            lr[u][k] = cj + lane < m ? x : 0.0;   // past m: bordered row / padding
        }
    };
    double acc[NV];
    double xd[8];
    const int I0 = BWD ? T - 1 : 0, dI = BWD ? -1 : 1;
#pragma unroll
    for (int u = 0; u < kBPF; ++u)
        if (u < cnt_of(I0)) issue(u, I0, u);
    for (int I = I0; BWD ? I >= 0 : I < T; I += dI) {
        const int r0 = kT * I, jmax = min(kT, m - r0), cnt = cnt_of(I);
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // this row tile's diagonal inverse block (used at its end)
            const int q = 8 * part + k;
            const int64_t o = BWD ? static_cast<int64_t>(r0 + row) * ld + r0 + q
                                  : static_cast<int64_t>(r0 + q) * ld + r0 + row;
            const double x = A[o];
            xd[k] = (BWD ? (q >= row && q < jmax) : (q <= row && row < jmax)) ? x : 0.0;
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) acc[q] = 0.0;
        for (int t0 = 0; t0 < cnt; t0 += kBPF) {
#pragma unroll
            for (int u = 0; u < kBPF; ++u) {
                const int t = t0 + u;
                if (t < cnt) {
                    const double* vv = v + kT * col_of(I, t) + lane;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
#pragma unroll
                        for (int c = 0; c < NR; ++c) acc[k * NR + c] += lr[u][k] * vv[c * vld];
                    if (t + kBPF < cnt) issue(u, I, t + kBPF);
                }
            }
        }
        const int In = I + dI;
        if (BWD ? In >= 0 : In < T) {
            const int cn = cnt_of(In);
#pragma unroll
            for (int u = 0; u < kBPF; ++u)
                if (u < cn) issue(u, In, u);
        }
        // w = v_I - sum_J L_IJ v_J (lanes: butterfly sums), then v_I = X_I w / X_I^T w
        const double s = wave_sums<NV>(acc, lane);
        constexpr int kSh = NV == 16 ? 2 : NV == 8 ? 3 : 4;
        if ((lane & ((1 << kSh) - 1)) == 0) {
            const int vi = lane >> kSh, k = vi / NR, c = vi - k * NR, r = 8 * wave + k;
            ws[r * NR + c] = r < jmax ? v[c * vld + r0 + r] - s : 0.0;
        }
        __syncthreads();
        double y[NR];
#pragma unroll
        for (int c = 0; c < NR; ++c) y[c] = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
            for (int c = 0; c < NR; ++c) y[c] += xd[k] * ws[(8 * part + k) * NR + c];
#pragma unroll
        for (int c = 0; c < NR; ++c) y[c] = red8(y[c]);
        if (part == 0 && row < jmax)
#pragma unroll
            for (int c = 0; c < NR; ++c) v[c * vld + r0 + row] = y[c];
        __syncthreads();
    }
}
}  // namespace trsv

// All K iterations of a Chebyshev copy group for the listed tiled blocks, one workgroup per block
// (blocks[g], largest first).  x_base: the base copy's solution (slot vectors); X / R / D / S: the
// group's state vectors (stride vs per copy); coef [K][NR][3]; betas of copies cix[c]; status of
// the copies = the base's.
struct TChebArgs {
    const double* M;
    const int64_t* matoff;
    const int32_t* ld;
    const int32_t* m;
    const int32_t* ms;
    const int32_t* row0;
    const int32_t* blk_id;
    const int32_t* slot_out;
    const int32_t* blocks;
    int32_t n_blocks;
    int32_t iters;
    int32_t vld;                 // LDS stride of the work vector (>= 64 T of every listed block)
    int64_t vs;
    const double* x_base;
    double* X;
    double* R;
    double* D;
    double* S;
    const double* coef;
    double inv_sqrt_n;
    double* beta_s;
    double* beta_l;
    int64_t ns_stride, nl_stride;
    int32_t cix[trsv::kMaxR];
    const int32_t* st_base;
    int32_t* status;
    int64_t st_stride;
};

template <int NR>
__global__ __launch_bounds__(trsv::kBThreads, 2) void dbslmm_tcheb(TChebArgs a) {
    using namespace trsv;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    if (static_cast<int>(blockIdx.x) >= a.n_blocks) return;
    const int b = a.blocks[blockIdx.x];
    const int tid = threadIdx.x;
    const int m = a.m[b], ms = a.ms[b], ld = a.ld[b], g0 = a.row0[b];
    const int T = (m + kT - 1) / kT;
    const double* A = a.M + a.matoff[b];
    double* v = lds;                            // [NR][vld]
    double* ws = v + NR * a.vld;                // [64][NR]
    const int32_t st = a.st_base[a.blk_id[b]];
    const bool fail = st >= DBSLMM_BLOCK_NOT_PD;
    if (tid < NR) a.status[a.cix[tid] * a.st_stride + a.blk_id[b]] = st;
    // start: x = x_b, r = -delta P_s x_b, d = s = 0 (dbslmm_cheb_init)
    for (int e = tid; e < NR * m; e += kBThreads) {
        const int c = e / m, i = e - c * m;
        const int64_t o = c * a.vs + g0 + i;
        const double xb = a.x_base[g0 + i];
        a.X[o] = xb;
        a.R[o] = i < ms ? -a.coef[3 * c + 2] * xb : 0.0;
        a.D[o] = 0.0;
        a.S[o] = 0.0;
    }
    for (int k = 0; k < a.iters && !fail; ++k) {
        for (int e = tid; e < NR * a.vld; e += kBThreads) {
            const int c = e / a.vld, i = e - c * a.vld;
            v[e] = i < m ? a.R[c * a.vs + g0 + i] : 0.0;
        }
        __syncthreads();
        block_pass<NR, false>(A, ld, m, T, v, a.vld, ws, tid);
        block_pass<NR, true>(A, ld, m, T, v, a.vld, ws, tid);
        // d = alpha d + beta z; s = alpha s + beta r; x += d; r -= s + delta P_s d
        const double* cf = a.coef + static_cast<int64_t>(k) * NR * 3;
        const bool last = k == a.iters - 1;
        for (int e = tid; e < NR * m; e += kBThreads) {
            const int c = e / m, i = e - c * m;
            const int64_t o = c * a.vs + g0 + i;
            const double al = cf[3 * c], be = cf[3 * c + 1], de = cf[3 * c + 2];
            const double d = al * a.D[o] + be * v[c * a.vld + i];
            const double x = a.X[o] + d;
            a.X[o] = x;
            if (!last) {
                const double r = a.R[o];
                const double s2 = al * a.S[o] + be * r;
                a.D[o] = d;
                a.S[o] = s2;
                a.R[o] = r - s2 - (i < ms ? de * d : 0.0);
            }
        }
        __syncthreads();
    }
    for (int e = tid; e < NR * m; e += kBThreads) {
        const int c = e / m, i = e - c * m;
        const double x = a.X[c * a.vs + g0 + i];
        const double bv = fail ? __builtin_nan("") : x * a.inv_sqrt_n;
        const int so = a.slot_out[g0 + i];
        if (so >= 0) a.beta_s[a.cix[c] * a.ns_stride + so] = bv;
        else a.beta_l[a.cix[c] * a.nl_stride - 1 - so] = bv;
    }
}
