// pcg.hip -- the iterative route of the per-block solve (round 6): DBSLMMFIT's own algorithm,
// Jacobi-preconditioned CG (PCGv / PCGm, reference scr/dbslmmfit.cpp:629-678), run on the LD
// matrix the FP4 Gram kernels (kernels.hip) build, for every block of a plan and every h2f copy at
// once.
//
// What it solves.  estBlock (scr/dbslmmfit.cpp:680-770) is one solve of the joint matrix
//     M_c = [[Sigma_ss + d_c I, Sigma_sl], [Sigma_ls, Sigma_ll]],   d_c = 1 / (sigma_c n)
// with beta = M_c^{-1} [z_s; z_l] / sqrt(n) (the reference's PCGm /
// Schur-complement steps are block elimination of exactly this system; LMM-only is m_l = 0).  The
// reference iterates on A = Sigma_ss + d I with Jacobi-PCG; here one Jacobi-PCG runs on the whole
// joint M_c (diagonal c0 + d_c on small SNPs, c0 on large ones, c0 = tau (n_ref - 1) / n_ref +
// 1 - tau for every standardised column), which needs no Schur step and no per-large-SNP
// right-hand side: the few large SNPs are a handful of outlying eigenvalues of the scaled matrix
// (tools/cg_gate.py: 13 -> 17 iterations from 0 to 10 large SNPs in a block at config 4).
//
// Why it is cheap.  Sigma_ss >= (1 - tau) I, so lambda_min(M_c) >= 1 - tau, and >= d_c + 1 - tau
// for a block without large SNPs; at the BASELINE configs d_c = nsnp / (h n) = 10 .. 25 and
// lambda_max(tau X^T X / n_ref) ~ 10, so kappa ~ 1.4 - 2 and PCG reaches a relative error of 1e-12
// in ~13 - 19 iterations (tools/cg_gate.py) -- where the factorisation costs m^3 / 3 flops on a
// dependency chain of m columns.  Stopping rule per block and copy: |r| <= tol lambda |x| with
// lambda the bound above, a bound on the relative 2-norm error of x that holds for any data; a
// copy that reaches the iteration cap without it reports DBSLMM_BLOCK_NOT_CONVERGED (the
// reference prints "Matrix is Singular!" at maxiter and returns the iterate, :664-666).
//
// The operator.  The Gram kernels store, for blocks without missing calls and n_ref <= 16383, the
// INTEGER Gram G_ij = sum_k g_ik g_jk of the dosages as uint16 (lower triangle, the block's ld x ld
// row-major layout: a quarter of the bytes of the fp64 Sigma), and the product is formed around it:
//     Sigma u = tau / n_ref * rsd o (G (rsd o u) - S (S . (rsd o u)) / n_ref) + (1 - tau) u
// (S = per-SNP dosage sums, rsd = 1/sd with the N-1 divisor: the Gram epilogue's centring and
// standardisation, scr/dtpr.cpp:375-380).  Blocks with missing calls (mean imputation) or larger
// panels read the fp64 Sigma the Gram wrote instead.  Each iteration streams the lower triangle
// ONCE: a 128 x 128 tile (I, J) adds G_IJ v_J to rows I and G_IJ^T v_I to rows J.
//
// Kernels (one launch each per iteration, every block of the plan in each):
//   dbslmm_pcg_symv    one wave per item = a run of up to `run` tiles along a tile row; per lane an
//                      8 x 8 sub-block of each 64 x 64 quadrant, row and column sums reduce-
//                      scattered over the lanes (fixed order); writes the row partial of the run
//                      and each tile's column partial into per-block slots (no atomics: the sums
//                      are deterministic, run to run and device to device).
//   dbslmm_pcg_rows    per 128-row tile row: w = M_c u from the partial slots (fixed order),
//                      partial dots r.u, w.u, r.r, x.x.
//   dbslmm_pcg_update  per tile row: block sums of the dots (fixed order, the same in every
//                      workgroup of the block), the stopping test, alpha / beta (Chronopoulos-Gear
//                      form: one reduction phase per iteration), p, s, x, r.
//   dbslmm_pcg_init / dbslmm_pcg_final   right-hand sides and state; beta = x / sqrt(n) in the
//                      caller's order, status per copy.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pcg {
constexpr int kT = 128;           // tile edge of the operator's lower triangle (slots of a block)
constexpr int kRunMax = 8;        // tiles per symv item (along a tile row): 8, or fewer when the
                                  // plan has too few items to fill the chip (PcgArgs::run)
constexpr int kMaxNC = 4;         // h2f copies per run (right-hand sides) on this route
constexpr int kWaves = 4;         // symv items per 256-thread workgroup
constexpr int kVS = kT + 8;       // LDS stride of a staged vector column (doubles)
constexpr int kNDot = 5;          // per tile row and copy: r.u, w.u, r.r, x.x, S.(rsd o u)
constexpr int kQS = 8;            // recurrence state doubles per block and copy
constexpr int kThreads = 256;
constexpr int kFTb = 8;           // dbslmm_pcg_block: blocks of at most kFTb tile rows (1024 slots)
constexpr int kFRows = kFTb * kT;
constexpr int kFPer = kFRows / kThreads;   // rows per thread
// symv LDS per wave: the staged rsd o u of the item's tile row and of two tile columns, and the
// reduce-scattered row / column sums ([2][copy][64] each)
constexpr int wave_lds_doubles(int nc) { return 3 * nc * kVS + 4 * nc * 64; }
constexpr size_t lds_bytes(int nc) { return sizeof(double) * kWaves * wave_lds_doubles(nc); }
}  // namespace pcg

// One block of the route (plan block `blk`).  Slots row0 .. row0 + m: [small | large]; the block's
// matrix at element matoff, row stride ld (as the factor route lays it out).
struct PcgBlk {
    int32_t blk, row0, m, ms;
    int32_t ld, Tb, Ns, sco;        // Tb = ceil(m / kT) tile rows, Ns partial slots per tile row
    int64_t matoff, vo, po, dof;    // vectors (per copy Tb * kT), partials, dots
    int64_t off16;                  // the integer Gram: Tb kT x Tb kT uint16 at off16 (rows and
                                    // columns past m stay zero: no masks in the product)
    int32_t nc;                     // product columns: 1 (multi-shift block) or the copies
    int32_t mshift;                 // 1: no large SNP and several copies -> one Krylov sequence
    int32_t fused;                  // 1: <= kFTb tile rows -- on the uint16 Gram the whole solve
                                    // runs in dbslmm_pcg_block (done = 3), one entry per sequence
    int32_t pad_;
};

struct PcgArgs {
    const PcgBlk* blk;
    const uint16_t* G16;            // integer Gram (u16), or null (every block on the fp64 Sigma)
    const double* M;                // fp64 Sigma (copy 0): blocks with missing calls
    const int32_t* flags;           // per plan block, bit 0: missing calls
    const double* S;                // per slot: dosage sum
    const double* rsd;              // per slot: 1 / sd (N-1)
    const double* z;                // per slot: z-score
    const int32_t* slot_out;        // per slot: >= 0 small beta index, -1-l large
    const int32_t* blk_id;          // plan block -> original block id
    const double* dshift;           // per copy: 1 / (sigma_c n)
    double *X, *R, *P, *Sv, *W;     // state vectors, [copy][Tb * kT] per block
    double* U;                      // the product's input per product column: (rsd on the uint16
                                    // path) o r / diag, zero past m -- written with r
    double* part;                   // symv partial slots
    double* dot;                    // per tile row [kNDot][copy]
    double* qs;                     // per block copy: {gamma, alpha} x 2 parities, then the
                                    // multi-shift {zeta_k, zeta_k-1} x 2 parities (kQS doubles)
    int32_t* cnv;                   // per block copy: iteration + 1 at convergence (0: running)
    int32_t* itb;                   // per block: rows launches since init
    int32_t* done;                  // per block: 0 iterating, 1 converged, 2 monomorphic
    int32_t* active;                // blocks still iterating
    double* beta_s;
    double* beta_l;
    int32_t* status;
    int64_t vstride;                // elements per copy-major vector array
    int64_t ns, nl, nbk;            // beta / status strides per copy
    double tau, rn, c0, tol, inv_sqrt_n;
    int32_t ncopy;
    int32_t run;                    // tiles per symv item (1, 2, 4 or 8)
    int32_t seed;                   // multi-shift seed: the copy with the smallest shift
};

namespace pcg {

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v from lane ^ X.  X = 1, 2, 4, 8 stay inside a 16-lane row and move through DPP (VALU, no LDS
// round trip): xor 1 / 2 as quad permutations, xor 4 as the half-row mirror (lane i <- 7 - i of
// its eight) then the quad reversal, xor 8 as the row rotation by 8; wider ones go through
// ds_bpermute (__shfl_xor).
template <int Ctrl>
__device__ __forceinline__ double dpp_mov(double v) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const int lo = __builtin_amdgcn_mov_dpp(static_cast<int>(b & 0xffffffffu), Ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp(static_cast<int>(b >> 32), Ctrl, 0xf, 0xf, false);
    return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}
// xor 16 / 32 through gfx950's row swaps: v_permlane16_swap / v_permlane32_swap of a value with
// itself leave, in a lane of an odd 16-lane row (upper 32-lane half), its partner's value in the
// first result and in an even row (lower half) in the second (tools/micro/probe_permlane.hip)
template <int X>
__device__ __forceinline__ uint32_t swap_xor(uint32_t x, bool up) {
    if constexpr (X == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return up ? r[0] : r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return up ? r[0] : r[1];
    }
}
template <int X>
__device__ __forceinline__ double lane_xor(double v) {
#ifndef PCG_NO_DPP
    if constexpr (X == 1) return dpp_mov<0xB1>(v);                   // quad_perm [1, 0, 3, 2]
    else if constexpr (X == 2) return dpp_mov<0x4E>(v);              // quad_perm [2, 3, 0, 1]
    else if constexpr (X == 4) return dpp_mov<0x1B>(dpp_mov<0x141>(v));   // row_half_mirror, quad_perm [3, 2, 1, 0]
    else if constexpr (X == 8) return dpp_mov<0x128>(v);             // row_ror:8
#ifndef PCG_NO_PERMLANE
    else if constexpr (X == 16 || X == 32) {
        const uint64_t b = __builtin_bit_cast(uint64_t, v);
        const bool up = (__lane_id() & X) != 0;
        const uint32_t lo = swap_xor<X>(static_cast<uint32_t>(b & 0xffffffffu), up);
        const uint32_t hi = swap_xor<X>(static_cast<uint32_t>(b >> 32), up);
        return __builtin_bit_cast(double, (static_cast<uint64_t>(hi) << 32) | lo);
    }
#endif
    else
#endif
        return __shfl_xor(v, X);
}

// Reduce-scatter of v[0..8) over the 8 lanes that differ in lane bits (X2, X1, X0): the lane
// whose bits read s = 4 b2 + 2 b1 + b0 returns the sum of v[s] over those lanes (fixed order).
template <int X2, int X1, int X0>
__device__ __forceinline__ double rscatter8(const double (&v)[8], int lane) {
    const bool h2 = (lane & X2) != 0, h1 = (lane & X1) != 0, h0 = (lane & X0) != 0;
    double u[4], w[2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const double send = h2 ? v[q] : v[q + 4], keep = h2 ? v[q + 4] : v[q];
        u[q] = keep + lane_xor<X2>(send);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const double send = h1 ? u[q] : u[q + 2], keep = h1 ? u[q + 2] : u[q];
        w[q] = keep + lane_xor<X1>(send);
    }
    const double send = h0 ? w[0] : w[1], keep = h0 ? w[1] : w[0];
    return keep + lane_xor<X0>(send);
}

__device__ __forceinline__ double wave_sum(double v) {   // (fixed order: xor 32, 16, .., 1)
    v += lane_xor<32>(v);
    v += lane_xor<16>(v);
    v += lane_xor<8>(v);
    v += lane_xor<4>(v);
    v += lane_xor<2>(v);
    v += lane_xor<1>(v);
    return v;
}



// sum of p[s * st] over s in [s0, s1) in order, eight loads in flight (a serial chain of dependent
// loads over a 76-slot tile row cost ~100 us per launch)
__device__ __forceinline__ double ordered_sum(const double* __restrict__ p, int64_t st, int s0, int s1, double acc) {
    for (int s = s0; s < s1; s += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = s + u < s1 ? p[static_cast<int64_t>(s + u) * st] : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
    }
    return acc;
}

__device__ __forceinline__ bool on_u16(const PcgArgs& a, const PcgBlk& B) {
    return a.G16 != nullptr && (a.flags[B.blk] & 1) == 0;
}

// Jacobi diagonal of M_c at block slot i (c0 + d_c on small SNPs); 1 on a multi-shift block
// (no large SNP: the diagonal is the constant c0 + d_c, and the shifted systems share one Krylov
// space only without a preconditioner)
__device__ __forceinline__ double jdiag(const PcgArgs& a, const PcgBlk& B, int i, double dc) {
    return B.mshift ? 1.0 : i < B.ms ? a.c0 + dc : a.c0;
}
// the shift of product column k (the seed's on a multi-shift block)
__device__ __forceinline__ double col_shift(const PcgArgs& a, const PcgBlk& B, int k) {
    return a.dshift[B.mshift ? a.seed : k];
}

// uint16 -> fp64 of the low / high half of a dword.  Volatile asm: the conversions stay inside the
// copy loop (hoisted out of it, the 64 values of a quadrant would take 128 registers and half the
// occupancy the loads need; tools: 234 -> 119 VGPRs).
__device__ __forceinline__ double cvt_lo(uint32_t w) {
    double g;
    uint32_t t;
    asm volatile("v_and_b32 %1, 0xffff, %2\n\tv_cvt_f64_u32 %0, %1" : "=v"(g), "=&v"(t) : "v"(w));
    return g;
}
__device__ __forceinline__ double cvt_hi(uint32_t w) {
    double g;
    uint32_t t;
    asm volatile("v_lshrrev_b32 %1, 16, %2\n\tv_cvt_f64_u32 %0, %1" : "=v"(g), "=&v"(t) : "v"(w));
    return g;
}

typedef uint32_t pcg_u4 __attribute__((ext_vector_type(4)));

// A range-checked buffer descriptor over `bytes` of the integer Gram from `base` (wave-uniform: its
// inputs go through readfirstlane, as 32-bit unsigned halves -- readfirstlane returns int, and a
// low half >= 2^31 widened as int would set the high word).  A load at an offset >= bytes returns
// zeros and touches no memory.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t g16_rsrc(const uint16_t* base, uint32_t bytes) {
    const uint64_t gb = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(gb & 0xffffffffu)));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(gb >> 32)));
    const int nb = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo),
                                             static_cast<short>(0), nb, 0x00020000);
}
constexpr uint32_t kG16Oob = 0x80000000u;   // (an offset beyond any descriptor's range)

// One 64 x 64 quadrant of a tile: lane (rg = lane >> 3, cg = lane & 7) holds rows 8 rg .. + 7,
// columns 8 cg .. + 7 as 8 x 8 uint16 (raw: four dwords per row; on a diagonal quadrant the row
// sums take j <= i, the column sums j < i).  Per copy k: row sums (G v_J) reduce-scatter over cg
// -> row 8 rg + cg, added to rsum[k * 64 + lane]; column sums (G^T v_I) over rg -> column
// 8 cg + rg, added to csum[k * 64 + lane] (wave-private LDS: the copy loop stays a loop).
__device__ __forceinline__ void quad_mul16(const pcg_u4 (&raw)[8], bool diagq, int lane, int nc,
                                           const double* vI, const double* vJ, double* rsum, double* csum) {
    const int rg = lane >> 3, cg = lane & 7;
#pragma unroll 1
    for (int k = 0; k < nc; ++k) {
        double vi[8], vj[8], racc[8], cacc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            vi[q] = vI[k * kVS + 8 * rg + q];
            vj[q] = vJ[k * kVS + 8 * cg + q];
            racc[q] = cacc[q] = 0.0;
        }
        if (!diagq) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t w = raw[r][c >> 1];
                    const double g = (c & 1) ? cvt_hi(w) : cvt_lo(w);
                    racc[r] = __builtin_fma(g, vj[c], racc[r]);
                    cacc[c] = __builtin_fma(g, vi[r], cacc[c]);
                }
        } else {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t w = raw[r][c >> 1];
                    const double g = (c & 1) ? cvt_hi(w) : cvt_lo(w);
                    const int dd = 8 * (cg - rg) + c - r;   // j - i
                    racc[r] = __builtin_fma(dd <= 0 ? g : 0.0, vj[c], racc[r]);
                    cacc[c] = __builtin_fma(dd < 0 ? g : 0.0, vi[r], cacc[c]);
                }
        }
        rsum[k * 64 + lane] += rscatter8<4, 2, 1>(racc, lane);
        csum[k * 64 + lane] += rscatter8<32, 16, 8>(cacc, lane);
    }
}

// the same on the fp64 Sigma (blocks with missing calls, panels beyond uint16): elements read per
// copy from global (cache hits after the first copy)
__device__ __forceinline__ void quad_mul64(const double* __restrict__ base, int64_t ld, int rows_ok, int cols_ok,
                                           bool diagq, int lane, int nc, const double* vI, const double* vJ,
                                           double* rsum, double* csum) {
    const int rg = lane >> 3, cg = lane & 7;
#pragma unroll 1
    for (int k = 0; k < nc; ++k) {
        double vi[8], vj[8], racc[8], cacc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            vi[q] = vI[k * kVS + 8 * rg + q];
            vj[q] = vJ[k * kVS + 8 * cg + q];
            racc[q] = cacc[q] = 0.0;
        }
#pragma unroll 1
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const double g = (r < rows_ok && c < cols_ok) ? base[r * ld + c] : 0.0;
                const int dd = 8 * (cg - rg) + c - r;
                // (racc / cacc indexed by r at run time: the row loop is not unrolled here)
                const double gr = !diagq || dd <= 0 ? g : 0.0, gc = !diagq || dd < 0 ? g : 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (q == r) racc[q] = __builtin_fma(gr, vj[c], racc[q]);
                cacc[c] = __builtin_fma(gc, vi[r], cacc[c]);
            }
        rsum[k * 64 + lane] += rscatter8<4, 2, 1>(racc, lane);
        csum[k * 64 + lane] += rscatter8<32, 16, 8>(cacc, lane);
    }
}

// the product's input of tile row T (every product column) into LDS: U = (rsd o) r / diag, as
// the last update (or init) wrote it -- zero past m
__device__ __forceinline__ void stage_v(const PcgArgs& a, const PcgBlk& B, int T, int nc, int lane, double* v) {
    for (int k = 0; k < nc; ++k) {
        const double* src = a.U + k * a.vstride + B.vo + static_cast<int64_t>(T) * kT;
        const double x0 = src[lane], x1 = src[lane + 64];
        v[k * kVS + lane] = x0;
        v[k * kVS + lane + 64] = x1;
    }
}

// One symv item on one wave.  LDS (wave-private): vI = rsd o u of the item's tile row, vJ[2] = the
// same of the current and the next tile column ([copy][kVS] each), rsum / csum = the
// reduce-scattered row results of the run and column results of the current tile
// ([qi or qj][copy][lane]).  The item's active quadrants are visited in order (tiles J0 .. J1,
// quadrants q = 2 qi + qj: a diagonal tile has no upper quadrant, quadrants wholly past m are
// skipped), software-pipelined: the next quadrant's 8 KB of row segments and, at a tile change,
// the next column vector are in flight while the current quadrant is multiplied.
__device__ __forceinline__ bool quad_active(const PcgBlk& B, int I, int J, int q) {
    const int qi = q >> 1, qj = q & 1;
    return !(J == I && qj > qi) && I * kT + 64 * qi < B.m && J * kT + 64 * qj < B.m;
}
// the next active quadrant after (J, q) within tiles .. J1; false at the end
__device__ __forceinline__ bool next_quad(const PcgBlk& B, int I, int J1, int& J, int& q) {
    for (;;) {
        if (++q == 4) {
            q = 0;
            if (++J > J1) return false;
        }
        if (quad_active(B, I, J, q)) return true;
    }
}

template <bool U16>
__device__ void symv_item(const PcgArgs& a, int4 item, int lane, double* vI, double* vJb, double* rsum,
                          double* csum) {
    const PcgBlk B = a.blk[item.x];
    if (a.done[item.x] || on_u16(a, B) != U16) return;
    const int I = item.y, J0 = item.z, J1 = item.w, nc = B.nc;
    const int64_t ld16 = static_cast<int64_t>(B.Tb) * kT;
    const int rg = lane >> 3, cg = lane & 7;
    auto vj_of = [&](int J) -> double* { return J == I ? vI : vJb + ((J - J0) & 1) * nc * kVS; };
    // tile row I of the Gram through a range-checked buffer descriptor (wave-uniform: one item per
    // wave): sub-block rows wholly above the diagonal or past m, and the quadrant after the item's
    // last (none), read beyond the range -- zeros, no memory access -- so every load() issues its 8
    // loads unconditionally and the wait before a quadrant's product counts only its own loads
    const __amdgpu_buffer_rsrc_t g16 =
        g16_rsrc(a.G16 + B.off16 + static_cast<int64_t>(I) * kT * ld16, U16 ? static_cast<uint32_t>(kT * ld16 * 2) : 0u);
    auto load = [&](int J, int q, pcg_u4 (&raw)[8], bool none) {
        if constexpr (U16) {
            const int i0 = 64 * (q >> 1) + 8 * rg, j0 = J * kT + 64 * (q & 1) + 8 * cg;   // (i0 within the tile row)
            const bool skip = none || j0 >= B.m || (J == I && (q == 0 || q == 3) && cg > rg);
            const uint32_t o = static_cast<uint32_t>((static_cast<int64_t>(i0) * ld16 + j0) * 2);
#pragma unroll
            for (int r = 0; r < 8; ++r)
                raw[r] = __builtin_amdgcn_raw_buffer_load_b128(
                    g16, (skip || I * kT + i0 + r >= B.m) ? kG16Oob : o + static_cast<uint32_t>(r * ld16 * 2), 0, 0);
        }
    };
    auto mult = [&](int J, int q, const pcg_u4 (&raw)[8]) {
        const int qi = q >> 1, qj = q & 1;
        const bool dq = J == I && qi == qj;
        const double* vj = vj_of(J);
        double* rs = rsum + qi * nc * 64;
        double* cs = csum + qj * nc * 64;
        if constexpr (U16) {
            quad_mul16(raw, dq, lane, nc, vI + 64 * qi, vj + 64 * qj, rs, cs);
        } else {
            const int ib = I * kT + 64 * qi + 8 * rg, jb = J * kT + 64 * qj + 8 * cg;
            quad_mul64(a.M + B.matoff + static_cast<int64_t>(ib) * B.ld + jb, B.ld, B.m - ib, B.m - jb, dq,
                       lane, nc, vI + 64 * qi, vj + 64 * qj, rs, cs);
        }
    };
    auto flush = [&](int J) {   // column partial of tile (I, J): slot I of tile row J
        double* dst = a.part + B.po + (static_cast<int64_t>(J) * B.Ns + I) * nc * kT;
        for (int qj = 0; qj < 2; ++qj)
            for (int k = 0; k < nc; ++k) {
                dst[k * kT + 64 * qj + 8 * cg + rg] = csum[(qj * nc + k) * 64 + lane];
                csum[(qj * nc + k) * 64 + lane] = 0.0;
            }
    };
    pcg_u4 ra[8], rb[8];
    int J = J0, q = 0;                       // quadrant 0 of a tile of the run is always active
    load(J, q, ra, false);
    stage_v(a, B, I, nc, lane, vI);
    if (J != I) stage_v(a, B, J, nc, lane, vj_of(J));
    for (int t = 0; t < 2 * nc; ++t) rsum[t * 64 + lane] = csum[t * 64 + lane] = 0.0;
    wave_fence();
    // one pipeline step: prefetch the next quadrant into `nxt` (and its column vector at a tile
    // change), multiply the current one from `cur`; false when the item is done.  (Issuing the
    // column vector's loads before the quadrant's was measured slower: 290 vs 257 us at config 4.)
    auto step = [&](pcg_u4 (&cur)[8], pcg_u4 (&nxt)[8]) -> bool {
        int Jn = J, qn = q;
        const bool more = next_quad(B, I, J1, Jn, qn);
        load(more ? Jn : J, more ? qn : q, nxt, !more);        // (issued either way: counted waits)
        if (more && Jn != J && Jn != I) stage_v(a, B, Jn, nc, lane, vj_of(Jn));
        mult(J, q, cur);
        if (!more || Jn != J) flush(J);
        wave_fence();                        // the next column vector is in LDS before its use
        J = Jn;
        q = qn;
        return more;
    };
    while (step(ra, rb) && step(rb, ra)) {
    }
    // row partial of the run: slot Tb + run of tile row I
    double* dst = a.part + B.po + (static_cast<int64_t>(I) * B.Ns + B.Tb + J0 / a.run) * nc * kT;
    for (int qi = 0; qi < 2; ++qi)
        for (int k = 0; k < nc; ++k) dst[k * kT + 64 * qi + 8 * rg + cg] = rsum[(qi * nc + k) * 64 + lane];
}

}  // namespace pcg

// ------------------------------------------------------------------------------------------
// Right-hand sides and state.  One workgroup per (block, 128-row tile row): x = p = s = w = 0,
// r = z (every product column), the partial S.(rsd o u) of the first product.  Tile row 0 also
// resets the block's counters and recurrence state and flags a monomorphic block (a zero-variance
// SNP: the reference's 0/0 column, beta NaN for the whole block, status MONOMORPHIC) as done.
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(pcg::kThreads) void dbslmm_pcg_init(PcgArgs a, const int2* __restrict__ rows) {
    using namespace pcg;
    __shared__ double red[kThreads / 64][kMaxNC];
    __shared__ int mono_s;
    const int2 it = rows[blockIdx.x];
    const int bi = it.x, I = it.y, tid = threadIdx.x;
    const PcgBlk B = a.blk[bi];
    const bool u16 = on_u16(a, B);
    const int n = a.ncopy, nc = B.nc;
    if (I == 0) {
        if (tid == 0) mono_s = 0;
        __syncthreads();
        bool mono = false;
        for (int i = tid; i < B.m; i += kThreads) mono |= !(a.rsd[B.row0 + i] < INFINITY);
        if (mono) atomicOr(&mono_s, 1);
        __syncthreads();
        if (tid < n) {
            a.cnv[B.sco + tid] = 0;
            double* q = a.qs + static_cast<int64_t>(B.sco + tid) * kQS;
            q[4] = q[5] = 1.0;           // zeta_0 = zeta_-1 = 1 (parity 0)
        }
        if (tid == 0) {
            a.itb[bi] = 0;
            const bool fz = B.fused && u16;       // solved whole by dbslmm_pcg_block
            a.done[bi] = mono_s ? 2 : fz ? 3 : 0;
            if (!mono_s && !fz) atomicAdd(a.active, 1);
        }
    }
    // rows 0..127 of the tile row, two halves of the columns
    const int r = tid & (kT - 1), h = tid >> 7, i = I * kT + r;
    const bool in = i < B.m;
    double sv[kMaxNC];
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k) sv[k] = 0.0;
    for (int c = h; c < n; c += 2) {
        const int64_t o = c * a.vstride + B.vo + i;
        const double rhs = in ? a.z[B.row0 + i] : 0.0;
        a.X[o] = 0.0;
        a.P[o] = 0.0;
        if (c < nc) {
            a.Sv[o] = 0.0;
            a.W[o] = 0.0;
            a.R[o] = rhs;
            double uv = 0.0;
            if (in) {
                uv = rhs / jdiag(a, B, i, col_shift(a, B, c));
                if (u16) uv *= a.rsd[B.row0 + i];
            }
            a.U[o] = uv;
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k)
        if (k < nc && (k & 1) == h && in && u16) {
            const double rhs = a.z[B.row0 + i];
            sv[k] = a.S[B.row0 + i] * a.rsd[B.row0 + i] * (rhs / jdiag(a, B, i, col_shift(a, B, k)));
        }
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k) sv[k] = wave_sum(sv[k]);
    if ((tid & 63) == 0)
#pragma unroll
        for (int k = 0; k < kMaxNC; ++k) red[tid >> 6][k] = sv[k];
    __syncthreads();
    if (tid < nc) {
        const int hk = tid & 1;   // the half that handled column tid: waves 2 hk, 2 hk + 1
        a.dot[B.dof + (static_cast<int64_t>(I) * kNDot + 4) * n + tid] = red[2 * hk][tid] + red[2 * hk + 1][tid];
    }
}

// ------------------------------------------------------------------------------------------
// The product's partial sums: one wave per item (block, tile row I, tiles J0 .. J1 <= I).
// ------------------------------------------------------------------------------------------
// Two kernels over the same item list, each taking the blocks of its storage (the other's items
// return at once): the uint16 integer Gram (the common case, held to 128 registers: 4 waves per
// SIMD keep enough row segments in flight) and the fp64 Sigma (blocks with missing calls, panels
// with n_ref > 16383; launched only when the plan has such blocks).
template <bool U16>
__device__ __forceinline__ void symv_body(const PcgArgs& a, const int4* __restrict__ items, int32_t n_items) {
    using namespace pcg;
    extern __shared__ double vlds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int e = blockIdx.x * kWaves + wave;
    if (e >= n_items) return;
    const int nc = a.ncopy;
    double* w = vlds + wave * wave_lds_doubles(nc);
    symv_item<U16>(a, items[e], lane, w, w + nc * kVS, w + 3 * nc * kVS, w + 3 * nc * kVS + 2 * nc * 64);
}
#ifndef PCG_SYMV_WAVES
#define PCG_SYMV_WAVES 2   // waves per SIMD the uint16 product is compiled for (a whole tile in flight per wave)
#endif
extern "C" __global__ __launch_bounds__(pcg::kThreads) __attribute__((amdgpu_waves_per_eu(PCG_SYMV_WAVES, 8)))
void dbslmm_pcg_symv16(PcgArgs a, const int4* __restrict__ items, int32_t n_items) {
    symv_body<true>(a, items, n_items);
}
extern "C" __global__ __launch_bounds__(pcg::kThreads)
void dbslmm_pcg_symv64(PcgArgs a, const int4* __restrict__ items, int32_t n_items) {
    symv_body<false>(a, items, n_items);
}

// ------------------------------------------------------------------------------------------
// w = M_c u for one tile row from its partial slots (fixed order), and the partial dots: per
// product column r.u, w.u, r.r; per copy x.x (a multi-shift block's copies share its one column).
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(pcg::kThreads) void dbslmm_pcg_rows(PcgArgs a, const int2* __restrict__ rows) {
    using namespace pcg;
    __shared__ double red[kThreads / 64][kMaxNC][4];
    __shared__ double sig[kMaxNC];
    const int2 it = rows[blockIdx.x];
    const int bi = it.x, I = it.y, tid = threadIdx.x;
    if (a.done[bi]) return;
    const PcgBlk B = a.blk[bi];
    const bool u16 = on_u16(a, B);
    const int n = a.ncopy, nc = B.nc;
    if (tid < nc)                        // sigma_k = S . (rsd o u) over the block (fixed order)
        sig[tid] = ordered_sum(a.dot + B.dof + 4 * n + tid, kNDot * n, 0, B.Tb, 0.0);
    __syncthreads();
    const int r = tid & (kT - 1), h = tid >> 7, i = I * kT + r;
    const bool in = i < B.m;
    const double Si = in ? a.S[B.row0 + i] : 0.0, ri = in ? a.rsd[B.row0 + i] : 0.0;
    const int nrun = (I + a.run) / a.run;   // runs of tile row I: ceil((I + 1) / run)
    double dv[kMaxNC][4];
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k)
#pragma unroll
        for (int f = 0; f < 4; ++f) dv[k][f] = 0.0;
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k) {
        if (k >= n || (k & 1) != h) continue;
        const int64_t o = k * a.vstride + B.vo + i;
        if (k < nc) {
            const double* pp = a.part + B.po + static_cast<int64_t>(I) * B.Ns * nc * kT + k * kT + r;
            double y = ordered_sum(pp, nc * kT, I, B.Tb, 0.0);
            y = ordered_sum(pp, nc * kT, B.Tb, B.Tb + nrun, y);
            const double dc = col_shift(a, B, k);
            const double rv = a.R[o];
            const double u = in ? rv / jdiag(a, B, i, dc) : 0.0;
            const double sh = i < B.ms ? dc : 0.0;
            double w = 0.0;
            if (in) {
                if (u16) w = a.tau * a.rn * ri * __builtin_fma(-Si, sig[k] * a.rn, y) + (1.0 - a.tau + sh) * u;
                else w = y + sh * u;
            }
            a.W[o] = w;
            dv[k][0] = rv * u;
            dv[k][1] = w * u;
            dv[k][2] = rv * rv;
        }
        const double xv = a.X[o];
        dv[k][3] = xv * xv;
    }
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k)
#pragma unroll
        for (int f = 0; f < 4; ++f) dv[k][f] = wave_sum(dv[k][f]);
    if ((tid & 63) == 0)
#pragma unroll
        for (int k = 0; k < kMaxNC; ++k)
#pragma unroll
            for (int f = 0; f < 4; ++f) red[tid >> 6][k][f] = dv[k][f];
    __syncthreads();
    if (tid < 4 * n) {
        const int k = tid >> 2, f = tid & 3, hk = k & 1;
        if (f == 3 || k < nc)
            a.dot[B.dof + (static_cast<int64_t>(I) * kNDot + f) * n + k] = red[2 * hk][k][f] + red[2 * hk + 1][k][f];
    }
    if (I == 0 && tid == 0) a.itb[bi] += 1;
}

// ------------------------------------------------------------------------------------------
// The iteration's coefficients and update for one tile row.  Every workgroup of a block sums the
// block's dots in the same order, so every tile row takes the same decisions; tile row 0 alone
// writes the recurrence state (the other parity than the one read), the convergence iteration
// and the block's done flag.
//   per-copy blocks: Jacobi-PCG per copy in the Chronopoulos-Gear form
//       gamma = r.u, delta = w.u, beta = gamma / gamma_prev, alpha = gamma / (delta - beta gamma / alpha_prev)
//       p = u + beta p, s = w + beta s, x += alpha p, r -= alpha s
//   multi-shift blocks (tools/multishift_check.py): the same for the seed (smallest shift, column
//   0, no preconditioner); copy c (shift e = d_c - d_seed >= 0) follows from the seed's scalars,
//   c' = alpha_k beta_k-1 / alpha_k-1:
//       zeta_k+1 = zeta_k zeta_k-1 / ((1 + c' + alpha_k e) zeta_k-1 - c' zeta_k)
//       alpha_c = alpha_k zeta_k+1 / zeta_k, beta_c = (zeta_k / zeta_k-1)^2 beta_k-1
//       p_c = zeta_k r + beta_c p_c, x_c += alpha_c p_c, |r_c| = |zeta_k| |r|
// Stopping per copy: |r_c| <= tol lambda_c |x_c|.
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(pcg::kThreads) void dbslmm_pcg_update(PcgArgs a, const int2* __restrict__ rows) {
    using namespace pcg;
    __shared__ double tot[kMaxNC][4];
    __shared__ double coef[kMaxNC][3];   // per copy: alpha, beta, zeta_k (multi-shift; 1 otherwise)
    __shared__ double seedc[2];          // multi-shift: the seed's alpha, beta
    __shared__ int run_s[kMaxNC];
    __shared__ double red[kThreads / 64][kMaxNC];
    const int2 it = rows[blockIdx.x];
    const int bi = it.x, I = it.y, tid = threadIdx.x;
    if (a.done[bi]) return;
    const PcgBlk B = a.blk[bi];
    const bool u16 = on_u16(a, B);
    const int n = a.ncopy, nc = B.nc;
    const int itn = a.itb[bi] - 1;       // the iteration whose dots the rows launch wrote
    const int par = itn & 1;
    if (tid < 4 * n) {
        const int k = tid >> 2, f = tid & 3;
        tot[k][f] = (f == 3 || k < nc) ? ordered_sum(a.dot + B.dof + f * n + k, kNDot * n, 0, B.Tb, 0.0) : 0.0;
    }
    __syncthreads();
    if (B.mshift) {
        if (tid == 0) {                  // the seed's coefficients (identical in every workgroup)
            const double gam = tot[0][0], del = tot[0][1];
            const double* q = a.qs + static_cast<int64_t>(B.sco) * kQS;
            double al, be = 0.0;
            if (itn == 0) {
                al = gam / del;
            } else {
                be = gam / q[2 * par];
                al = gam / (del - be * gam / q[2 * par + 1]);
            }
            seedc[0] = al;
            seedc[1] = be;
        }
        __syncthreads();
        if (tid < n) {
            const int c = tid;
            double* q = a.qs + static_cast<int64_t>(B.sco + c) * kQS;
            const double al = seedc[0], be = seedc[1];
            const double zk = q[4 + 2 * par], zk1 = q[4 + 2 * par + 1];
            const double rr = tot[0][2] * zk * zk, xx = tot[c][3];
            const double t = a.tol * (a.dshift[c] + 1.0 - a.tau);
            const bool conv = a.cnv[B.sco + c] != 0 || rr == 0.0 || rr <= t * t * xx;
            const double e = a.dshift[c] - a.dshift[a.seed];
            const double cp = itn == 0 ? 0.0 : al * be / a.qs[static_cast<int64_t>(B.sco) * kQS + 2 * par + 1];
            const double zn = zk * zk1 / ((1.0 + cp + al * e) * zk1 - cp * zk);
            coef[c][0] = al * zn / zk;
            coef[c][1] = zk1 != 0.0 ? (zk / zk1) * (zk / zk1) * be : 0.0;
            coef[c][2] = zk;
            run_s[c] = conv ? 0 : 1;
            if (I == 0) {
                if (conv && a.cnv[B.sco + c] == 0) a.cnv[B.sco + c] = itn + 1;
                q[4 + 2 * (par ^ 1)] = zn;
                q[4 + 2 * (par ^ 1) + 1] = zk;
            }
        }
        __syncthreads();
        if (I == 0 && tid == 0) {        // the seed's recurrence state (after every reader above)
            double* q = a.qs + static_cast<int64_t>(B.sco) * kQS;
            q[2 * (par ^ 1)] = tot[0][0];
            q[2 * (par ^ 1) + 1] = seedc[0];
        }
    } else {
        if (tid < n) {
            const int k = tid;
            const double gam = tot[k][0], del = tot[k][1], rr = tot[k][2], xx = tot[k][3];
            const double lam = B.ms == B.m ? a.dshift[k] + 1.0 - a.tau : 1.0 - a.tau;
            const double t = a.tol * lam;
            // converged: |r| <= tol lambda_min |x| (a bound on the relative error of x), or r = 0;
            // NaN never converges (the cap then reports it)
            const bool conv = a.cnv[B.sco + k] != 0 || rr == 0.0 || rr <= t * t * xx;
            double al = 0.0, be = 0.0;
            if (!conv) {
                double* q = a.qs + static_cast<int64_t>(B.sco + k) * kQS;
                if (itn == 0) {
                    al = gam / del;
                } else {
                    be = gam / q[2 * par];
                    al = gam / (del - be * gam / q[2 * par + 1]);
                }
                if (I == 0) {
                    q[2 * (par ^ 1)] = gam;
                    q[2 * (par ^ 1) + 1] = al;
                }
            } else if (I == 0 && a.cnv[B.sco + k] == 0) {
                a.cnv[B.sco + k] = itn + 1;
            }
            coef[k][0] = al;
            coef[k][1] = be;
            coef[k][2] = 1.0;
            run_s[k] = conv ? 0 : 1;
        }
        __syncthreads();
    }
    int running = 0;
    for (int k = 0; k < n; ++k) running += run_s[k];
    if (running == 0) {
        if (I == 0 && tid == 0) {
            a.done[bi] = 1;
            atomicSub(a.active, 1);
        }
        return;
    }
    const int r = tid & (kT - 1), h = tid >> 7, i = I * kT + r;
    const bool in = i < B.m;
    double sv[kMaxNC];
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k) sv[k] = 0.0;
    if (B.mshift) {
        if (in) {
            const int64_t o0 = B.vo + i;
            const double rv = a.R[o0];
#pragma unroll
            for (int c = 0; c < kMaxNC; ++c) {
                if (c >= n || (c & 1) != h || !run_s[c]) continue;
                const int64_t o = c * a.vstride + o0;
                const double p = __builtin_fma(coef[c][1], a.P[o], coef[c][2] * rv);
                a.P[o] = p;
                a.X[o] = __builtin_fma(coef[c][0], p, a.X[o]);
            }
            if (h == 0) {                // the seed's residual (column 0); P / X of the seed copy above
                const double al = seedc[0], be = seedc[1];
                const double sn = __builtin_fma(be, a.Sv[o0], a.W[o0]);
                const double rn = __builtin_fma(-al, sn, rv);
                a.Sv[o0] = sn;
                a.R[o0] = rn;
                a.U[o0] = u16 ? rn * a.rsd[B.row0 + i] : rn;
                if (u16) sv[0] = a.S[B.row0 + i] * a.rsd[B.row0 + i] * rn;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < kMaxNC; ++k) {
            if (k >= n || (k & 1) != h || !run_s[k] || !in) continue;
            const int64_t o = k * a.vstride + B.vo + i;
            const double al = coef[k][0], be = coef[k][1];
            const double dg = jdiag(a, B, i, a.dshift[k]);
            const double u = a.R[o] / dg;
            const double p = __builtin_fma(be, a.P[o], u);
            const double s = __builtin_fma(be, a.Sv[o], a.W[o]);
            const double x = __builtin_fma(al, p, a.X[o]);
            const double rn = __builtin_fma(-al, s, a.R[o]);
            a.P[o] = p;
            a.Sv[o] = s;
            a.X[o] = x;
            a.R[o] = rn;
            a.U[o] = u16 ? (rn / dg) * a.rsd[B.row0 + i] : rn / dg;
            if (u16) sv[k] = a.S[B.row0 + i] * a.rsd[B.row0 + i] * (rn / dg);
        }
    }
#pragma unroll
    for (int k = 0; k < kMaxNC; ++k) sv[k] = wave_sum(sv[k]);
    if ((tid & 63) == 0)
#pragma unroll
        for (int k = 0; k < kMaxNC; ++k) red[tid >> 6][k] = sv[k];
    __syncthreads();
    if (tid < nc && (B.mshift || run_s[tid])) {
        const int hk = tid & 1;
        a.dot[B.dof + (static_cast<int64_t>(I) * kNDot + 4) * n + tid] = red[2 * hk][tid] + red[2 * hk + 1][tid];
    }
}

// ------------------------------------------------------------------------------------------
// The small blocks' whole solve in one launch (round 6).  A block of at most kFTb tile rows on the
// uint16 Gram is solved by ONE workgroup per Krylov sequence (a multi-shift block: one for every
// copy; a block with large SNPs: one per copy) from the right-hand side to convergence (a persistent grid of one workgroup per CU
// takes the blocks from a counter, so the chip-wide kernels keep half of every CU): per iteration the block's quadrants are
// streamed once (the 8 x 8 lane sub-blocks and reduce-scatters of quad_mul16, next quadrant in
// flight), each wave adding its row and column sums into its own LDS copy of y (fixed order, no
// atomics), then w, the dots, the coefficients, the convergence test and the update exactly as
// dbslmm_pcg_rows / dbslmm_pcg_update compute them -- with no partial slots, no per-iteration
// launches and no hand-off between workgroups.  Thread t owns slots t + 256 q (q < kFPer): r, s
// and w in registers, U = rsd o u and x and p of every copy in LDS (x goes to the block's global
// vectors at the end).  The chip-wide kernels skip these blocks (init marks them
// done = 3); dbslmm_pcg_final writes their betas and status from x and cnv as for the others.
// ------------------------------------------------------------------------------------------
#ifndef PCG_BLOCK_DEPTH
#define PCG_BLOCK_DEPTH 3   // quadrant buffers per wave in dbslmm_pcg_block (2: one in flight)
#endif
namespace pcg {
// sum of v over the workgroup, every thread gets the total (fixed order: lanes, then waves 0..3)
template <int N>
__device__ __forceinline__ void block_sum(double (&v)[N], double* red, int tid) {
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = wave_sum(v[k]);
    __syncthreads();                          // (red free: its previous readers are past this)
    if ((tid & 63) == 0)
#pragma unroll
        for (int k = 0; k < N; ++k) red[(tid >> 6) * N + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = ((red[k] + red[N + k]) + red[2 * N + k]) + red[3 * N + k];
}
// LDS of n copies: y per wave, U, x and p of every copy, the block_sum scratch, the recurrence
// state and flags (56 / 88 KB at 1 / 3 copies: one workgroup per CU, and at 3 copies still room
// for a chip-wide product workgroup, 64 KB, beside it)
constexpr size_t block_lds_bytes(int n) {
    return sizeof(double) * ((5 + 2 * n) * kFRows + 4 * (3 + kMaxNC) + 12 + 3 * kMaxNC + 4);
}
}  // namespace pcg

// One list entry: block bi, copy cc (-1: a multi-shift block, every copy in one sequence; else one
// copy's own Jacobi-preconditioned sequence -- a block with large SNPs and several copies has one
// entry per copy, each on its own workgroup).
__device__ __forceinline__ void pcg_block_solve(const PcgArgs& a, int bi, int cc, int32_t maxit) {
    using namespace pcg;
    extern __shared__ double blds[];
    double* yw = blds;                       // [4][kFRows] per-wave product sums
    double* Ul = blds + 4 * kFRows;          // [kFRows] rsd o u
    const int n = a.ncopy;
    double* Xl = Ul + kFRows;                // [copy][kFRows] x (to global at the end)
    double* Pl = Xl + n * kFRows;            // [copy][kFRows] p
    double* red = Pl + n * kFRows;           // block_sum scratch
    if (a.done[bi] != 3) return;             // (monomorphic, or missing calls: the chip-wide path)
    const PcgBlk B = a.blk[bi];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int m = B.m, Tb = B.Tb;
    const bool msh = cc < 0;
    const int nx = msh ? n : 1;              // copies of x this sequence yields
    const double dc = msh ? col_shift(a, B, 0) : a.dshift[cc];   // the sequence's shift (the seed's: multi-shift)
    // ---- state: x = p = 0, r = z, s = w = 0, U = rsd o r / diag
    // (S and rsd of the thread's slots in registers: no global reads inside the iterations)
    double r[kFPer], sv[kFPer], wv[kFPer], Sr[kFPer], Rr[kFPer], sg[1] = {0.0};
#pragma unroll
    for (int q = 0; q < kFPer; ++q) {
        const int i = tid + kThreads * q;
        const bool in = i < m;
        r[q] = in ? a.z[B.row0 + i] : 0.0;
        Sr[q] = in ? a.S[B.row0 + i] : 0.0;
        Rr[q] = in ? a.rsd[B.row0 + i] : 0.0;
        sv[q] = wv[q] = 0.0;
        double u = 0.0;
        if (in) {
            u = (r[q] / jdiag(a, B, i, dc)) * Rr[q];
            sg[0] += Sr[q] * u;
        }
        Ul[i] = u;                           // (zero past m)
        for (int w = 0; w < 4; ++w) yw[w * kFRows + i] = 0.0;
        for (int c = 0; c < nx; ++c) Xl[c * kFRows + i] = Pl[c * kFRows + i] = 0.0;
    }
    block_sum(sg, red, tid);
    double sig = sg[0];
    // quadrants of the block's lower triangle (rows and columns < m), dealt to the waves in turn
    const int Q = (m + 63) / 64;
    const int nq = Q * (Q + 1) / 2;
    const int64_t ld16 = static_cast<int64_t>(Tb) * kT;
    const int rg = lane >> 3, cg = lane & 7;
    auto quad_of = [&](int t, int& qi, int& qj) {   // t-th lower-triangle quadrant, row-major
        qi = static_cast<int>((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
        while (qi * (qi + 1) / 2 > t) --qi;
        while ((qi + 1) * (qi + 2) / 2 <= t) ++qi;
        qj = t - qi * (qi + 1) / 2;
    };
    // The block's Gram through a range-checked buffer descriptor: a sub-block row wholly above the
    // diagonal or past m, and every quadrant past the last (t >= nq), reads at an offset beyond the
    // range -- zeros with no memory access -- so each load() issues exactly 8 loads unconditionally
    // and the waits before mult() count only the quadrant they need (with the loads under branches
    // the compiler waited for all of them, vmcnt(0): one quadrant in flight, 16.5 GB/s per CU).
    const __amdgpu_buffer_rsrc_t g16 = g16_rsrc(a.G16 + B.off16, static_cast<uint32_t>(ld16 * ld16 * 2));
    auto load = [&](int t, pcg_u4 (&raw)[8]) {
        int qi, qj;
        quad_of(t, qi, qj);
        const int r0 = 64 * qi + 8 * rg, c0 = 64 * qj + 8 * cg;
        const bool skip = t >= nq || c0 >= m || (qi == qj && cg > rg);
        const uint32_t o = static_cast<uint32_t>((r0 * static_cast<int>(ld16) + c0) * 2);
#pragma unroll
        for (int rr = 0; rr < 8; ++rr)
            raw[rr] = __builtin_amdgcn_raw_buffer_load_b128(
                g16, (skip || r0 + rr >= m) ? kG16Oob : o + static_cast<uint32_t>(rr * ld16 * 2), 0, 0);
    };
    auto mult = [&](int t, const pcg_u4 (&raw)[8]) {
        int qi, qj;
        quad_of(t, qi, qj);
        const bool dq = qi == qj;
        double vi[8], vj[8], racc[8], cacc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            vi[q] = Ul[64 * qi + 8 * rg + q];
            vj[q] = Ul[64 * qj + 8 * cg + q];
            racc[q] = cacc[q] = 0.0;
        }
        if (!dq) {
#pragma unroll
            for (int rr = 0; rr < 8; ++rr)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t w = raw[rr][c >> 1];
                    const double g = (c & 1) ? cvt_hi(w) : cvt_lo(w);
                    racc[rr] = __builtin_fma(g, vj[c], racc[rr]);
                    cacc[c] = __builtin_fma(g, vi[rr], cacc[c]);
                }
        } else {
#pragma unroll
            for (int rr = 0; rr < 8; ++rr)
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const uint32_t w = raw[rr][c >> 1];
                    const double g = (c & 1) ? cvt_hi(w) : cvt_lo(w);
                    const int dd = 8 * (cg - rg) + c - rr;   // j - i
                    racc[rr] = __builtin_fma(dd <= 0 ? g : 0.0, vj[c], racc[rr]);
                    cacc[c] = __builtin_fma(dd < 0 ? g : 0.0, vi[rr], cacc[c]);
                }
        }
        double* y = yw + wave * kFRows;
        const int ri = 64 * qi + 8 * rg + cg, ci = 64 * qj + 8 * cg + rg;
        y[ri] += rscatter8<4, 2, 1>(racc, lane);
        wave_fence();                          // (a diagonal quadrant: the row sums land first)
        y[ci] += rscatter8<32, 16, 8>(cacc, lane);
    };
    // recurrence state: thread 0 keeps it in LDS (kept out of the registers of the product loop)
    double* st = red + 4 * (3 + kMaxNC);     // [0] gamma_prev, [1] alpha_prev, [2] alpha, [3] beta,
                                             // [4 + c] zeta_k, [8 + c] zeta_k-1, [12 + 3c ..] coef
    int* flag = reinterpret_cast<int*>(st + 12 + 3 * kMaxNC);   // [c] converged, [kMaxNC] running
    if (tid == 0) {
        for (int c = 0; c < kMaxNC; ++c) {
            st[4 + c] = st[8 + c] = 1.0;
            flag[c] = c >= n;
        }
    }
    int it = 0;
    for (; it < maxit; ++it) {
        // ---- product y = G U (U in LDS since the last update)
        __syncthreads();
        {
#if PCG_BLOCK_DEPTH == 3
            // two quadrants in flight while one is multiplied (three register buffers, rotated)
            // (loads past the last quadrant are out of range: issued, no memory access)
            pcg_u4 ra[8], rb[8], rc[8];
            int t = wave;
            load(t, ra);
            load(t + 4, rb);
            while (t < nq) {
                load(t + 8, rc);
                mult(t, ra);
                t += 4;
                if (t >= nq) break;
                load(t + 8, ra);
                mult(t, rb);
                t += 4;
                if (t >= nq) break;
                load(t + 8, rb);
                mult(t, rc);
                t += 4;
            }
#else
            pcg_u4 ra[8], rb[8];
            int t = wave;
            load(t, ra);
            while (t < nq) {
                load(t + 4, rb);
                mult(t, ra);
                t += 4;
                if (t >= nq) break;
                load(t + 4, ra);
                mult(t, rb);
                t += 4;
            }
#endif
        }
        __syncthreads();
        // ---- w = M u, dots r.u, w.u, r.r and x.x per copy (dbslmm_pcg_rows)
        double d[3 + kMaxNC];
#pragma unroll
        for (int k = 0; k < 3 + kMaxNC; ++k) d[k] = 0.0;
#pragma unroll
        for (int q = 0; q < kFPer; ++q) {
            const int i = tid + kThreads * q;
            double y = 0.0;
            if (i < Tb * kT) {
                y = ((yw[i] + yw[kFRows + i]) + yw[2 * kFRows + i]) + yw[3 * kFRows + i];
#pragma unroll
                for (int w = 0; w < 4; ++w) yw[w * kFRows + i] = 0.0;
            }
            if (i < m) {
                const double Si = Sr[q], ri = Rr[q];
                const double u = r[q] / jdiag(a, B, i, dc);
                const double sh = i < B.ms ? dc : 0.0;
                const double w = a.tau * a.rn * ri * __builtin_fma(-Si, sig * a.rn, y) + (1.0 - a.tau + sh) * u;
                wv[q] = w;
                d[0] += r[q] * u;
                d[1] += w * u;
                d[2] += r[q] * r[q];
                for (int c = 0; c < nx; ++c) {
                    const double xv = Xl[c * kFRows + i];
                    d[3 + c] += xv * xv;
                }
            }
        }
        block_sum(d, red, tid);
        // ---- coefficients and convergence (dbslmm_pcg_update), by thread 0
        if (tid == 0) {
            const double gam = d[0], del = d[1], rr = d[2];
            double al, be = 0.0;
            if (it == 0) {
                al = gam / del;
            } else {
                be = gam / st[0];
                al = gam / (del - be * gam / st[1]);
            }
            int running = 0;
            if (msh) {
                const double cp = it == 0 ? 0.0 : al * be / st[1];
                for (int c = 0; c < n; ++c) {
                    const double zk = st[4 + c], zk1 = st[8 + c];
                    const double t = a.tol * (a.dshift[c] + 1.0 - a.tau);
                    const double rrc = rr * zk * zk;
                    if (!flag[c] && (rrc == 0.0 || rrc <= t * t * d[3 + c])) {
                        flag[c] = 1;
                        a.cnv[B.sco + c] = it + 1;
                    }
                    const double e = a.dshift[c] - a.dshift[a.seed];
                    const double zn = zk * zk1 / ((1.0 + cp + al * e) * zk1 - cp * zk);
                    st[12 + 3 * c] = al * zn / zk;
                    st[12 + 3 * c + 1] = zk1 != 0.0 ? (zk / zk1) * (zk / zk1) * be : 0.0;
                    st[12 + 3 * c + 2] = zk;
                    st[8 + c] = zk;
                    st[4 + c] = zn;
                    running += flag[c] ? 0 : 1;
                }
            } else {                          // one copy (n = 1), Jacobi-preconditioned
                const double lam = B.ms == B.m ? dc + 1.0 - a.tau : 1.0 - a.tau;
                const double t = a.tol * lam;
                if (rr == 0.0 || rr <= t * t * d[3]) {
                    flag[0] = 1;
                    a.cnv[B.sco + cc] = it + 1;
                }
                running = flag[0] ? 0 : 1;
            }
            st[0] = gam;
            st[1] = al;
            st[2] = al;
            st[3] = be;
            flag[kMaxNC] = running;
        }
        __syncthreads();
        if (flag[kMaxNC] == 0) break;
        const double al = st[2], be = st[3];
        // ---- update p, x (every running copy), s, r, U
        double sg2[1] = {0.0};
#pragma unroll
        for (int q = 0; q < kFPer; ++q) {
            const int i = tid + kThreads * q;
            if (i >= m) continue;
            const double rsd_i = Rr[q];
            double rn;
            if (msh) {
                for (int c = 0; c < n; ++c) {
                    if (flag[c]) continue;
                    const int o = c * kFRows + i;
                    const double pv = __builtin_fma(st[12 + 3 * c + 1], Pl[o], st[12 + 3 * c + 2] * r[q]);
                    Pl[o] = pv;
                    Xl[o] = __builtin_fma(st[12 + 3 * c], pv, Xl[o]);
                }
                const double sn = __builtin_fma(be, sv[q], wv[q]);
                rn = __builtin_fma(-al, sn, r[q]);
                sv[q] = sn;
                r[q] = rn;
                Ul[i] = rn * rsd_i;
            } else {
                const double dg = jdiag(a, B, i, dc);
                const double u = r[q] / dg;
                const double pv = __builtin_fma(be, Pl[i], u);
                const double sn = __builtin_fma(be, sv[q], wv[q]);
                Pl[i] = pv;
                Xl[i] = __builtin_fma(al, pv, Xl[i]);
                rn = __builtin_fma(-al, sn, r[q]);
                sv[q] = sn;
                r[q] = rn;
                Ul[i] = (rn / dg) * rsd_i;
            }
            sg2[0] += Sr[q] * Ul[i];
        }
        block_sum(sg2, red, tid);
        sig = sg2[0];
    }
    // x to the block's global vectors (dbslmm_pcg_final reads it); each thread its own rows
#pragma unroll
    for (int q = 0; q < kFPer; ++q) {
        const int i = tid + kThreads * q;
        if (i < m)
            for (int c = 0; c < nx; ++c) a.X[(msh ? c : cc) * a.vstride + B.vo + i] = Xl[c * kFRows + i];
    }
    if (tid == 0) atomicMax(a.itb + bi, it + (it < maxit ? 1 : 0));   // (several copies: the slowest)
}

extern "C" __global__ __launch_bounds__(pcg::kThreads)
#if PCG_BLOCK_DEPTH == 3
// one wave per SIMD (its LDS allows one workgroup per CU); at most 312 VGPRs, so a chip-wide
// product wave (192) still fits beside it on every SIMD
__attribute__((amdgpu_waves_per_eu(1, 8), amdgpu_num_vgpr(312)))
#else
__attribute__((amdgpu_waves_per_eu(2, 8)))
#endif
void dbslmm_pcg_block(PcgArgs a, const int2* __restrict__ list, int32_t n_list, int32_t* __restrict__ next,
                      int32_t maxit) {
    // blocks taken in list order (biggest first) by whichever workgroup is free: the next index from
    // one counter (zeroed before the launch); which workgroup solves a block never changes its result
    __shared__ int e_s;
    for (;;) {
        __syncthreads();                     // (the previous block's LDS readers are done)
        if (threadIdx.x == 0) e_s = atomicAdd(next, 1);
        __syncthreads();
        const int e = e_s;
        if (e >= n_list) break;
        pcg_block_solve(a, list[e].x, list[e].y, maxit);
    }
}

// ------------------------------------------------------------------------------------------
// beta = x / sqrt(n) into the caller's order (every copy), status per copy: MONOMORPHIC (beta NaN),
// NOT_CONVERGED (the iterate at the cap), OK.  One workgroup per tile row.
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(pcg::kThreads) void dbslmm_pcg_final(PcgArgs a, const int2* __restrict__ rows) {
    using namespace pcg;
    const int2 it = rows[blockIdx.x];
    const int bi = it.x, I = it.y, tid = threadIdx.x;
    const PcgBlk B = a.blk[bi];
    const bool mono = a.done[bi] == 2;
    const int r = tid & (kT - 1), h = tid >> 7, i = I * kT + r;
    if (i < B.m) {
        const int so = a.slot_out[B.row0 + i];
        for (int k = h; k < a.ncopy; k += 2) {
            const double bv = mono ? __builtin_nan("") : a.X[k * a.vstride + B.vo + i] * a.inv_sqrt_n;
            if (so >= 0) a.beta_s[k * a.ns + so] = bv;
            else a.beta_l[k * a.nl - 1 - so] = bv;
        }
    }
    if (I == 0 && tid < a.ncopy) {
        const int st = mono ? DBSLMM_BLOCK_MONOMORPHIC
                            : a.cnv[B.sco + tid] == 0 ? DBSLMM_BLOCK_NOT_CONVERGED : DBSLMM_BLOCK_OK;
        a.status[tid * a.nbk + a.blk_id[B.blk]] = st;
    }
}
