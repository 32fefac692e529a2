// kernels.hip -- gfx950 (CDNA4) kernels of the per-LD-block effect-size solver.
//
// The hot path of DBSLMMFIT::est (reference scr/dbslmmfit.cpp:56-363) as three launches:
//
//   dbslmm_unpack_stats  IO::readSNPIm + nomalizeVec statistics (scr/dtpr.cpp:285-380):
//                        2-bit PLINK rows -> int8 dosages {0,1,2, 0x80 = missing} in a
//                        block-ordered slot matrix G[slot][individual], plus exact integer
//                        per-SNP count / sum / sum-of-squares and the fp64 mean, 1/sd (N-1).
//                        HBM-bound streaming kernel, one wave per SNP row.
//   dbslmm_gram_i8       estBlock's LD matrices (scr/dbslmmfit.cpp:697-709, 751-756) as ONE
//                        joint Gram per block over [small | large] SNPs on i8 MFMA
//                        (v_mfma_i32_32x32x32_i8, exact int32 accumulation) with an fp64
//                        epilogue that centres, standardises and applies tau:
//                          Sigma_ij = tau/n_ref * C_ij /(s_i s_j) + (1-tau) delta_ij,
//                          C_ij = G_ij - S_i S_j / n   (no missing calls in the block)
//                        Blocks with missing calls add the observed-mask Grams (4 MFMAs/step).
//   dbslmm_chol_solve    the whole per-block solve (PCGm/PCGv at :713-729, :758-764) as one
//                        SPD solve of the joint matrix
//                          M = [[Sigma_ss + I/(sigma_s n), Sigma_sl], [Sigma_ls, Sigma_ll]],
//                          beta = M^{-1} [z_s; z_l] / sqrt(n)
//                        (block elimination of M reproduces beta_l = S^{-1}(z_l - Sigma_ls q)/sqrt n
//                        and beta_s = (q - P beta_l sqrt n)/sqrt n of :714-729 exactly; see
//                        DESIGN.md).  fp64 blocked right-looking Cholesky, one workgroup per
//                        block, 32x32 tiles staged in LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kWave = 64;
constexpr int kTile = 32;          // gram / cholesky tile edge (SNP slots)
constexpr int kLdsStride = 33;     // padded LDS row stride (doubles) -> conflict-free column reads

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// 4 bytes starting at an arbitrary byte offset, from two aligned dword loads.
// The .bed image keeps its 3 magic bytes so row starts are generally unaligned.
__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* __restrict__ base, int64_t off) {
    const int64_t a = off & ~int64_t(3);
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(base + a);
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(base + a + 4);
    return __builtin_amdgcn_alignbyte(w1, w0, static_cast<uint32_t>(off & 3));
}

// Expand one packed dword (16 genotype codes, code j in bits 2j..2j+1) into 16 int8 dosages.
// Output word k holds codes {k, 4+k, 8+k, 12+k} in bytes 0..3: individuals are stored in a
// fixed within-16 permutation, which every Gram entry is invariant to (it sums over all
// individuals of two rows stored the same way).  code 0 -> 2, 2 -> 1, 3 -> 0, 1 -> 0x80 (missing).
__device__ __forceinline__ v4i expand16(uint32_t w, uint32_t valid_mask_2bit) {
    // padding individuals (>= n_ref) must contribute 0: force their code to 3 (dosage 0)
    w |= ~valid_mask_2bit & 0x55555555u;
    w |= (~valid_mask_2bit & 0x55555555u) << 1;
    v4i out;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t y = (w >> (2 * k)) & 0x03030303u;
        const uint32_t L = y & 0x01010101u;
        const uint32_t H = (y >> 1) & 0x01010101u;
        const uint32_t miss = L & ~H;
        const uint32_t dose = 0x02020202u - L - H - miss;   // per byte: 2,1,0 or 0 for missing
        out[k] = static_cast<int>(dose | (miss << 7));
    }
    return out;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Kernel 1: unpack + per-SNP statistics.  One wave per slot (SNP row of a block), 4 waves/WG.
//   G (optional)   [n_slots][kpad] int8; rows of padding slots (pos < 0) are written as zeros.
//   stat_*         exact integer statistics over the n_ref individuals.
//   mu, rsd, S     fp64: mean over observed calls (= the imputation value, dtpr.cpp:358),
//                  1/sd with the N-1 divisor (nomalizeVec), sum of observed dosages.
//   maf (optional) min(af, 1-af), af = mu/2 (dtpr.cpp:361-362).
//   block_flags    bit 0 set when a slot of the block has a missing call.
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void dbslmm_unpack_stats(
    const uint8_t* __restrict__ bed, int32_t n_ref, int64_t bytes_per_snp,
    const int32_t* __restrict__ slot_pos, const int32_t* __restrict__ slot_block, int32_t n_slots,
    int8_t* __restrict__ G, int64_t kpad,
    double* __restrict__ S_out, double* __restrict__ mu_out, double* __restrict__ rsd_out,
    double* __restrict__ maf_out, int32_t* __restrict__ block_flags) {
    const int lane = threadIdx.x & (kWave - 1);
    const int slot = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (slot >= n_slots) return;
    const int32_t pos = slot_pos[slot];
    const int64_t n_words = kpad / 16;          // 16 individuals per lane-word
    int8_t* grow = G ? G + static_cast<int64_t>(slot) * kpad : nullptr;
    if (pos < 0) {                              // padding slot
        if (grow)
            for (int64_t w = lane; w < n_words; w += kWave)
                *reinterpret_cast<v4i*>(grow + 16 * w) = v4i{0, 0, 0, 0};
        if (lane == 0) {
            if (S_out) S_out[slot] = 0.0;
            if (mu_out) mu_out[slot] = 0.0;
            if (rsd_out) rsd_out[slot] = 0.0;
            if (maf_out) maf_out[slot] = 0.0;
        }
        return;
    }
    const int64_t row_off = 3 + static_cast<int64_t>(pos) * bytes_per_snp;
    int cnt = 0, sum = 0, sq = 0, nmiss = 0;
    for (int64_t w = lane; w < n_words; w += kWave) {
        const int64_t first = 16 * w;
        const int nv = static_cast<int>(min<int64_t>(16, max<int64_t>(0, n_ref - first)));
        uint32_t word = 0;
        if (nv > 0) word = load_u32_any(bed, row_off + 4 * w);
        const uint32_t vmask = nv >= 16 ? 0x55555555u : ((1u << (2 * nv)) - 1u) & 0x55555555u;
        const uint32_t lo = word & vmask;
        const uint32_t hi = (word >> 1) & vmask;
        const int n_miss = __builtin_popcount(lo & ~hi);
        const int n_two = __builtin_popcount(~lo & ~hi & vmask);
        const int n_one = __builtin_popcount(~lo & hi);
        nmiss += n_miss;
        cnt += __builtin_popcount(vmask) - n_miss;
        sum += 2 * n_two + n_one;
        sq += 4 * n_two + n_one;
        if (grow) *reinterpret_cast<v4i*>(grow + first) = expand16(word, vmask);
    }
    cnt = wave_sum_i32(cnt);
    sum = wave_sum_i32(sum);
    sq = wave_sum_i32(sq);
    nmiss = wave_sum_i32(nmiss);
    if (lane == 0) {
        const double dc = static_cast<double>(cnt);
        const double ds = static_cast<double>(sum);
        const double mu = ds / dc;                                   // imputation value
        const double css = static_cast<double>(sq) - ds * ds / dc;  // centred sum of squares
        const double sd = sqrt(css / static_cast<double>(n_ref - 1));
        if (S_out) S_out[slot] = ds;
        if (mu_out) mu_out[slot] = mu;
        if (rsd_out) rsd_out[slot] = 1.0 / sd;                      // +inf when monomorphic
        if (maf_out) {
            const double af = 0.5 * mu;
            maf_out[slot] = af < 1.0 - af ? af : 1.0 - af;
        }
        if (nmiss > 0 && block_flags) atomicOr(block_flags + slot_block[slot], 1);
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 2: grouped joint Gram on i8 MFMA.  One wave = one 32x32 output tile (block, ti, tj),
// ti >= tj, K loop over the padded individuals 32 at a time.  Lane l loads 16 contiguous bytes
// of row (l & 31) at k-offset 16*(l >> 5) for both operands (identical k-permutation on the A
// and B side, so any lane->k assignment the instruction uses is summed consistently).
// Output: row-major lower triangle of the block's joint matrix
//     Sigma (no d shift; the Cholesky kernel adds 1/(sigma_s n) on the small diagonal).
// ------------------------------------------------------------------------------------------
struct GramTile { int32_t block, ti, tj, pad; };

extern "C" __global__ __launch_bounds__(256) void dbslmm_gram_i8(
    const int8_t* __restrict__ G, int64_t kpad,
    const GramTile* __restrict__ tiles, int32_t n_tiles,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ld, const int64_t* __restrict__ blk_matoff,
    const int32_t* __restrict__ block_flags,
    const double* __restrict__ S, const double* __restrict__ mu, const double* __restrict__ rsd,
    double n_ref_d, double pad_k, double tau, double* __restrict__ M) {
    const int lane = threadIdx.x & (kWave - 1);
    const int t = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (t >= n_tiles) return;
    const GramTile tile = tiles[t];
    const int b = tile.block;
    const int row0 = blk_row0[b];
    const int m = blk_m[b];
    const int ld = blk_ld[b];
    const int64_t moff = blk_matoff[b];
    const bool missing = (block_flags[b] & 1) != 0;

    const int8_t* pa = G + static_cast<int64_t>(row0 + kTile * tile.ti + (lane & 31)) * kpad + 16 * (lane >> 5);
    const int8_t* pb = G + static_cast<int64_t>(row0 + kTile * tile.tj + (lane & 31)) * kpad + 16 * (lane >> 5);

    v16i acc = {0};
    v16i acc_go = {0}, acc_og = {0}, acc_oo = {0};
    if (!missing) {
        int64_t k = 0;
        for (; k + 128 <= kpad; k += 128) {
            const v4i a0 = *reinterpret_cast<const v4i*>(pa + k);
            const v4i b0 = *reinterpret_cast<const v4i*>(pb + k);
            const v4i a1 = *reinterpret_cast<const v4i*>(pa + k + 32);
            const v4i b1 = *reinterpret_cast<const v4i*>(pb + k + 32);
            const v4i a2 = *reinterpret_cast<const v4i*>(pa + k + 64);
            const v4i b2 = *reinterpret_cast<const v4i*>(pb + k + 64);
            const v4i a3 = *reinterpret_cast<const v4i*>(pa + k + 96);
            const v4i b3 = *reinterpret_cast<const v4i*>(pb + k + 96);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a1, b1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a2, b2, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a3, b3, acc, 0, 0, 0);
        }
        for (; k < kpad; k += 32) {
            const v4i a0 = *reinterpret_cast<const v4i*>(pa + k);
            const v4i b0 = *reinterpret_cast<const v4i*>(pb + k);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a0, b0, acc, 0, 0, 0);
        }
    } else {
        // x = dosage or 0x80: g = x & 3 (0 for missing), o = 1 - (x >> 7)
        for (int64_t k = 0; k < kpad; k += 32) {
            const v4i a0 = *reinterpret_cast<const v4i*>(pa + k);
            const v4i b0 = *reinterpret_cast<const v4i*>(pb + k);
            v4i ga, oa, gb, ob;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t xa = static_cast<uint32_t>(a0[q]);
                const uint32_t xb = static_cast<uint32_t>(b0[q]);
                ga[q] = static_cast<int>(xa & 0x03030303u);
                gb[q] = static_cast<int>(xb & 0x03030303u);
                oa[q] = static_cast<int>((~xa >> 7) & 0x01010101u);
                ob[q] = static_cast<int>((~xb >> 7) & 0x01010101u);
            }
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(ga, gb, acc, 0, 0, 0);
            acc_go = __builtin_amdgcn_mfma_i32_32x32x32_i8(ga, ob, acc_go, 0, 0, 0);
            acc_og = __builtin_amdgcn_mfma_i32_32x32x32_i8(oa, gb, acc_og, 0, 0, 0);
            acc_oo = __builtin_amdgcn_mfma_i32_32x32x32_i8(oa, ob, acc_oo, 0, 0, 0);
        }
    }

    // fp64 epilogue.  C/D map of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    const int j = lane & 31;
    const int lj = kTile * tile.tj + j;
    const int sj = row0 + lj;
    const double Sj = lj < m ? S[sj] : 0.0;
    const double muj = lj < m ? mu[sj] : 0.0;
    const double rj = lj < m ? rsd[sj] : 0.0;
    const double scale = tau / n_ref_d;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int li = kTile * tile.ti + i;
        if (li >= m || lj >= m) continue;
        const int si = row0 + li;
        double c;
        if (!missing) {
            c = static_cast<double>(acc[r]) - S[si] * Sj / n_ref_d;
        } else {
            const double mui = mu[si];
            c = static_cast<double>(acc[r]) - muj * static_cast<double>(acc_go[r]) -
                mui * static_cast<double>(acc_og[r]) +
                mui * muj * (static_cast<double>(acc_oo[r]) - pad_k);   // padding counts as observed
        }
        double v = scale * (c * rsd[si] * rj);
        if (li == lj) v += 1.0 - tau;
        M[moff + static_cast<int64_t>(li) * ld + lj] = v;
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 3: per-block fp64 Cholesky of the joint matrix + forward/back substitution.
// One workgroup (256 threads, 4 waves) per block, blocks visited largest first (order[]).
// M is row-major, lower triangle valid (tile (I,J), I >= J); tiles of 32.
// LDS: D (diag tile, 32x33) + red (8x32) + per-wave staging (2 x 32x33 doubles) when
// the block has more than one tile (dynamic LDS size chosen by the host per launch).
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void dbslmm_chol_solve(
    double* __restrict__ M, const int32_t* __restrict__ order, int32_t n_blocks,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ms, const int32_t* __restrict__ blk_ld,
    const int64_t* __restrict__ blk_matoff,
    const double* __restrict__ z_slot, const int32_t* __restrict__ slot_out,
    const double* __restrict__ rsd, double dshift, double inv_sqrt_n,
    double* __restrict__ y, double* __restrict__ beta_s, double* __restrict__ beta_l,
    int32_t* __restrict__ status, int32_t* __restrict__ blk_id) {
    // one dynamic LDS array (no static __shared__: keeps the fp64 carve 16-B aligned)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    int* s_fail = reinterpret_cast<int*>(lds);  // 16 B header
    double* D = lds + 2;                       // 32 x 33
    double* red = D + kTile * kLdsStride;      // 8 x 32
    double* stage = red + 8 * kTile;           // 4 waves x 2 x 32 x 33 (only when T > 1)

    if (blockIdx.x >= static_cast<unsigned>(n_blocks)) return;
    const int b = order[blockIdx.x];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const int row0 = blk_row0[b];
    const int m = blk_m[b];
    const int ms = blk_ms[b];
    const int ld = blk_ld[b];
    const int T = ld / kTile;
    double* A = M + blk_matoff[b];
    if (tid == 0) *s_fail = 0;
    __syncthreads();

    for (int kb = 0; kb < T; ++kb) {
        // (1) diagonal tile -> LDS, with the 1/(sigma_s n) shift on small SNPs, identity padding
        for (int e = tid; e < kTile * kTile; e += 256) {
            const int r = e >> 5, c = e & 31;
            const int gr = kTile * kb + r, gc = kTile * kb + c;
            double v;
            if (gr < m && gc < m) {
                v = A[static_cast<int64_t>(gr) * ld + gc];
                if (gr == gc && gr < ms) v += dshift;
            } else {
                v = (r == c) ? 1.0 : 0.0;
            }
            D[r * kLdsStride + c] = v;
        }
        __syncthreads();
        // (2) unblocked right-looking Cholesky of D (lower)
        for (int jj = 0; jj < kTile; ++jj) {
            __syncthreads();                            // previous trailing update complete
            const double djj = D[jj * kLdsStride + jj];
            const double d = sqrt(djj);
            if (!(djj > 0.0) && tid == 0 && *s_fail == 0) *s_fail = kTile * kb + jj + 1;
            if (tid > jj && tid < kTile) D[tid * kLdsStride + jj] /= d;
            __syncthreads();                            // every thread has read D[jj][jj]
            if (tid == 0) D[jj * kLdsStride + jj] = d;
            const int rem = kTile - 1 - jj;            // trailing rows jj+1..31
            for (int e = tid; e < rem * rem; e += 256) {
                const int i = jj + 1 + e / rem, k = jj + 1 + e % rem;
                if (k <= i) D[i * kLdsStride + k] -= D[i * kLdsStride + jj] * D[k * kLdsStride + jj];
            }
        }
        __syncthreads();
        for (int e = tid; e < kTile * kTile; e += 256) {
            const int r = e >> 5, c = e & 31;
            const int gr = kTile * kb + r, gc = kTile * kb + c;
            if (c <= r && gr < m && gc < m) A[static_cast<int64_t>(gr) * ld + gc] = D[r * kLdsStride + c];
        }
        // (3) panel: rows below the diagonal tile solve x * L_kk^T = a (one thread per row)
        for (int row = kTile * (kb + 1) + tid; row < kTile * T; row += 256) {
            if (row >= m) continue;
            double x[kTile];
            double* prow = A + static_cast<int64_t>(row) * ld + kTile * kb;
#pragma unroll
            for (int c = 0; c < kTile; ++c) x[c] = (kTile * kb + c < m) ? prow[c] : 0.0;
#pragma unroll
            for (int c = 0; c < kTile; ++c) {
                double s = x[c];
#pragma unroll
                for (int c2 = 0; c2 < c; ++c2) s -= x[c2] * D[c * kLdsStride + c2];
                x[c] = s / D[c * kLdsStride + c];
            }
#pragma unroll
            for (int c = 0; c < kTile; ++c)
                if (kTile * kb + c < m) prow[c] = x[c];
        }
        __syncthreads();
        // (4) trailing update C_IJ -= L_I L_J^T over pairs kb < J <= I < T
        const int nt = T - kb - 1;
        if (nt > 0) {
            double* WI = stage + wave * 2 * kTile * kLdsStride;
            double* WJ = WI + kTile * kLdsStride;
            const int npairs = nt * (nt + 1) / 2;
            for (int p = wave; p < npairs; p += 4) {
                // p -> (I, J) with 0 <= J <= I < nt (row-wise enumeration)
                int I = static_cast<int>((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
                while ((I + 1) * (I + 2) / 2 <= p) ++I;
                while (I * (I + 1) / 2 > p) --I;
                const int J = p - I * (I + 1) / 2;
                const int gI = kb + 1 + I, gJ = kb + 1 + J;
                for (int e = lane; e < kTile * kTile; e += kWave) {
                    const int r = e >> 5, c = e & 31;
                    const int rI = kTile * gI + r, rJ = kTile * gJ + r;
                    WI[r * kLdsStride + c] = rI < m ? A[static_cast<int64_t>(rI) * ld + kTile * kb + c] : 0.0;
                    WJ[r * kLdsStride + c] = rJ < m ? A[static_cast<int64_t>(rJ) * ld + kTile * kb + c] : 0.0;
                }
                wave_sync();
                const int c = lane & 31;
                const int rb = 16 * (lane >> 5);
                double acc[16];
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) acc[rr] = 0.0;
#pragma unroll 4
                for (int k = 0; k < kTile; ++k) {
                    const double bj = WJ[c * kLdsStride + k];
#pragma unroll
                    for (int rr = 0; rr < 16; ++rr) acc[rr] += WI[(rb + rr) * kLdsStride + k] * bj;
                }
                const int gc = kTile * gJ + c;
#pragma unroll
                for (int rr = 0; rr < 16; ++rr) {
                    const int gr = kTile * gI + rb + rr;
                    if (gr < m && gc < m && gc <= gr) A[static_cast<int64_t>(gr) * ld + gc] -= acc[rr];
                }
                wave_sync();
            }
        }
        __syncthreads();
    }

    const int fail = *s_fail;
    double* yb = y + row0;
    if (fail == 0) {
        // forward: L y = z
        for (int I = 0; I < T; ++I) {
            // partial dot products of rows of tile I with y[0 .. 32I): wave w -> rows w, w+4, ..
            for (int rr = wave; rr < kTile; rr += 4) {
                const int gr = kTile * I + rr;
                double s = 0.0;
                if (gr < m) {
                    const double* prow = A + static_cast<int64_t>(gr) * ld;
                    for (int c = lane; c < kTile * I; c += kWave) s += prow[c] * yb[c];
                }
                s = wave_sum_f64(s);
                if (lane == 0) red[rr] = s;
            }
            __syncthreads();
            if (tid < kTile) {
                const int gr = kTile * I + tid;
                double v = gr < m ? z_slot[row0 + gr] - red[tid] : 0.0;
                // diag tile solve with lanes 0..31 (wave 0)
                for (int c = 0; c < kTile; ++c) {
                    const int gc = kTile * I + c;
                    const double Lcc = gc < m ? A[static_cast<int64_t>(gc) * ld + gc] : 1.0;
                    const double xc = __shfl(v, c, kWave) / Lcc;
                    if (tid == c) v = xc;
                    else if (tid > c && gr < m && gc < m) v -= A[static_cast<int64_t>(gr) * ld + gc] * xc;
                }
                if (gr < m) yb[gr] = v;
            }
            __syncthreads();
        }
        // backward: L^T x = y
        for (int I = T - 1; I >= 0; --I) {
            const int c = tid & 31, g = tid >> 5;
            double s = 0.0;
            const int gc = kTile * I + c;
            for (int row = kTile * (I + 1) + g; row < m; row += 8)
                s += A[static_cast<int64_t>(row) * ld + gc] * yb[row];
            red[g * kTile + c] = s;
            __syncthreads();
            if (tid < kTile) {
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < 8; ++q) acc += red[q * kTile + tid];
                double v = gc < m ? yb[gc] - acc : 0.0;
                for (int cc = kTile - 1; cc >= 0; --cc) {
                    const int gcc = kTile * I + cc;
                    const double Lcc = gcc < m ? A[static_cast<int64_t>(gcc) * ld + gcc] : 1.0;
                    const double xc = __shfl(v, cc, kWave) / Lcc;
                    if (tid == cc) v = xc;
                    else if (tid < cc && gcc < m && gc < m) v -= A[static_cast<int64_t>(gcc) * ld + gc] * xc;
                }
                if (gc < m) yb[gc] = v;
            }
            __syncthreads();
        }
    }
    // scatter beta = x / sqrt(n) to the caller's small / large order; NaN block on failure
    bool mono = false;
    for (int i = tid; i < m; i += 256) mono |= !(rsd[row0 + i] < INFINITY);
    const double nanv = __builtin_nan("");
    for (int i = tid; i < m; i += 256) {
        const double v = fail == 0 ? yb[i] * inv_sqrt_n : nanv;
        const int o = slot_out[row0 + i];
        if (o >= 0) beta_s[o] = v;
        else beta_l[-1 - o] = v;
    }
    if (fail != 0 || mono) atomicMax(status + blk_id[b], mono ? 3 : 2);
}

// ------------------------------------------------------------------------------------------
// readSNPIm + nomalizeVec for a list of rows in ORIGINAL individual order (diagnostics and
// parity): out[j * n_ref + i] = (g_ij - mu_j) * rsd_j with missing calls at the mean (0).
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void dbslmm_std_columns(
    const uint8_t* __restrict__ bed, int32_t n_ref, int64_t bytes_per_snp,
    const int32_t* __restrict__ pos, int32_t n_rows,
    const double* __restrict__ mu, const double* __restrict__ rsd, double* __restrict__ out) {
    const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (idx >= static_cast<int64_t>(n_rows) * n_ref) return;
    const int jrow = static_cast<int>(idx / n_ref);
    const int i = static_cast<int>(idx % n_ref);
    const uint8_t byte = bed[3 + static_cast<int64_t>(pos[jrow]) * bytes_per_snp + (i >> 2)];
    const int code = (byte >> (2 * (i & 3))) & 3;
    const double g = code == 0 ? 2.0 : code == 2 ? 1.0 : code == 3 ? 0.0 : mu[jrow];
    out[idx] = (g - mu[jrow]) * rsd[jrow];
}
