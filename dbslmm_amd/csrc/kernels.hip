// kernels.hip -- gfx950 (CDNA4) kernels of the per-LD-block effect-size solver.
//
// The front of the hot path of DBSLMMFIT::est (reference scr/dbslmmfit.cpp:56-363):
//
//   dbslmm_unpack_stats  IO::readSNPIm + nomalizeVec statistics (scr/dtpr.cpp:285-380):
//                        2-bit PLINK rows -> the 2-bit DOSAGE operand Gp (codes 0/1/2, 3 =
//                        missing, padding individuals 0; kpad / 16 dwords per slot, slots in
//                        block order) plus exact integer per-SNP count / sum / sum-of-squares
//                        (popcounts) and the fp64 mean and 1/sd (N-1).  HBM-bound, one wave per
//                        slot.
//   dbslmm_gram_i8 /     estBlock's LD matrices (scr/dbslmmfit.cpp:697-709, 751-756) as ONE
//   dbslmm_gram_big /    joint Gram per block over [small | large] SNPs on the FP4 matrix cores
//   dbslmm_gram_huge     (v_mfma_scale_f32_32x32x64_f8f6f4, exact integer sums in fp32; each Gp
//                        dword is expanded to FP4 operands in registers -- fp4_chunk below; the
//                        _i8 kernel keeps its round-2 name) with an fp64 epilogue that
//                        centres, standardises and applies tau:
//                          Sigma_ij = tau/n_ref * C_ij /(s_i s_j) + (1-tau) delta_ij,
//                          C_ij = G_ij - S_i S_j / n   (no missing calls in the block)
//                        Blocks with missing calls add the observed-mask Grams (4 MFMAs/step).
//                        32 x 32 tiles per wave (m < 96), 128 x 128 per workgroup, 256 x 256 per
//                        workgroup (the big blocks).
//
// The solve of the joint matrix M = [[Sigma_ss + I/(sigma_s n), Sigma_sl], [Sigma_ls, Sigma_ll]],
// beta = M^{-1} [z_s; z_l] / sqrt(n) (PCGm/PCGv at :713-729, :758-764) is
// in chol.hip (dbslmm_chol_small / _large), chol_tiled.hip (dbslmm_tchol_*) and trsv.hip.
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

// The Gram operand Gp: per slot, kpad / 16 dwords of 2-bit DOSAGE codes (0, 1, 2; 3 = missing;
// padding individuals 0), re-coded from the PLINK codes of one .bed dword (individual j in bits
// 2j..2j+1; 00 -> 2, 10 -> 1, 11 -> 0, 01 -> missing: d0 = lo ^ hi, d1 = ~hi).  A quarter of the
// bytes of an int8 operand; the Gram kernels expand it to FP4 on the fly (fp4_chunk).
__device__ __forceinline__ uint32_t dose_code16(uint32_t w, uint32_t valid_mask_2bit) {
    const uint32_t lo = w & 0x55555555u, hi = (w >> 1) & 0x55555555u;
    const uint32_t d0 = (lo ^ hi) & valid_mask_2bit, d1 = ~hi & valid_mask_2bit;
    return d0 | (d1 << 1);
}
// The Gram kernels multiply on the FP4 matrix cores: dosages 0 / 1 / 2 (and the 0 / 1 masks of
// the missing-call form) are exact e2m1 values, every product is exact and every partial sum an
// integer below 4 n_ref < 2^24, so v_mfma_scale_f32_32x32x64_f8f6f4 gives the integer Gram bit for
// bit -- at twice the MACs per clock of v_mfma_i32_32x32x32_i8, with half its operand bytes.  A Gp
// dword (16 two-bit codes c) becomes two FP4 dwords with one mask each and one shift per PAIR of
// dwords: w & 0x33333333 leaves the even-numbered codes in bits 0-1 of the nibbles, which as e2m1
// read 0.5 c (0.0 / 0.5 / 1.0); (w >> 2) & 0x33333333 the odd ones (one 64-bit shift serves both
// dwords of a pair -- the bits shifted in from the high dword are masked off).  The E8M0 block
// scales 2^1 on both operands restore c_a c_b exactly.  (A fixed permutation of the individuals,
// the same on both operands, so every product sums each individual once.)
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
constexpr int kE8M0Two = static_cast<int>(0x80808080u);   // E8M0 scale 2^1 in every byte
constexpr uint32_t kFp4Mask = 0x33333333u;
// 16 B of FP4 operand (32 individuals) from Gp dwords w0, w1
__device__ __forceinline__ v4i fp4_chunk(uint32_t w0, uint32_t w1) {
    const uint64_t t = ((static_cast<uint64_t>(w1) << 32) | w0) >> 2;
    return v4i{static_cast<int>(w0 & kFp4Mask), static_cast<int>(static_cast<uint32_t>(t) & kFp4Mask),
               static_cast<int>(w1 & kFp4Mask), static_cast<int>(static_cast<uint32_t>(t >> 32) & kFp4Mask)};
}
// C += A B^T over 64 individuals (32 per lane half), 32 x 32 tile
__device__ __forceinline__ v16f mfma_fp4(v4i a, v4i b, v16f c) {
    const v8i a8{a[0], a[1], a[2], a[3], 0, 0, 0, 0}, b8{b[0], b[1], b[2], b[3], 0, 0, 0, 0};
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, kE8M0Two, 0, kE8M0Two);
}
// centred Gram entry C_ij = G_ij - S_i S_j / n, as G - (S_i S_j) (1 / n) in one fma: S_i S_j is
// an exact integer (below 2^53), the product with the rounded reciprocal replaces an fp64 divide
// per element (relative deviation from the divided form ~1e-16 of S_i S_j / n)
__device__ __forceinline__ double centre(float g, double sisj, double rn) {
    return __builtin_fma(-sisj, rn, static_cast<double>(g));
}
// missing-call form of a Gp dword (code 3 = missing): g = the dosages with missing calls as 0,
// o = 1 for observed calls (padding individuals count as observed: pad_k in the epilogue)
__device__ __forceinline__ void split_missing(uint32_t x, uint32_t& g, uint32_t& o) {
    const uint32_t m2 = x & (x >> 1) & 0x55555555u;
    g = x & ~(3u * m2);
    o = m2 ^ 0x55555555u;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Kernel 1: unpack + per-SNP statistics.  One wave per slot (SNP row of a block), 4 waves/WG.
//   Gp (optional)  [n_slots][kpad / 16] dosage-code dwords (dose_code16); padding slots (pos < 0)
//                  and padding individuals are dosage 0.
//   stat_*         exact integer statistics over the n_ref individuals.
//   mu, rsd, S     fp64: mean over observed calls (= the imputation value, dtpr.cpp:358),
//                  1/sd with the N-1 divisor (nomalizeVec), sum of observed dosages.
//   block_flags    bit 0 set when a slot of the block has a missing call.
//   slot_list      optional: unpack only these n_slots slots (the plan unpacks its lead group first)
// A row starts at any byte (3 + pos * bytes_per_snp): lane q of a pass handles the row's 16-B
// chunk q (64 individuals) from the two aligned 16-B loads covering it (the second only when the
// row is not 16-B aligned), so a wave issues whole-dwordx4 loads for its row up front, kU chunks
// per lane, and writes dwordx4 stores.  The image is followed by kBedPad (64) allocated bytes, so
// the last row's loads stay inside the allocation; bytes past n_ref are masked.
// ------------------------------------------------------------------------------------------
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4v load_u4(const uint8_t* p) { return *reinterpret_cast<const u4v*>(p); }
// 16 bytes at byte offset 4 d + bs (d, bs wave-uniform) of the 32-byte pair (x | y)
__device__ __forceinline__ u4v shift_pair(u4v x, u4v y, int d, int bs) {
    uint32_t w[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
    uint32_t o[5];
    switch (d) {   // (wave-uniform: a scalar branch, register moves only)
        case 0: o[0] = w[0]; o[1] = w[1]; o[2] = w[2]; o[3] = w[3]; o[4] = w[4]; break;
        case 1: o[0] = w[1]; o[1] = w[2]; o[2] = w[3]; o[3] = w[4]; o[4] = w[5]; break;
        case 2: o[0] = w[2]; o[1] = w[3]; o[2] = w[4]; o[3] = w[5]; o[4] = w[6]; break;
        default: o[0] = w[3]; o[1] = w[4]; o[2] = w[5]; o[3] = w[6]; o[4] = w[7]; break;
    }
    u4v r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = __builtin_amdgcn_alignbyte(o[j + 1], o[j], static_cast<uint32_t>(bs));
    return r;
}

extern "C" __global__ __launch_bounds__(256) void dbslmm_unpack_stats(
    const uint8_t* __restrict__ bed, int32_t n_ref, int64_t bytes_per_snp,
    const int32_t* __restrict__ slot_pos, const int32_t* __restrict__ slot_block, int32_t n_slots,
    uint32_t* __restrict__ Gp, int64_t kpad,
    double* __restrict__ S_out, double* __restrict__ mu_out, double* __restrict__ rsd_out,
    int32_t* __restrict__ block_flags, const int32_t* __restrict__ slot_list) {
    constexpr int kU = 4;                       // chunks per lane per pass (loads in flight)
    const int lane = threadIdx.x & (kWave - 1);
    const int k = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (k >= n_slots) return;
    const int slot = slot_list ? slot_list[k] : k;   // a subset of the slots (n_slots of them)
    const int32_t pos = slot_pos ? slot_pos[slot] : slot;   // (null: slot k reads bed row k)
    const int64_t n_words = kpad / 16;          // 16 individuals per dword (kpad: a multiple of 64)
    const int nq = static_cast<int>(n_words / 4);           // 16-B chunks of the Gp row
    u4v* grow = Gp ? reinterpret_cast<u4v*>(Gp + static_cast<int64_t>(slot) * n_words) : nullptr;
    if (pos < 0) {                              // padding slot
        if (grow)
            for (int q = lane; q < nq; q += kWave) grow[q] = u4v{0u, 0u, 0u, 0u};
        if (lane == 0) {
            if (S_out) S_out[slot] = 0.0;
            if (mu_out) mu_out[slot] = 0.0;
            if (rsd_out) rsd_out[slot] = 0.0;
        }
        return;
    }
    const int64_t row_off = 3 + static_cast<int64_t>(pos) * bytes_per_snp;
    const uint8_t* base = bed + (row_off & ~int64_t(15));
    const int sh = static_cast<int>(row_off & 15), dsh = sh >> 2, bsh = sh & 3;
    const int nqd = (n_ref + 63) / 64;          // chunks holding individuals
    int cnt = 0, sum = 0, sq = 0, nmiss = 0;
    for (int q0 = 0; q0 < nq; q0 += kWave * kU) {
        u4v lo[kU], hi[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int q = q0 + kWave * u + lane;
            lo[u] = hi[u] = u4v{0u, 0u, 0u, 0u};
            if (q < nqd) {
                lo[u] = load_u4(base + 16 * static_cast<int64_t>(q));
                if (sh) hi[u] = load_u4(base + 16 * static_cast<int64_t>(q) + 16);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int q = q0 + kWave * u + lane;
            if (q >= nq) break;
            const u4v wv = sh ? shift_pair(lo[u], hi[u], dsh, bsh) : lo[u];
            u4v g;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int first = 64 * q + 16 * j;
                const int nv = min(16, max(0, n_ref - first));
                const uint32_t vmask = nv >= 16 ? 0x55555555u : ((1u << (2 * nv)) - 1u) & 0x55555555u;
                const uint32_t word = wv[j];
                const uint32_t lo2 = word & vmask;
                const uint32_t hi2 = (word >> 1) & vmask;
                const int n_miss = __builtin_popcount(lo2 & ~hi2);
                const int n_two = __builtin_popcount(~lo2 & ~hi2 & vmask);
                const int n_one = __builtin_popcount(~lo2 & hi2);
                nmiss += n_miss;
                cnt += __builtin_popcount(vmask) - n_miss;
                sum += 2 * n_two + n_one;
                sq += 4 * n_two + n_one;
                g[j] = dose_code16(word, vmask);
            }
            if (grow) grow[q] = g;
        }
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
        if (nmiss > 0 && block_flags) atomicOr(block_flags + (slot_block ? slot_block[slot] : slot), 1);
    }
}

// ------------------------------------------------------------------------------------------
// MAF of IO::readSNPIm as the reference rounds it (dtpr.cpp:356-362): missing calls take the
// mean of the observed calls (mu, exact S / count from dbslmm_unpack_stats), sum(geno) runs in
// Armadillo's arrayops::accumulate order -- two sequential accumulators over the even / odd
// individuals -- and af = 0.5 * sum / n.  Once a (non-integer) mean has been added, each later add
// rounds, so the order decides the last bits, and the MAF filter of matchRef (|maf_ref - maf| <
// mafMax, strict) can flip on them.  One thread per row: a sequential chain of n_ref fp64 adds,
// rounded exactly like the host's (no reassociation).
// ------------------------------------------------------------------------------------------
// Rows without a missing call (miss[k] == 0; miss / S from dbslmm_unpack_stats, optional) hold
// only integer dosages: every partial sum of that order is an exact integer, so a1 + a2 equals
// the exact observed sum S and the chain is skipped (bit-identical).
extern "C" __global__ __launch_bounds__(256) void dbslmm_maf_arma(
    const uint8_t* __restrict__ bed, int32_t n_ref, int64_t bytes_per_snp,
    const int32_t* __restrict__ pos, int32_t n_rows, const double* __restrict__ mu,
    double* __restrict__ maf_out, const double* __restrict__ S, const int32_t* __restrict__ miss) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_rows) return;
    if (miss && S && miss[k] == 0) {
        const double af = 0.5 * S[k] / static_cast<double>(n_ref);
        maf_out[k] = (1.0 - af) < af ? 1.0 - af : af;
        return;
    }
    const int64_t row_off = 3 + static_cast<int64_t>(pos ? pos[k] : k) * bytes_per_snp;
    const double m = mu[k];
    double a1 = 0.0, a2 = 0.0;
    for (int32_t i0 = 0; i0 < n_ref; i0 += 16) {
        const uint32_t word = load_u32_any(bed, row_off + i0 / 4);
        const int nv = min(16, n_ref - i0);
        for (int j = 0; j < nv; j += 2) {          // i0 is even: j even = even individual
            const uint32_t c0 = (word >> (2 * j)) & 3u;
            // PLINK 2-bit code (low bit first): 00 -> 2, 10 -> 1, 11 -> 0, 01 -> missing (mean)
            a1 += c0 == 0u ? 2.0 : c0 == 2u ? 1.0 : c0 == 3u ? 0.0 : m;
            if (j + 1 < nv) {
                const uint32_t c1 = (word >> (2 * j + 2)) & 3u;
                a2 += c1 == 0u ? 2.0 : c1 == 2u ? 1.0 : c1 == 3u ? 0.0 : m;
            }
        }
    }
    const double af = 0.5 * (a1 + a2) / static_cast<double>(n_ref);
    maf_out[k] = (1.0 - af) < af ? 1.0 - af : af;   // std::min(af, 1.0 - af)
}

// ------------------------------------------------------------------------------------------
// Kernel 2: grouped joint Gram on FP4 MFMA.  One wave = one 32x32 output tile (block, ti, tj),
// ti >= tj, K loop over the padded individuals 128 at a time (gram_tile32 below: each lane
// loads 4 Gp dwords of its row per operand and feeds two FP4 MFMAs; identical k-permutation on
// the A and B side, so any lane->k assignment the instruction uses is summed consistently).
// Output: row-major lower triangle of the block's joint matrix
//     Sigma (no d shift; the Cholesky kernel adds 1/(sigma_s n) on the small diagonal).
// ------------------------------------------------------------------------------------------
struct GramTile { int32_t block, ti, tj, pad; };

// Factorisation copies an epilogue writes (h2f tuning): copies [0, ncopy) of every block, except
// that with tcopy >= 0 a tiled block (m >= tmin) gets copy tcopy only -- the other h2f solves of
// the tiled blocks iterate on that one factor (trsv.hip) and need no matrix of their own.
__device__ __forceinline__ int copy_lo(int m, int32_t tmin, int32_t tcopy) {
    return tcopy >= 0 && m >= tmin ? tcopy : 0;
}
__device__ __forceinline__ int copy_hi(int m, int32_t tmin, int32_t tcopy, int32_t ncopy) {
    return tcopy >= 0 && m >= tmin ? tcopy + 1 : ncopy;
}

// One 32 x 32 output tile (rows r0.., cols c0.. of block-local slots) on one wave, K over all
// kpad individuals with operands straight from Gp (L2), FP4 MFMAs.  Per 128 individuals (8 Gp
// dwords) lane (row, h = lane >> 5) loads dwords 4 h .. 4 h + 3 of its row and feeds dwords
// 4 h + 2 s, 4 h + 2 s + 1 to MFMA s: both operands use the same individual -> k map, so every
// product sums each individual once.  missing: the four products GG, GO, OG, OO of the
// observed-call expansion.
__device__ __forceinline__ void gram_tile32(
    const uint32_t* __restrict__ Gp, int64_t kpad, int row0, int m, int ld, int64_t moff, bool missing,
    int r0, int c0, int lane, const double* __restrict__ S, const double* __restrict__ mu,
    const double* __restrict__ rsd, double n_ref_d, double pad_k, double tau, double* __restrict__ M,
    int32_t ncopy, int64_t cstride, int32_t tmin, int32_t tcopy, uint16_t* __restrict__ G16,
    int64_t g16off, int64_t g16ld) {
    const int64_t kw = kpad / 16;                 // Gp dwords per slot (kpad: a multiple of 256)
    const uint32_t* pa = Gp + static_cast<int64_t>(row0 + r0 + (lane & 31)) * kw + 4 * (lane >> 5);
    const uint32_t* pb = Gp + static_cast<int64_t>(row0 + c0 + (lane & 31)) * kw + 4 * (lane >> 5);

    v16f acc = {0.0f};
    v16f acc_go = {0.0f}, acc_og = {0.0f}, acc_oo = {0.0f};
    if (!missing) {
        for (int64_t w = 0; w < kw; w += 8) {
            const v4i wa = *reinterpret_cast<const v4i*>(pa + w);
            const v4i wb = *reinterpret_cast<const v4i*>(pb + w);
#pragma unroll
            for (int q = 0; q < 2; ++q)
                acc = mfma_fp4(fp4_chunk(static_cast<uint32_t>(wa[2 * q]), static_cast<uint32_t>(wa[2 * q + 1])),
                               fp4_chunk(static_cast<uint32_t>(wb[2 * q]), static_cast<uint32_t>(wb[2 * q + 1])), acc);
        }
    } else {
        for (int64_t w = 0; w < kw; w += 8) {
          const v4i wa = *reinterpret_cast<const v4i*>(pa + w);
          const v4i wb = *reinterpret_cast<const v4i*>(pb + w);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            uint32_t ga0, oa0, ga1, oa1, gb0, ob0, gb1, ob1;
            split_missing(static_cast<uint32_t>(wa[2 * q]), ga0, oa0);
            split_missing(static_cast<uint32_t>(wa[2 * q + 1]), ga1, oa1);
            split_missing(static_cast<uint32_t>(wb[2 * q]), gb0, ob0);
            split_missing(static_cast<uint32_t>(wb[2 * q + 1]), gb1, ob1);
            const v4i ga = fp4_chunk(ga0, ga1), oa = fp4_chunk(oa0, oa1);
            const v4i gb = fp4_chunk(gb0, gb1), ob = fp4_chunk(ob0, ob1);
            acc = mfma_fp4(ga, gb, acc);
            acc_go = mfma_fp4(ga, ob, acc_go);
            acc_og = mfma_fp4(oa, gb, acc_og);
            acc_oo = mfma_fp4(oa, ob, acc_oo);
          }
        }
    }

    // fp64 epilogue.  C/D map of the 32x32 MFMA: col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5)
    const int j = lane & 31;
    const int lj = c0 + j;
    if (G16 && !missing) {   // PCG route: the exact integer Gram (pcg.hip forms Sigma around it)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int li = r0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            if (li < m && lj < m) G16[g16off + li * g16ld + lj] = static_cast<uint16_t>(acc[r]);
        }
        return;
    }
    const int sj = row0 + lj;
    const double Sj = lj < m ? S[sj] : 0.0;
    const double muj = lj < m ? mu[sj] : 0.0;
    const double rj = lj < m ? rsd[sj] : 0.0;
    const double scale = tau / n_ref_d, rn = 1.0 / n_ref_d;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int li = r0 + i;
        if (li >= m || lj >= m) continue;
        const int si = row0 + li;
        double c;
        if (!missing) {
            c = centre(acc[r], S[si] * Sj, rn);
        } else {
            const double mui = mu[si];
            c = static_cast<double>(acc[r]) - muj * static_cast<double>(acc_go[r]) -
                mui * static_cast<double>(acc_og[r]) +
                mui * muj * (static_cast<double>(acc_oo[r]) - pad_k);   // padding counts as observed
        }
        double v = scale * (c * rsd[si] * rj);
        if (li == lj) v += 1.0 - tau;
        const int c_lo = copy_lo(m, tmin, tcopy), c_hi = copy_hi(m, tmin, tcopy, ncopy);
        for (int cp = c_lo; cp < c_hi; ++cp) M[moff + cp * cstride + static_cast<int64_t>(li) * ld + lj] = v;
    }
}

extern "C" __global__ __launch_bounds__(256) void dbslmm_gram_i8(
    const uint32_t* __restrict__ Gp, int64_t kpad,
    const GramTile* __restrict__ tiles, int32_t n_tiles,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ld, const int64_t* __restrict__ blk_matoff,
    const int32_t* __restrict__ block_flags,
    const double* __restrict__ S, const double* __restrict__ mu, const double* __restrict__ rsd,
    double n_ref_d, double pad_k, double tau, double* __restrict__ M,
    int32_t ncopy, int64_t cstride, int32_t tmin, int32_t tcopy, uint16_t* __restrict__ G16,
    const int64_t* __restrict__ g16off, const int32_t* __restrict__ g16ld) {
    const int lane = threadIdx.x & (kWave - 1);
    const int t = blockIdx.x * (blockDim.x / kWave) + (threadIdx.x / kWave);
    if (t >= n_tiles) return;
    const GramTile tile = tiles[t];
    const int b = tile.block;
    gram_tile32(Gp, kpad, blk_row0[b], blk_m[b], blk_ld[b], blk_matoff[b], (block_flags[b] & 1) != 0,
                kTile * tile.ti, kTile * tile.tj, lane, S, mu, rsd, n_ref_d, pad_k, tau, M, ncopy, cstride,
                tmin, tcopy, G16, G16 ? g16off[b] : 0, G16 ? g16ld[b] : 0);
}

// ------------------------------------------------------------------------------------------
// Kernel 2b: the same Gram for blocks without missing calls, 128 x 128 output tile per
// 256-thread workgroup (wave w: 64 x 64 quadrant (w >> 1, w & 1) = 2 x 2 FP4 MFMA 32x32x64).
// K runs in stages of 256 individuals through double-buffered LDS: 128 B of FP4 codes per row,
// row stride 144 B (the 16 rows of a ds_read_b128 lane group land on 16 distinct 16-B bank
// groups); global loads run two stages ahead (two register sets, loop unrolled by two) of the
// current stage's 16 MFMAs per wave.  Diagonal tiles stage one operand and skip the
// strictly-upper quadrant.  Tiles come in per-XCD queues (entry e runs on XCD e % 8) so a block's
// rows stay in one L2; entries with block < 0 are padding.  Blocks with a missing call (flag set
// by the unpack) take the exact 4-product 32 x 32 path.
// ------------------------------------------------------------------------------------------
namespace gram {
constexpr int kGT = 128;                  // output tile edge
constexpr int kKS = 256;                  // individuals per K stage
constexpr int kRS = kKS / 2 + 16;         // LDS row stride (bytes): 128 B of FP4 codes + pad
constexpr int kOpBytes = kGT * kRS;       // one operand stage
constexpr int kLdsBytes = 2 * 2 * kOpBytes;   // 2 stages x (A, B) = 73,728 B
}  // namespace gram

extern "C" __global__ __launch_bounds__(256) void dbslmm_gram_big(
    const uint32_t* __restrict__ Gp, int64_t kpad,
    const GramTile* __restrict__ tiles, int32_t n_tiles,
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,
    const int32_t* __restrict__ blk_ld, const int64_t* __restrict__ blk_matoff,
    const int32_t* __restrict__ block_flags,
    const double* __restrict__ S, const double* __restrict__ mu, const double* __restrict__ rsd,
    double n_ref_d, double pad_k, double tau, double* __restrict__ M,
    int32_t ncopy, int64_t cstride, int32_t tmin, int32_t tcopy, uint16_t* __restrict__ G16,
    const int64_t* __restrict__ g16off, const int32_t* __restrict__ g16ld) {
    using namespace gram;
    extern __shared__ __attribute__((aligned(16))) int8_t glds[];
    if (static_cast<int>(blockIdx.x) >= n_tiles) return;
    const GramTile tile = tiles[blockIdx.x];
    const int b = tile.block;
    if (b < 0) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int row0 = blk_row0[b], m = blk_m[b], ld = blk_ld[b];
    const int64_t moff = blk_matoff[b];
    const bool diag = tile.ti == tile.tj;
    if (block_flags[b] & 1) {   // missing calls: 4-product form, 4 x 4 sub-tiles of 32, 4 per wave
        for (int q = wave; q < 16; q += 4) {
            const int si = q >> 2, sj = q & 3;
            if (diag && sj > si) continue;
            const int r0 = kGT * tile.ti + 32 * si, c0 = kGT * tile.tj + 32 * sj;
            if (r0 >= m || c0 >= m) continue;
            gram_tile32(Gp, kpad, row0, m, ld, moff, true, r0, c0, lane, S, mu, rsd, n_ref_d, pad_k,
                        tau, M, ncopy, cstride, tmin, tcopy, nullptr, 0, 0);
        }
        return;
    }
    const int64_t kw = kpad / 16;
    const uint32_t* ga = Gp + static_cast<int64_t>(row0 + kGT * tile.ti) * kw;
    const uint32_t* gb = Gp + static_cast<int64_t>(row0 + kGT * tile.tj) * kw;
    // staging map: 128 rows x 16 Gp dwords (16 individuals each) per operand and stage; thread t
    // moves dword pairs e = t + 256 q (row e >> 3, pair e & 7) and expands each pair to one 16-B
    // FP4 chunk on the way into LDS.  Two register sets: the global loads of stage s + 2 are
    // issued before stage s's MFMAs.
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    u2 ra0[4], rb0[4], ra1[4], rb1[4];
    auto gload = [&](u2 (&ra)[4], u2 (&rb)[4], int st) {
        const int64_t w0 = static_cast<int64_t>(st) * (kKS / 16);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = q * 256 + tid, r = e >> 3, c = e & 7;
            ra[q] = *reinterpret_cast<const u2*>(ga + static_cast<int64_t>(r) * kw + w0 + 2 * c);
            if (!diag) rb[q] = *reinterpret_cast<const u2*>(gb + static_cast<int64_t>(r) * kw + w0 + 2 * c);
        }
    };
    auto lstore = [&](const u2 (&ra)[4], const u2 (&rb)[4], int buf) {
        int8_t* A = glds + buf * 2 * kOpBytes;
        int8_t* B = A + kOpBytes;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = q * 256 + tid, r = e >> 3, c = e & 7;
            *reinterpret_cast<v4i*>(A + r * kRS + 16 * c) = fp4_chunk(ra[q][0], ra[q][1]);
            if (!diag) *reinterpret_cast<v4i*>(B + r * kRS + 16 * c) = fp4_chunk(rb[q][0], rb[q][1]);
        }
    };
    const int wr = wave >> 1, wc = wave & 1;
    const bool idle = diag && wc > wr;            // strictly-upper quadrant of a diagonal tile
    v16f acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = v16f{0.0f};
    // operand read offsets: lane l -> row (l & 31) of a 32-row group, the 16-B half (l >> 5) of a
    // 32-byte (64-individual) k-step
    const int rsub = lane & 31, ksub = 16 * (lane >> 5);
    auto compute = [&](int buf) {
        if (idle) return;
        const int8_t* A = glds + buf * 2 * kOpBytes;
        const int8_t* B = diag ? A : A + kOpBytes;
        const int8_t* pa = A + (64 * wr + rsub) * kRS + ksub;
        const int8_t* pb = B + (64 * wc + rsub) * kRS + ksub;
#pragma unroll
        for (int kk = 0; kk < kKS / 2; kk += 32) {
            const v4i a0 = *reinterpret_cast<const v4i*>(pa + kk);
            const v4i a1 = *reinterpret_cast<const v4i*>(pa + 32 * kRS + kk);
            const v4i b0 = *reinterpret_cast<const v4i*>(pb + kk);
            const v4i b1 = *reinterpret_cast<const v4i*>(pb + 32 * kRS + kk);
            acc[0][0] = mfma_fp4(a0, b0, acc[0][0]);
            acc[0][1] = mfma_fp4(a0, b1, acc[0][1]);
            acc[1][0] = mfma_fp4(a1, b0, acc[1][0]);
            acc[1][1] = mfma_fp4(a1, b1, acc[1][1]);
        }
    };
    const int nst = static_cast<int>(kpad / kKS);
    gload(ra0, rb0, 0);
    lstore(ra0, rb0, 0);
    if (nst > 1) gload(ra1, rb1, 1);
    __syncthreads();
    for (int st = 0; st < nst; st += 2) {
        // stage st from LDS buffer 0; ra1 holds st + 1, ra0 receives st + 2
        if (st + 2 < nst) gload(ra0, rb0, st + 2);
        compute(0);
        if (st + 1 < nst) lstore(ra1, rb1, 1);
        __syncthreads();
        if (st + 1 >= nst) break;
        // stage st + 1 from LDS buffer 1; ra0 holds st + 2, ra1 receives st + 3
        if (st + 3 < nst) gload(ra1, rb1, st + 3);
        compute(1);
        if (st + 2 < nst) lstore(ra0, rb0, 0);
        __syncthreads();
    }
    if (idle) return;
    if (G16) {   // PCG route: the exact integer Gram
        const int64_t go = g16off[b], gl = g16ld[b];
#pragma unroll
        for (int sj = 0; sj < 2; ++sj) {
            const int lj = kGT * tile.tj + 64 * wc + 32 * sj + (lane & 31);
#pragma unroll
            for (int si = 0; si < 2; ++si)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int li = kGT * tile.ti + 64 * wr + 32 * si + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    if (li < m && lj < m)
                        G16[go + li * gl + lj] = static_cast<uint16_t>(acc[si][sj][r]);
                }
        }
        return;
    }
    // fp64 epilogue (as dbslmm_gram_i8, no-missing form): C/D col = lane & 31,
    // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    const double scale = tau / n_ref_d, rn = 1.0 / n_ref_d;
#pragma unroll
    for (int sj = 0; sj < 2; ++sj) {
        const int lj = kGT * tile.tj + 64 * wc + 32 * sj + (lane & 31);
        if (lj >= m) continue;
        const double Sj = S[row0 + lj], rj = rsd[row0 + lj];
#pragma unroll
        for (int si = 0; si < 2; ++si) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int li = kGT * tile.ti + 64 * wr + 32 * si + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (li >= m) continue;
                const double c = centre(acc[si][sj][r], S[row0 + li] * Sj, rn);
                double v = scale * (c * rsd[row0 + li] * rj);
                if (li == lj) v += 1.0 - tau;
                for (int cp = copy_lo(m, tmin, tcopy); cp < copy_hi(m, tmin, tcopy, ncopy); ++cp)
                    M[moff + cp * cstride + static_cast<int64_t>(li) * ld + lj] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 2c: the Gram of the big blocks (m >= 384), 256 x 256 output tile per 512-thread
// workgroup, on the FP4 matrix cores (fp4_chunk / mfma_fp4 above: exact integer Gram).  Every
// wave computes a 64 x 128 piece (2 x 4 MFMA tiles, 128 accumulator registers), pieces paired on
// the SIMDs by their active MFMA count.  K runs in stages of 256 individuals whose raw 2-bit
// codes reach LDS by LDS-DMA (gram_huge_dma_loop) and are expanded to FP4 after the operand reads.
// Diagonal tiles stage one operand; MFMA tiles strictly above the diagonal or wholly past m (edge
// tiles) are skipped.  Missing-call blocks: the exact 4-product path per 32 x 32 sub-tile.
// ------------------------------------------------------------------------------------------
namespace gram {
constexpr int kHT = 256;                   // output tile edge
constexpr int kHK = 256;                   // individuals per K stage (64 B of 2-bit codes per row)
constexpr int kHLdsBytes = 4 * 2 * kHT * (kHK / 4);   // 4 DMA slots x (A | B) x 16 KiB = 128 KiB
constexpr int kKpadAlign = kHK;            // kpad: a multiple of the stage
}  // namespace gram

// K loop of dbslmm_gram_huge fed by LDS-DMA.  A stage (256 individuals) of a tile row is its 64 B
// of raw 2-bit Gp codes; global_load_lds_dwordx4 moves them straight into LDS (no staging
// registers, no LDS store instructions), four slots (32 KiB each: A | B), three stages in flight.
// LDS image: row r of an operand at r * 64 B, its 16-B chunk q at position q ^ ((r >> 2) & 3) --
// the DMA writes lane-linear, so the swizzle goes through the source address -- which puts the
// 16 rows of every ds_read_b128 lane group on 16 distinct bank groups.  Consumer: lane (row,
// h = lane >> 5) reads chunk q = 2 j + h of its row (16 B = 64 codes) for k-steps 2 j and 2 j + 1
// and expands each half (Gp dwords 0-1, 2-3) to one 16-B FP4 operand (fp4_chunk); A and B use the
// same individual -> k map, so every product sums each individual once.  NOP = operands staged
// (1: a diagonal tile, B = A); kFull: every MFMA tile of the wave's piece is active.
template <int NOP, bool kFull>
__device__ __forceinline__ void gram_huge_dma_loop(const uint32_t* __restrict__ Gp, int64_t kw,
                                                   const int64_t (&rbase)[2], const int (&svl)[2], int nst,
                                                   int8_t* lds, int wave, int lane, int wr, int wc,
                                                   uint32_t act, v16f (&acc)[2][4]) {
    typedef __attribute__((address_space(1))) const void* gptr_g;
    typedef __attribute__((address_space(3))) void* lptr_g;
    constexpr int kRowB = 64;                        // raw bytes per row and stage
    constexpr int kOpB = gram::kHT * kRowB;          // 16 KiB per operand stage
    constexpr int kSlotB = 2 * kOpB;                 // A | B
    // DMA map: wave w moves rows 32 w .. 32 w + 31 of each staged operand, 16 rows per
    // instruction; lane L -> row + (L >> 2), LDS position L & 3 holding chunk (L & 3) ^ ((row >> 2) & 3)
    const int dr = lane >> 2, dp = lane & 3;
    const uint32_t* gsrc[NOP][2];
#pragma unroll
    for (int op = 0; op < NOP; ++op)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = 32 * wave + 16 * h + dr;
            const int q = dp ^ ((r >> 2) & 3);
            gsrc[op][h] = Gp + (rbase[op] + min(r, svl[op] - 1)) * kw + 4 * q;
        }
    auto issue = [&](int st) {
        int8_t* slot = lds + (st & 3) * kSlotB;
#pragma unroll
        for (int op = 0; op < NOP; ++op)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                __builtin_amdgcn_global_load_lds((gptr_g)(gsrc[op][h] + 16 * st),
                                                 (lptr_g)(slot + op * kOpB + (32 * wave + 16 * h) * kRowB), 16, 0, 0);
    };
    const int rsub = lane & 31, hh = lane >> 5;
    // operand read offsets within a slot (chunk 2 j + hh of the row; j adds 32 B before the swizzle)
    auto roff = [&](int r, int j) { return r * kRowB + 16 * ((2 * j + hh) ^ ((r >> 2) & 3)); };
    auto compute = [&](int st) {
        const int8_t* A = lds + (st & 3) * kSlotB;
        const int8_t* B = NOP == 1 ? A : A + kOpB;
        v4i ar[2][2], br[2][4];
        auto read = [&](int j) {
#pragma unroll
            for (int i = 0; i < 2; ++i) ar[j][i] = *reinterpret_cast<const v4i*>(A + roff(64 * wr + 32 * i + rsub, j));
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) br[j][jj] = *reinterpret_cast<const v4i*>(B + roff(128 * wc + 32 * jj + rsub, j));
        };
        v4i av[2], bv[4];
        auto expand = [&](int j, int e) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
                av[i] = fp4_chunk(static_cast<uint32_t>(ar[j][i][2 * e]), static_cast<uint32_t>(ar[j][i][2 * e + 1]));
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
                bv[jj] = fp4_chunk(static_cast<uint32_t>(br[j][jj][2 * e]), static_cast<uint32_t>(br[j][jj][2 * e + 1]));
        };
        auto mult = [&]() {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (kFull || (act & (1u << (4 * i + jj)))) acc[i][jj] = mfma_fp4(av[i], bv[jj], acc[i][jj]);
        };
        // k-steps 2 j + e: the reads of j = 1 are issued once k-step 0's operands are expanded, so
        // they land under k-steps 0 and 1's MFMAs (sched_barrier pins that order)
        read(0);
        __builtin_amdgcn_sched_barrier(0);
        expand(0, 0);
        __builtin_amdgcn_sched_barrier(0);
        read(1);
        __builtin_amdgcn_sched_barrier(0);
        mult();
        expand(0, 1);
        mult();
        __builtin_amdgcn_sched_barrier(0);
        expand(1, 0);
        mult();
        expand(1, 1);
        mult();
    };
    // vmcnt counts this wave's DMA instructions in issue order (2 NOP per stage)
    auto wait_stage = [&](int ahead) {   // ahead = stages issued after the one awaited
        if (ahead >= 2) {
            if constexpr (NOP == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else if (ahead == 1) {
            if constexpr (NOP == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };
    for (int st = 0; st < min(3, nst); ++st) issue(st);
    for (int st = 0; st < nst; ++st) {
        wait_stage(min(2, nst - 1 - st));
        __builtin_amdgcn_s_barrier();            // stage st is in LDS; slot (st + 3) & 3 is free
        if (st + 3 < nst) issue(st + 3);
        compute(st);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();                // every wave is done with the slots
}

#define GRAM_HUGE_PARAMS                                                                            \
    const uint32_t* __restrict__ Gp, int64_t kpad,                                                 \
    const GramTile* __restrict__ tiles, int32_t n_tiles,                                           \
    const int32_t* __restrict__ blk_row0, const int32_t* __restrict__ blk_m,                       \
    const int32_t* __restrict__ blk_ld, const int64_t* __restrict__ blk_matoff,                    \
    const int32_t* __restrict__ block_flags,                                                       \
    const double* __restrict__ S, const double* __restrict__ mu, const double* __restrict__ rsd,   \
    double n_ref_d, double pad_k, double tau, double* __restrict__ M,                              \
    int32_t ncopy, int64_t cstride, int32_t tmin, int32_t tcopy, uint16_t* __restrict__ G16,          \
    const int64_t* __restrict__ g16off, const int32_t* __restrict__ g16ld
#define GRAM_HUGE_ARGS Gp, kpad, tiles, n_tiles, blk_row0, blk_m, blk_ld, blk_matoff, block_flags, S, \
    mu, rsd, n_ref_d, pad_k, tau, M, ncopy, cstride, tmin, tcopy, G16, g16off, g16ld
__device__ __forceinline__ void gram_huge_body(GRAM_HUGE_PARAMS) {
    using namespace gram;
    extern __shared__ __attribute__((aligned(16))) int8_t hlds[];
    if (static_cast<int>(blockIdx.x) >= n_tiles) return;
    const GramTile tile = tiles[blockIdx.x];
    const int b = tile.block;
    if (b < 0) return;
    // (wave and the per-wave MFMA mask are wave-uniform: readfirstlane keeps their branches scalar)
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int row0 = blk_row0[b], m = blk_m[b], ld = blk_ld[b];
    const int64_t moff = blk_matoff[b];
    const bool diag = tile.ti == tile.tj;
    if (block_flags[b] & 1) {   // missing calls: 8 x 8 sub-tiles of 32, 4-product form
        for (int q = wave; q < 64; q += 8) {
            const int si = q >> 3, sj = q & 7;
            if (diag && sj > si) continue;
            const int r0 = kHT * tile.ti + 32 * si, c0 = kHT * tile.tj + 32 * sj;
            if (r0 >= m || c0 >= m) continue;
            gram_tile32(Gp, kpad, row0, m, ld, moff, true, r0, c0, lane, S, mu, rsd, n_ref_d, pad_k,
                        tau, M, ncopy, cstride, tmin, tcopy, nullptr, 0, 0);
        }
        return;
    }
    // ragged edge tiles: rows / columns of the tile inside the block (the last tile row / column
    // of a block is partly padding).  The DMA re-reads the last valid row for rows past them (an
    // L2 hit); the MFMAs that would only produce rows or columns past m are skipped, so an edge
    // tile costs about its valid area.
    const int rv = min(kHT, m - kHT * tile.ti), cv = min(kHT, m - kHT * tile.tj);
    const int64_t kw = kpad / 16;
    // wave -> piece (wr, wc): rows 64 wr .., columns 128 wc ...  act: bit 4 i + j = MFMA tile (i, j)
    // produces rows / columns < m and is not strictly above a diagonal tile's diagonal (32 x 32
    // granularity, as dbslmm_gram_i8).  The two waves of a SIMD (w, w + 4) share its matrix pipe,
    // so the pieces are paired by their active MFMA count, largest with smallest (waves 0-3 take
    // the pieces in descending count, waves 4-7 ascending): a diagonal tile's pieces (8, 8, 7, 7,
    // 3, 3, 0, 0 MFMA tiles) leave every SIMD <= 10 instead of up to 14 of 16.  The same for every
    // wave (uniform values), and an output element is still computed by one wave in one k order.
    auto piece_act = [&](int pr, int pc) {
        uint32_t a = 0;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ri = 64 * pr + 32 * i, cj = 128 * pc + 32 * j;
                if (ri < rv && cj < cv && !(diag && cj >= ri + 32)) a |= 1u << (4 * i + j);
            }
        return a;
    };
    int cnt[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) cnt[q] = __builtin_popcount(piece_act(q >> 1, q & 1));
    const int rank_want = wave < 4 ? wave : 11 - wave;
    int pc_sel = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        int rk = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) rk += (cnt[u] > cnt[q] || (cnt[u] == cnt[q] && u < q)) ? 1 : 0;
        if (rk == rank_want) pc_sel = q;
    }
    pc_sel = __builtin_amdgcn_readfirstlane(pc_sel);
    const int wr = pc_sel >> 1, wc = pc_sel & 1;
    uint32_t act = piece_act(wr, wc);
    act = __builtin_amdgcn_readfirstlane(act);
    const bool idle = act == 0;
    v16f acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = v16f{0.0f};
    {
        const int nst = static_cast<int>(kpad / kHK);
        const int64_t rbase[2] = {row0 + kHT * tile.ti, row0 + kHT * tile.tj};
        const int svl[2] = {rv, cv};
        if (diag) {
            if (act == 0xFFu) gram_huge_dma_loop<1, true>(Gp, kw, rbase, svl, nst, hlds, wave, lane, wr, wc, act, acc);
            else gram_huge_dma_loop<1, false>(Gp, kw, rbase, svl, nst, hlds, wave, lane, wr, wc, act, acc);
        } else {
            if (act == 0xFFu) gram_huge_dma_loop<2, true>(Gp, kw, rbase, svl, nst, hlds, wave, lane, wr, wc, act, acc);
            else gram_huge_dma_loop<2, false>(Gp, kw, rbase, svl, nst, hlds, wave, lane, wr, wc, act, acc);
        }
    }
    if (G16) {   // PCG route: the exact integer Gram
        if (idle) return;
        const int64_t go = g16off[b], gl = g16ld[b];
#pragma unroll
        for (int si = 0; si < 2; ++si)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int li = kHT * tile.ti + 64 * wr + 32 * si + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (li >= m) continue;
#pragma unroll
                for (int sj = 0; sj < 4; ++sj) {
                    const int lj = kHT * tile.tj + 128 * wc + 32 * sj + (lane & 31);
                    if (!(act & (1u << (4 * si + sj))) || lj >= m) continue;
                    G16[go + li * gl + lj] = static_cast<uint16_t>(acc[si][sj][r]);
                }
            }
        return;
    }
    // fp64 epilogue.  The per-row (S, rsd) and per-column values of the tile go through LDS (the
    // K loop's last barrier has passed: no wave reads the stages any more), so the element loop
    // issues no global loads; rows outer, the four column tiles inner.
    double* eRow = reinterpret_cast<double*>(hlds);   // [S | rsd] of the tile's 256 rows
    double* eCol = eRow + 2 * kHT;                     // [S | rsd] of its 256 columns
    {
        const int sop = tid >> 8, k = tid & 255, idx = kHT * (sop ? tile.tj : tile.ti) + k;
        double* e = sop ? eCol : eRow;
        e[k] = idx < m ? S[row0 + idx] : 0.0;
        e[kHT + k] = idx < m ? rsd[row0 + idx] : 0.0;
    }
    __syncthreads();
    if (idle) return;
    const double scale = tau / n_ref_d, rn = 1.0 / n_ref_d;
    double Sj[4], rj[4];
#pragma unroll
    for (int sj = 0; sj < 4; ++sj) {
        const int cl = 128 * wc + 32 * sj + (lane & 31);
        Sj[sj] = eCol[cl];
        rj[sj] = eCol[kHT + cl];
    }
#pragma unroll
    for (int si = 0; si < 2; ++si) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rl = 64 * wr + 32 * si + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int li = kHT * tile.ti + rl;
            if (li >= m) continue;
            const double Si = eRow[rl], ri = eRow[kHT + rl];
#pragma unroll
            for (int sj = 0; sj < 4; ++sj) {
                const int lj = kHT * tile.tj + 128 * wc + 32 * sj + (lane & 31);
                if (!(act & (1u << (4 * si + sj))) || lj >= m) continue;
                const double c = centre(acc[si][sj][r], Si * Sj[sj], rn);
                double v = scale * (c * ri * rj[sj]);
                if (li == lj) v += 1.0 - tau;
                for (int cp = copy_lo(m, tmin, tcopy); cp < copy_hi(m, tmin, tcopy, ncopy); ++cp)
                    M[moff + cp * cstride + static_cast<int64_t>(li) * ld + lj] = v;
            }
        }
    }
}

extern "C" __global__ __launch_bounds__(512) void dbslmm_gram_huge(GRAM_HUGE_PARAMS) {
    gram_huge_body(GRAM_HUGE_ARGS);
}

// ------------------------------------------------------------------------------------------
// `valid` (scr/validate.cpp:221-257): deno_b = z1^T (X^T X / n_ref) z1 = |X z1|^2 / n_ref per
// block, X the nomalizeVec-standardised reference genotypes (missing calls at the mean -> 0).
// Computed as a weighted row sum straight from the packed .bed (no Gram): thread = one packed
// dword column (16 individuals), looping over the block's SNPs; y = X z1 in fp64 registers; the
// workgroup reduces sum(y^2) into partial[b][blockIdx.x]; dbslmm_valid_reduce sums the
// partials of each block in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------
extern "C" __global__ __launch_bounds__(256) void dbslmm_valid_partial(
    const uint8_t* __restrict__ bed, int32_t n_ref, int64_t bytes_per_snp,
    const int64_t* __restrict__ ptr, const int32_t* __restrict__ pos,
    const double* __restrict__ z1, const double* __restrict__ mu, const double* __restrict__ rsd,
    double* __restrict__ partial, int32_t n_chunks) {
    __shared__ double red[256 / kWave];
    const int b = blockIdx.y;
    const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t n_words = (n_ref + 15) / 16;
    double y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = 0.0;
    if (w < n_words) {
        const int nv = static_cast<int>(min<int64_t>(16, n_ref - 16 * w));
        for (int64_t j = ptr[b]; j < ptr[b + 1]; ++j) {
            const uint32_t word = load_u32_any(bed, 3 + static_cast<int64_t>(pos[j]) * bytes_per_snp + 4 * w);
            const double m0 = mu[j], wt = z1[j] * rsd[j];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t code = (word >> (2 * i)) & 3u;
                // 00 -> 2, 10 -> 1, 11 -> 0, 01 -> missing (the mean: contributes 0)
                const double g = code == 0 ? 2.0 : (code == 2 ? 1.0 : (code == 3 ? 0.0 : m0));
                if (i < nv) y[i] += (g - m0) * wt;
            }
        }
    }
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += y[i] * y[i];
    for (int off = kWave / 2; off > 0; off >>= 1) s += __shfl_down(s, off, kWave);
    if ((threadIdx.x & (kWave - 1)) == 0) red[threadIdx.x / kWave] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < 256 / kWave; ++q) t += red[q];
        partial[static_cast<int64_t>(b) * n_chunks + blockIdx.x] = t;
    }
}

extern "C" __global__ void dbslmm_valid_reduce(const double* __restrict__ partial, int32_t n_chunks,
                                               int32_t num_block, double n_ref_d,
                                               double* __restrict__ deno) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= num_block) return;
    double t = 0.0;
    for (int c = 0; c < n_chunks; ++c) t += partial[static_cast<int64_t>(b) * n_chunks + c];
    deno[b] = t / n_ref_d;
}

// one device scalar, in stream order (the solve kernels read sigma's shift from it)
extern "C" __global__ void dbslmm_set_scalar(double* __restrict__ dst, double v) { *dst = v; }

// testing only (dbslmm_options.debug_delay_us): one wave that holds its stream for `ticks` of the
// 100 MHz real-time counter, so work queued behind it on that stream starts late and any
// dependency another stream is missing on it shows up deterministically
extern "C" __global__ void dbslmm_debug_spin(int64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (static_cast<int64_t>(__builtin_amdgcn_s_memrealtime() - t0) < ticks) __builtin_amdgcn_s_sleep(16);
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
