// variance.hip -- test-set variance diag (included by plan.hip).
//
// Reference: calcBlock (scr/dbslmmfit.cpp:366-539, 542-626) reads each block's SNPs from the
// test panel (readSNPIm over the indicator-1 individuals, nomalizeVec) and returns
// diag(X_l var_bl X_l^T + X_s var_bs X_s^T) from calc_nt_by_nt_matrix
// (scr/calc_asymptotic_variance.cpp:22-137):
//   A = Sigma_ss + I/(n sigma),  var_bl = (Sigma_ll - Sigma_ls A^-1 Sigma_sl)^-1 / n,
//   var_bs = n sigma^2 (Sigma_ss - Sigma_ss A^-1 Sigma_ss + n mat2 var_bl mat2^T),
//   mat2 = Sigma_sl - Sigma_ss A^-1 Sigma_sl.
// With the joint matrix M = [[A, Sigma_sl], [Sigma_ls, Sigma_ll]] = L L^T already factored by the
// solve (strict lower = L, diagonal = 1/L_ii in every solve path) and d = 1/(n sigma), this is
// per test individual t (verified to 1e-16 against the literal formulas, tests/test_variance.py):
//   y = L^-1 [x_s; 0],  q1 = |y_s|^2 (= x_s^T A^-1 x_s),  w2 = |y_l|^2,
//   y' = L^-1 [0; x_l], q3 = |y'|^2 (= x_l^T (M^-1)_ll x_l),
//   diag_t = q3 / n + n sigma^2 (d |x_s|^2 - d^2 (q1 - w2)).
// The forward substitutions run blocked over 32-row chunks: a rank update of the chunk from all
// earlier rows (4 waves, 8 rows each, 64 test individuals per workgroup) and a 32-row triangular
// solve inside the chunk (wave 0, one individual per lane).

// Compact the needed rows of the test .bed to the indicator-1 individuals: out row s (plan slot
// order) = test row tpos[s] restricted to sel[0..n_test) (-1: padding slot, left as zeros).
extern "C" __global__ __launch_bounds__(256) void dbslmm_test_compact(
    const uint8_t* __restrict__ tbed, int64_t tbps, const int32_t* __restrict__ tpos,
    int32_t n_slots, const int32_t* __restrict__ sel, int32_t n_test, int64_t cbps,
    uint8_t* __restrict__ out) {
    const int s = blockIdx.y;
    const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (s >= n_slots || q >= cbps) return;
    const int32_t row = tpos[s];
    uint32_t byte = 0;
    if (row >= 0) {
        const uint8_t* src = tbed + 3 + static_cast<int64_t>(row) * tbps;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t t = 4 * q + j;
            if (t < n_test) {
                const int idx = sel[t];
                byte |= ((static_cast<uint32_t>(src[idx >> 2]) >> (2 * (idx & 3))) & 3u) << (2 * j);
            }
        }
    }
    out[3 + static_cast<int64_t>(s) * cbps + q] = static_cast<uint8_t>(byte);
}

namespace var {
constexpr int kRhs = 64;      // test individuals per workgroup
constexpr int kChunk = 32;    // rows per substitution chunk

// standardised test genotype of slot s for individual t (missing -> the mean -> 0)
__device__ __forceinline__ double xval(const uint8_t* cbed, int64_t cbps, const double* mu,
                                       const double* rsd, int s, int t) {
    const uint32_t code = (static_cast<uint32_t>(cbed[3 + static_cast<int64_t>(s) * cbps + (t >> 2)]) >> (2 * (t & 3))) & 3u;
    if (code == 1u) return 0.0;
    const double g = code == 0 ? 2.0 : (code == 2 ? 1.0 : 0.0);
    return (g - mu[s]) * rsd[s];
}
}  // namespace var

extern "C" __global__ __launch_bounds__(256) void dbslmm_variance(
    const double* __restrict__ M, const int32_t* __restrict__ blk_row0,
    const int32_t* __restrict__ blk_m, const int32_t* __restrict__ blk_ms,
    const int32_t* __restrict__ blk_ld, const int64_t* __restrict__ blk_matoff,
    const int32_t* __restrict__ blk_id, const int32_t* __restrict__ status,
    const uint8_t* __restrict__ cbed, int64_t cbps, const double* __restrict__ mu,
    const double* __restrict__ rsd, int32_t n_test, double sigma_s, double n_obs,
    double* __restrict__ Y, int64_t nt_pad, double* __restrict__ diags) {
    using namespace var;
    __shared__ double acc[kChunk][kRhs];
    __shared__ double red[4][kRhs];
    const int b = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, g = tid >> 6;
    const int t = blockIdx.x * kRhs + lane;
    const bool act = t < n_test;
    const int row0 = blk_row0[b], m = blk_m[b], ms = blk_ms[b], ld = blk_ld[b];
    const double* A = M + blk_matoff[b];
    double* Yb = Y + static_cast<int64_t>(row0) * nt_pad + (t < n_test ? t : 0);
    double xs2 = 0.0, q1 = 0.0, w2 = 0.0, q3 = 0.0;
    // pass 1: y = L^-1 [x_s; 0]
    for (int i0 = 0; i0 < m; i0 += kChunk) {
        double a8[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int r = i0 + 8 * g + u;
            double x = 0.0;
            if (act && r < ms) {
                x = var::xval(cbed, cbps, mu, rsd, row0 + r, t);
                xs2 += x * x;
            }
            a8[u] = x;
        }
        for (int k = 0; k < i0; ++k) {
            const double yk = act ? Yb[static_cast<int64_t>(k) * nt_pad] : 0.0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int r = i0 + 8 * g + u;
                if (r < m) a8[u] -= A[static_cast<int64_t>(r) * ld + k] * yk;
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[8 * g + u][lane] = a8[u];
        __syncthreads();
        if (g == 0) {
            const int nr = min(kChunk, m - i0);
            double yc[kChunk];
#pragma unroll
            for (int j = 0; j < kChunk; ++j) {
                if (j < nr) {
                    const int r = i0 + j;
                    double a = acc[j][lane];
#pragma unroll
                    for (int k = 0; k < j; ++k) a -= A[static_cast<int64_t>(r) * ld + i0 + k] * yc[k];
                    const double y = a * A[static_cast<int64_t>(r) * ld + r];   // diagonal = 1/L_rr
                    yc[j] = y;
                    if (act) Yb[static_cast<int64_t>(r) * nt_pad] = y;
                    if (r < ms) q1 += y * y;
                    else w2 += y * y;
                }
            }
        }
        __syncthreads();
    }
    // pass 2 (blocks with large SNPs): y' = L^-1 [0; x_l], rows ms .. m-1 only (wave 0)
    if (g == 0 && m > ms) {
        for (int r = ms; r < m; ++r) {
            double a = act ? var::xval(cbed, cbps, mu, rsd, row0 + r, t) : 0.0;
            for (int k = ms; k < r; ++k) a -= A[static_cast<int64_t>(r) * ld + k] * (act ? Yb[static_cast<int64_t>(k) * nt_pad] : 0.0);
            const double y = a * A[static_cast<int64_t>(r) * ld + r];
            if (act) Yb[static_cast<int64_t>(r) * nt_pad] = y;
            q3 += y * y;
        }
    }
    red[g][lane] = xs2;
    __syncthreads();
    if (g == 0 && act) {
        const double xsum = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
        const double d = 1.0 / (n_obs * sigma_s);
        double v = q3 / n_obs + n_obs * sigma_s * sigma_s * (d * xsum - d * d * (q1 - w2));
        if (status[blk_id[b]] >= DBSLMM_BLOCK_NOT_PD) v = __builtin_nan("");
        diags[static_cast<int64_t>(blk_id[b]) * n_test + t] = v;
    }
}
