/*
 * dbslmm_oracle.c -- CPU restatement of DBSLMM's per-LD-block effect-size path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / the timed CPU baseline.  The product
 * library (dbslmm_amd/libdbslmm_hip.so) never links or calls it.
 *
 * It restates the reference algorithm (fboehm/DBSLMM, paths under scr/):
 *   oracle_read_snp_im   IO::readSNPIm            dtpr.cpp:285-364  (byte-wise decode, mean impute)
 *   oracle_normalize     SNPPROC::nomalizeVec     dtpr.cpp:375-380  (Armadillo mean/var order, N-1)
 *   oracle_bed_maf       MAF pass of IO::readBim  dtpr.cpp:93-102
 *   pcg_v                DBSLMMFIT::PCGv          dbslmmfit.cpp:629-668 (abs tol 1e-7, maxiter 1000)
 *   oracle_est_block     DBSLMMFIT::estBlock x2   dbslmmfit.cpp:680-738, 740-770
 *   oracle_est           DBSLMMFIT::est x2        dbslmmfit.cpp:56-244, 247-363 (beta part;
 *                        OpenMP schedule(dynamic) over blocks as at :191-192)
 *
 * Gram products (Armadillo -> BLAS dsyrk/dgemm, gemv in PCG) use the OpenBLAS that ships with
 * NumPy when oracle_use_blas() was given its path (mirrors the reference's -lblas build,
 * scr/Makefile:20), otherwise plain loops.  Parity is pinned by tests/test_oracle.py against the
 * Manual known-answer test (Rmd/Manual.Rmd:126-145) and the committed golden vectors.
 */
#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ optional OpenBLAS (ILP64) */
typedef void (*dsyrk_fn)(int, int, int, int64_t, int64_t, double, const double*, int64_t, double,
                         double*, int64_t);
typedef void (*dgemm_fn)(int, int, int, int64_t, int64_t, int64_t, double, const double*, int64_t,
                         const double*, int64_t, double, double*, int64_t);
typedef void (*dgemv_fn)(int, int, int64_t, int64_t, double, const double*, int64_t, const double*,
                         int64_t, double, double*, int64_t);
typedef void (*setthr_fn)(int);
static setthr_fn p_setthr;
static dsyrk_fn p_dsyrk;
static dgemm_fn p_dgemm;
static dgemv_fn p_dgemv;
enum { kColMajor = 102, kNoTrans = 111, kTrans = 112, kUpper = 121 };

int oracle_use_blas(const char* path) {
    void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    p_dsyrk = (dsyrk_fn)dlsym(h, "scipy_cblas_dsyrk64_");
    p_dgemm = (dgemm_fn)dlsym(h, "scipy_cblas_dgemm64_");
    p_dgemv = (dgemv_fn)dlsym(h, "scipy_cblas_dgemv64_");
    p_setthr = (setthr_fn)dlsym(h, "scipy_openblas_set_num_threads64_");
    if (p_setthr) p_setthr(1); /* block-level OpenMP over single-threaded BLAS, as the reference */
    if (!p_dsyrk || !p_dgemm || !p_dgemv) { p_dsyrk = 0; p_dgemm = 0; p_dgemv = 0; return -2; }
    return 0;
}

int oracle_blas_active(void) { return p_dsyrk != 0; }

/* BLAS threads inside one call (default 1 = the reference's -lblas build).  The full-size parity
 * tests give a single huge block (m ~ 10k) all host cores; NumPy shares this OpenBLAS, so the
 * setting also governs NumPy's matmul / LAPACK in the same process. */
int oracle_blas_threads(int n) {
    if (!p_setthr) return -1;
    p_setthr(n > 0 ? n : 1);
    return 0;
}

/* C(m x m) = A^T A, A col-major n x m (both triangles filled). */
static void gram_tt(const double* A, int64_t n, int64_t m, double* C) {
    if (m == 0) return;
    if (p_dsyrk) {
        p_dsyrk(kColMajor, kUpper, kTrans, m, n, 1.0, A, n, 0.0, C, m);
        for (int64_t j = 0; j < m; ++j)
            for (int64_t i = j + 1; i < m; ++i) C[i + j * m] = C[j + i * m];
        return;
    }
    for (int64_t j = 0; j < m; ++j)
        for (int64_t i = 0; i <= j; ++i) {
            const double* a = A + i * n;
            const double* b = A + j * n;
            double s = 0.0;
            for (int64_t k = 0; k < n; ++k) s += a[k] * b[k];
            C[i + j * m] = s;
            C[j + i * m] = s;
        }
}

/* C(p x q) = A^T B ; A n x p, B n x q col-major. */
static void gemm_tn(const double* A, const double* B, int64_t n, int64_t p, int64_t q, double* C) {
    if (p == 0 || q == 0) return;
    if (p_dgemm) { p_dgemm(kColMajor, kTrans, kNoTrans, p, q, n, 1.0, A, n, B, n, 0.0, C, p); return; }
    for (int64_t j = 0; j < q; ++j)
        for (int64_t i = 0; i < p; ++i) {
            double s = 0.0;
            for (int64_t k = 0; k < n; ++k) s += A[k + i * n] * B[k + j * n];
            C[i + j * p] = s;
        }
}

/* y = op(A) x ; A rows x cols col-major */
static void gemv(int trans, const double* A, int64_t rows, int64_t cols, const double* x, double* y) {
    int64_t ylen = trans ? cols : rows;
    if (ylen == 0) return;
    if (p_dgemv && rows > 0 && cols > 0) {
        p_dgemv(kColMajor, trans ? kTrans : kNoTrans, rows, cols, 1.0, A, rows, x, 1, 0.0, y, 1);
        return;
    }
    if (!trans) {
        for (int64_t i = 0; i < rows; ++i) y[i] = 0.0;
        for (int64_t j = 0; j < cols; ++j)
            for (int64_t i = 0; i < rows; ++i) y[i] += A[i + j * rows] * x[j];
    } else {
        for (int64_t j = 0; j < cols; ++j) {
            double s = 0.0;
            for (int64_t i = 0; i < rows; ++i) s += A[i + j * rows] * x[i];
            y[j] = s;
        }
    }
}

static double dot(const double* a, const double* b, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += a[i] * b[i];
    return s;
}

/* ------------------------------------------------------------------ genotype reader */

static int64_t n_bytes_per_snp(int64_t n) { return n / 4 + ((n % 4) ? 1 : 0); }

/* IO::readSNPIm (dtpr.cpp:285-364).  bed = whole .bed file incl. 3 magic bytes.
 * indicator: ni_total 0/1 entries; geno receives the selected individuals. */
int oracle_read_snp_im(const uint8_t* bed, int64_t pos, const int32_t* indicator,
                       int64_t ni_total, double* geno, int64_t geno_len, double* maf) {
    const int64_t n_bit = n_bytes_per_snp(ni_total);
    const uint8_t* row = bed + 3 + pos * n_bit;                 /* seekg(pos*n_bit + 3) :302 */
    double geno_mean = 0.0;
    int64_t c = 0, c_idv = 0, n_miss = 0;
    int64_t* miss = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ni_total + 1));
    for (int64_t i = 0; i < n_bit; ++i) {
        const unsigned b = row[i];
        for (int j = 0; j < 4; ++j) {
            if (i == n_bit - 1 && c == ni_total) break;          /* :321 */
            if (indicator[c] == 0) { c++; continue; }             /* :323-326 */
            c++;
            const unsigned lo = (b >> (2 * j)) & 1u, hi = (b >> (2 * j + 1)) & 1u;
            if (lo == 0) {
                if (hi == 0) { geno[c_idv] = 2.0; geno_mean += 2.0; }
                else { geno[c_idv] = 1.0; geno_mean += 1.0; }
            } else {
                if (hi == 1) { geno[c_idv] = 0.0; }
                else { miss[n_miss++] = c_idv; }
            }
            c_idv++;
        }
    }
    geno_mean /= (double)(c_idv - n_miss);                        /* :358 */
    for (int64_t i = 0; i < n_miss; ++i) geno[miss[i]] = geno_mean;
    free(miss);
    /* af = 0.5 * sum(geno) / geno.n_elem  (:361; Armadillo accumulate order) */
    double a1 = 0.0, a2 = 0.0;
    int64_t i = 0, j = 1;
    for (; j < geno_len; i += 2, j += 2) { a1 += geno[i]; a2 += geno[j]; }
    if (i < geno_len) a1 += geno[i];
    const double af = 0.5 * (a1 + a2) / (double)geno_len;
    *maf = af < 1.0 - af ? af : 1.0 - af;
    return (int)c_idv;
}

/* SNPPROC::nomalizeVec (dtpr.cpp:375-380) with Armadillo's accumulate / direct_var order. */
static double arma_mean(const double* x, int64_t n) {
    double a1 = 0.0, a2 = 0.0;
    int64_t i = 0, j = 1;
    for (; j < n; i += 2, j += 2) { a1 += x[i]; a2 += x[j]; }
    if (i < n) a1 += x[i];
    return (a1 + a2) / (double)n;
}

void oracle_normalize(double* x, int64_t n) {
    const double m0 = arma_mean(x, n);
    for (int64_t k = 0; k < n; ++k) x[k] -= m0;
    const double m = arma_mean(x, n);
    double acc2 = 0.0, acc3 = 0.0;
    int64_t i = 0, j = 1;
    for (; j < n; i += 2, j += 2) {
        const double ti = m - x[i], tj = m - x[j];
        acc2 += ti * ti + tj * tj;
        acc3 += ti + tj;
    }
    if (i < n) { const double ti = m - x[i]; acc2 += ti * ti; acc3 += ti; }
    const double sd = sqrt((acc2 - acc3 * acc3 / (double)n) / (double)(n - 1));
    for (int64_t k = 0; k < n; ++k) x[k] /= sd;
}

/* MAF pass over every SNP (IO::readBim, dtpr.cpp:93-102). */
int oracle_bed_maf(const uint8_t* bed, int32_t n_ref, int64_t n_snp, double* maf, int threads) {
    int32_t* idv = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_ref);
    for (int i = 0; i < n_ref; ++i) idv[i] = 1;
#pragma omp parallel num_threads(threads > 0 ? threads : 1)
    {
        double* g = (double*)malloc(sizeof(double) * (size_t)n_ref);
#pragma omp for schedule(static)
        for (int64_t s = 0; s < n_snp; ++s) oracle_read_snp_im(bed, s, idv, n_ref, g, n_ref, &maf[s]);
        free(g);
    }
    free(idv);
    return 0;
}

/* calcBlock's column loop (dbslmmfit.cpp:419-430) for one block: readSNPIm + nomalizeVec of
 * bed rows rows[0..m) into out (n_ref x m col-major), columns in parallel. */
int oracle_read_block_std(const uint8_t* bed, int32_t n_ref, const int32_t* rows, int64_t m,
                          double* out, int threads) {
    int32_t* idv = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_ref);
    for (int i = 0; i < n_ref; ++i) idv[i] = 1;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (int64_t c = 0; c < m; ++c) {
        double maf;
        oracle_read_snp_im(bed, rows[c], idv, n_ref, out + c * (int64_t)n_ref, n_ref, &maf);
        oracle_normalize(out + c * (int64_t)n_ref, n_ref);
    }
    free(idv);
    return 0;
}

/* ------------------------------------------------------------------ solvers */

/* DBSLMMFIT::PCGv (dbslmmfit.cpp:629-668). Returns iterations. */
static int pcg_v(const double* A, int64_t m, const double* b, double* x, int maxiter, double tol) {
    if (m == 0) return 0;
    double* w = (double*)malloc(sizeof(double) * (size_t)m * 6);
    double *Minv = w, *r = w + m, *z = w + 2 * m, *p = w + 3 * m, *Ap = w + 4 * m, *z1 = w + 5 * m;
    for (int64_t i = 0; i < m; ++i) {
        double d = A[i + i * m];
        if (d == 0) d = 1e-4;
        Minv[i] = 1.0 / d;
        x[i] = 0.0;
        r[i] = b[i];
        z[i] = Minv[i] * r[i];
        p[i] = z[i];
    }
    int it = 0;
    double sumr2 = sqrt(dot(r, r, m));
    while (sumr2 > tol && it < maxiter) {
        it++;
        gemv(0, A, m, m, p, Ap);
        const double a = dot(r, z, m) / dot(p, Ap, m);
        for (int64_t i = 0; i < m; ++i) x[i] += a * p[i];
        const double rz_old = dot(z, r, m);
        for (int64_t i = 0; i < m; ++i) { r[i] -= a * Ap[i]; z1[i] = Minv[i] * r[i]; }
        const double bet = dot(z1, r, m) / rz_old;
        for (int64_t i = 0; i < m; ++i) { p[i] = z1[i] + bet * p[i]; z[i] = z1[i]; }
        sumr2 = sqrt(dot(r, r, m));
    }
    free(w);
    return it;
}

/* In-place Cholesky (lower) of SPD col-major m x m; returns 0 or the failing column + 1. */
static int chol(double* A, int64_t m) {
    for (int64_t j = 0; j < m; ++j) {
        double d = A[j + j * m];
        for (int64_t k = 0; k < j; ++k) d -= A[j + k * m] * A[j + k * m];
        if (!(d > 0.0)) return (int)j + 1;
        d = sqrt(d);
        A[j + j * m] = d;
        for (int64_t i = j + 1; i < m; ++i) {
            double s = A[i + j * m];
            for (int64_t k = 0; k < j; ++k) s -= A[i + k * m] * A[j + k * m];
            A[i + j * m] = s / d;
        }
    }
    return 0;
}

static void chol_solve(const double* L, int64_t m, double* b) {
    for (int64_t i = 0; i < m; ++i) {
        double s = b[i];
        for (int64_t k = 0; k < i; ++k) s -= L[i + k * m] * b[k];
        b[i] = s / L[i + i * m];
    }
    for (int64_t i = m - 1; i >= 0; --i) {
        double s = b[i];
        for (int64_t k = i + 1; k < m; ++k) s -= L[k + i * m] * b[k];
        b[i] = s / L[i + i * m];
    }
}

/* solve A x = b with method 0 = reference PCG, 1 = Cholesky. A is not modified. */
static int solve_v(const double* A, const double* Lfac, int64_t m, const double* b, double* x, int method) {
    if (method == 0) return pcg_v(A, m, b, x, 1000, 1e-7);
    memcpy(x, b, sizeof(double) * (size_t)m);
    chol_solve(Lfac, m, x);
    return 0;
}

/* DBSLMMFIT::estBlock.  Xs: n_ref x m_s, Xl: n_ref x m_l (col-major, standardised).
 * m_l == 0 -> small-only overload.  iters (optional) receives the summed PCG iterations.
 * Returns 0, or >0 when a Cholesky failed (method 1). */
int oracle_est_block(int n_ref, int n_obs, double sigma_s, double tau, const double* Xs, int m_s,
                     const double* Xl, int m_l, const double* z_s, const double* z_l,
                     double* beta_s, double* beta_l, int method, int* iters) {
    const int64_t ms = m_s, ml = m_l;
    const double dsh = 1.0 / (sigma_s * (double)n_obs);
    const double sqn = sqrt((double)n_obs);
    int total_it = 0, rc = 0;
    double* Sss = (double*)calloc((size_t)(ms * ms + 1), sizeof(double));
    gram_tt(Xs, n_ref, ms, Sss);
    for (int64_t k = 0; k < ms * ms; ++k) Sss[k] *= tau / (double)n_ref;
    for (int64_t i = 0; i < ms; ++i) Sss[i + i * ms] += 1.0 - tau;
    for (int64_t i = 0; i < ms; ++i) Sss[i + i * ms] += dsh;   /* A = Sss + dI (:712 / :759) */
    double* L = NULL;
    if (method == 1) {
        L = (double*)malloc(sizeof(double) * (size_t)(ms * ms + 1));
        memcpy(L, Sss, sizeof(double) * (size_t)(ms * ms));
        rc = chol(L, ms);
        if (rc) { free(L); free(Sss); return rc; }
    }
    double* q = (double*)calloc((size_t)ms + 1, sizeof(double));
    if (ml == 0) {
        total_it += solve_v(Sss, L, ms, z_s, q, method);                       /* :760 */
        for (int64_t i = 0; i < ms; ++i) Sss[i + i * ms] -= dsh;                /* :761 */
        double* t = (double*)calloc((size_t)ms + 1, sizeof(double));
        gemv(0, Sss, ms, ms, q, t);                                             /* :762 */
        for (int64_t i = 0; i < ms; ++i) beta_s[i] = sqn * sigma_s * (z_s[i] - t[i]);   /* :763-764 */
        free(t);
    } else {
        double* Sls = (double*)calloc((size_t)(ml * ms + 1), sizeof(double));   /* m_l x m_s */
        double* Sll = (double*)calloc((size_t)(ml * ml + 1), sizeof(double));
        gemm_tn(Xl, Xs, n_ref, ml, ms, Sls);                                    /* :698 */
        for (int64_t k = 0; k < ml * ms; ++k) Sls[k] *= tau / (double)n_ref;
        gram_tt(Xl, n_ref, ml, Sll);                                            /* :700 */
        for (int64_t k = 0; k < ml * ml; ++k) Sll[k] *= tau / (double)n_ref;
        for (int64_t i = 0; i < ml; ++i) Sll[i + i * ml] += 1.0 - tau;
        /* P = A^-1 Sigma_sl (m_s x m_l), column by column (PCGm :713) */
        double* P = (double*)calloc((size_t)(ms * ml + 1), sizeof(double));
        double* col = (double*)calloc((size_t)ms + 1, sizeof(double));
        for (int64_t c = 0; c < ml; ++c) {
            for (int64_t i = 0; i < ms; ++i) col[i] = Sls[c + i * ml];
            total_it += solve_v(Sss, L, ms, col, P + c * ms, method);
        }
        /* S = Sll - Sls P  (:714-715) */
        double* S = (double*)calloc((size_t)(ml * ml + 1), sizeof(double));
        for (int64_t j = 0; j < ml; ++j)
            for (int64_t i = 0; i < ml; ++i) {
                double s = 0.0;
                for (int64_t k = 0; k < ms; ++k) s += Sls[i + k * ml] * P[k + j * ms];
                S[i + j * ml] = Sll[i + j * ml] - s;
            }
        total_it += solve_v(Sss, L, ms, z_s, q, method);                       /* :716 */
        double* rhs = (double*)calloc((size_t)ml + 1, sizeof(double));
        gemv(0, Sls, ml, ms, q, rhs);                                           /* :717-718 */
        for (int64_t i = 0; i < ml; ++i) rhs[i] = z_l[i] - rhs[i];
        if (method == 0) {
            total_it += pcg_v(S, ml, rhs, beta_l, 1000, 1e-7);                 /* :719 */
        } else {
            double* LS = (double*)malloc(sizeof(double) * (size_t)(ml * ml));
            memcpy(LS, S, sizeof(double) * (size_t)(ml * ml));
            int r2 = chol(LS, ml);
            if (r2) rc = -r2;
            memcpy(beta_l, rhs, sizeof(double) * (size_t)ml);
            if (!r2) chol_solve(LS, ml, beta_l);
            free(LS);
        }
        for (int64_t i = 0; i < ml; ++i) beta_l[i] /= sqn;                     /* :720 */
        /* :723-729 in the reference's order of operations */
        double* Pb = (double*)calloc((size_t)ms + 1, sizeof(double));
        gemv(0, P, ms, ml, beta_l, Pb);
        double* w = (double*)calloc((size_t)ms + 1, sizeof(double));
        for (int64_t i = 0; i < ms; ++i) w[i] = q[i] * sqn - (double)n_obs * Pb[i];
        for (int64_t i = 0; i < ms; ++i) Sss[i + i * ms] -= dsh;                /* :726 */
        double* Sw = (double*)calloc((size_t)ms + 1, sizeof(double));
        gemv(0, Sss, ms, ms, w, Sw);                                            /* :727 */
        double* Sslb = (double*)calloc((size_t)ms + 1, sizeof(double));
        gemv(1, Sls, ml, ms, beta_l, Sslb);                                     /* Sls^T beta_l */
        for (int64_t i = 0; i < ms; ++i)
            beta_s[i] = (sqn * z_s[i] - (double)n_obs * Sslb[i] - Sw[i]) * sigma_s;   /* :728-729 */
        free(Pb); free(w); free(Sw); free(Sslb); free(rhs); free(S); free(col); free(P);
        free(Sll); free(Sls);
    }
    if (iters) *iters = total_it;
    free(q);
    free(L);
    free(Sss);
    return rc;
}

/* DBSLMMFIT::est (dbslmmfit.cpp:56-363), beta part.  CSR over blocks: block b's small SNPs are
 * s_rows[s_ptr[b] .. s_ptr[b+1]) (bed row indices) with z-scores z_s[...] and outputs
 * beta_s[...]; same for large (l_ptr may be NULL -> LMM-only overload).  Blocks run in an
 * OpenMP dynamic schedule (the reference batches 60 blocks at a time; batching only adds
 * barriers, it does not change any block's arithmetic). */
int oracle_est(const uint8_t* bed, int n_ref, int n_obs, double sigma_s, double tau, int num_block,
               const int64_t* s_ptr, const int32_t* s_rows, const double* z_s,
               const int64_t* l_ptr, const int32_t* l_rows, const double* z_l,
               double* beta_s, double* beta_l, int threads, int method, int32_t* status) {
    int32_t* idv = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_ref);
    for (int i = 0; i < n_ref; ++i) idv[i] = 1;
    int err = 0;
#pragma omp parallel for schedule(dynamic) num_threads(threads > 0 ? threads : 1) reduction(| : err)
    for (int b = 0; b < num_block; ++b) {
        const int64_t s0 = s_ptr[b], ms = s_ptr[b + 1] - s_ptr[b];
        const int64_t l0 = l_ptr ? l_ptr[b] : 0, ml = l_ptr ? l_ptr[b + 1] - l_ptr[b] : 0;
        if (ms + ml == 0) { if (status) status[b] = 0; continue; }
        double* Xs = (double*)malloc(sizeof(double) * (size_t)(n_ref * ms + 1));
        double* Xl = (double*)malloc(sizeof(double) * (size_t)(n_ref * ml + 1));
        double maf;
        for (int64_t i = 0; i < ms; ++i) {
            oracle_read_snp_im(bed, s_rows[s0 + i], idv, n_ref, Xs + i * n_ref, n_ref, &maf);
            oracle_normalize(Xs + i * n_ref, n_ref);
        }
        for (int64_t i = 0; i < ml; ++i) {
            oracle_read_snp_im(bed, l_rows[l0 + i], idv, n_ref, Xl + i * n_ref, n_ref, &maf);
            oracle_normalize(Xl + i * n_ref, n_ref);
        }
        int rc = oracle_est_block(n_ref, n_obs, sigma_s, tau, Xs, (int)ms, Xl, (int)ml, z_s + s0,
                                  ml ? z_l + l0 : NULL, beta_s + s0, ml ? beta_l + l0 : NULL,
                                  method, NULL);
        if (status) status[b] = rc;
        if (rc) err |= 1;
        free(Xs);
        free(Xl);
    }
    free(idv);
    return err;
}
