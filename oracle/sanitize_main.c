/*
 * sanitize_main.c -- host-sanitizer driver for the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Built with -fsanitize=address,undefined by `make -C oracle sanitize` and run by
 * tests/test_sanitizers.py (CPU suite).  It links dbslmm_oracle.c directly (no Python, no
 * preloaded runtime) and drives every entry point over a PLINK .bed image:
 *   oracle_bed_maf, oracle_read_snp_im (all-ones and 0/1 indicators), oracle_read_block_std,
 *   oracle_est (DBSLMM large+small and LMM-only, PCG and direct, ragged and empty blocks).
 *
 *   sanitize_main <bed path> <n_ref> <n_snp>
 * prints "ok <checksum>" and exits 0 when every call returned 0 (a sanitizer report aborts).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int oracle_bed_maf(const uint8_t* bed, int32_t n_ref, int64_t n_snp, double* maf, int threads);
int oracle_read_snp_im(const uint8_t* bed, int64_t pos, const int32_t* indicator, int64_t ni_total,
                       double* geno, int64_t geno_len, double* maf);
int oracle_read_block_std(const uint8_t* bed, int32_t n_ref, const int32_t* rows, int64_t m, double* out,
                          int threads);
int oracle_est(const uint8_t* bed, int n_ref, int n_obs, double sigma_s, double tau, int num_block,
               const int64_t* s_ptr, const int32_t* s_rows, const double* z_s, const int64_t* l_ptr,
               const int32_t* l_rows, const double* z_l, double* beta_s, double* beta_l, int threads,
               int method, int32_t* status);

static uint8_t* slurp(const char* path, long* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *len = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* b = (uint8_t*)malloc((size_t)*len);
    if (fread(b, 1, (size_t)*len, f) != (size_t)*len) { free(b); b = NULL; }
    fclose(f);
    return b;
}

int main(int argc, char** argv) {
    if (argc != 4) { fprintf(stderr, "usage: %s bed n_ref n_snp\n", argv[0]); return 2; }
    long len = 0;
    uint8_t* bed = slurp(argv[1], &len);
    const int n_ref = atoi(argv[2]);
    const int64_t n_snp = atoll(argv[3]);
    if (!bed || n_ref < 2 || n_snp < 8 || len < 3 + n_snp * ((n_ref + 3) / 4)) { fprintf(stderr, "bad input\n"); return 2; }
    double sum = 0.0;
    int rc = 0;

    double* maf = (double*)malloc(sizeof(double) * (size_t)n_snp);
    rc |= oracle_bed_maf(bed, n_ref, n_snp, maf, 2);
    for (int64_t i = 0; i < n_snp; ++i) sum += maf[i];

    /* readSNPIm with a 0/1 indicator (every third individual dropped) */
    int32_t* ind = (int32_t*)malloc(sizeof(int32_t) * (size_t)n_ref);
    int n_sel = 0;
    for (int i = 0; i < n_ref; ++i) n_sel += (ind[i] = (i % 3 != 2));
    double* geno = (double*)malloc(sizeof(double) * (size_t)n_ref);
    for (int64_t r = 0; r < n_snp; r += 7) {
        double mf = 0.0;
        rc |= oracle_read_snp_im(bed, r, ind, n_ref, geno, n_sel, &mf) != n_sel;   /* returns the kept count */
        sum += mf;
    }

    /* blocks of ragged sizes 0, 1, 2, ... over consecutive rows; every 5th SNP large */
    int nb = 0;
    int64_t used = 0;
    while (used + nb <= n_snp && nb < 64) used += nb++;
    int64_t* s_ptr = (int64_t*)calloc((size_t)nb + 1, sizeof(int64_t));
    int64_t* l_ptr = (int64_t*)calloc((size_t)nb + 1, sizeof(int64_t));
    int32_t* s_rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)(used + 1));
    int32_t* l_rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)(used + 1));
    double* z_s = (double*)malloc(sizeof(double) * (size_t)(used + 1));
    double* z_l = (double*)malloc(sizeof(double) * (size_t)(used + 1));
    int64_t ns = 0, nl = 0, row = 0;
    for (int b = 0; b < nb; ++b) {
        for (int i = 0; i < b; ++i, ++row) {
            const double z = sin(0.37 * (double)row) * 3.0;
            if (row % 5 == 4) { l_rows[nl] = (int32_t)row; z_l[nl++] = 6.0 * (z >= 0 ? 1 : -1); }
            else { s_rows[ns] = (int32_t)row; z_s[ns++] = z; }
        }
        s_ptr[b + 1] = ns;
        l_ptr[b + 1] = nl;
    }
    double* bs = (double*)malloc(sizeof(double) * (size_t)(ns + 1));
    double* bl = (double*)malloc(sizeof(double) * (size_t)(nl + 1));
    int32_t* st = (int32_t*)malloc(sizeof(int32_t) * (size_t)nb);
    int bad_blocks = 0;   /* non-PD / monomorphic blocks (status != 0): reported, not an error here */
    for (int method = 0; method < 2; ++method)
        for (int lmm = 0; lmm < 2; ++lmm) {
            oracle_est(bed, n_ref, 100000, 0.5 / (double)used, 0.8, nb, s_ptr, s_rows, z_s,
                       lmm ? NULL : l_ptr, l_rows, z_l, bs, bl, 2, method, st);
            for (int b = 0; b < nb; ++b) bad_blocks += st[b] != 0;
            for (int64_t i = 0; i < ns; ++i) sum += isfinite(bs[i]) ? bs[i] : 0.0;   /* NaN: monomorphic block */
            if (!lmm)
                for (int64_t i = 0; i < nl; ++i) sum += isfinite(bl[i]) ? bl[i] : 0.0;
        }

    /* standardised block columns */
    const int64_t mb = n_snp < 40 ? n_snp : 40;
    int32_t* rows = (int32_t*)malloc(sizeof(int32_t) * (size_t)mb);
    for (int64_t i = 0; i < mb; ++i) rows[i] = (int32_t)(n_snp - 1 - i);
    double* X = (double*)malloc(sizeof(double) * (size_t)(n_ref * mb));
    rc |= oracle_read_block_std(bed, n_ref, rows, mb, X, 2);
    for (int64_t i = 0; i < n_ref * mb; ++i) sum += isfinite(X[i]) ? X[i] * 1e-3 : 0.0;

    free(rows); free(X); free(bs); free(bl); free(st); free(s_ptr); free(l_ptr); free(s_rows);
    free(l_rows); free(z_s); free(z_l); free(geno); free(ind); free(maf); free(bed);
    if (rc) { fprintf(stderr, "oracle call failed rc=%d\n", rc); return 1; }
    printf("ok %.6e blocks %d nonzero-status %d\n", sum, nb, bad_blocks);
    return 0;
}
