/* Synthetic PLINK panel generator (benchmark / scale-test tooling; not a reference interface).
 * Model: SURVEY.md §8d synthetic generator -- AR(1) latent haplotypes per LD block, dosage =
 * h1 + h2, thresholded at Phi^-1(p).  Built as dbslmm_amd/libdbslmm_synth.so. */
#ifndef DBSLMM_SYNTH_H
#define DBSLMM_SYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* rows: host buffer of blk_ptr[num_block] * ceil(n_ref/4) bytes (SNP-major PLINK rows, no magic).
 * blk_ptr[b]..blk_ptr[b+1] = SNPs of block b (AR(1) restarts at each block), thr[s] = Phi^-1(p_s).
 * Returns 0, -1 (argument) or -2 (HIP error; see dbslmm_synth_last_error). */
int dbslmm_synth_bed(int device, int32_t num_block, const int64_t* blk_ptr, const float* thr,
                     int32_t n_ref, uint64_t seed, float rho, float miss_rate, uint8_t* rows);
const char* dbslmm_synth_last_error(void);
#ifdef __cplusplus
}
#endif
#endif
