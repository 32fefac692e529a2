/*
 * dbslmm_hip.h -- C-ABI of the MI355X (gfx950) per-LD-block effect-size solver.
 *
 * Drop-in boundary for the hot path of fboehm/DBSLMM.  Every entry point below replaces one
 * reference interface (paths relative to the reference's scr/):
 *
 *   dbslmm_est            DBSLMMFIT::est (large+small, dbslmmfit.hpp:38-53, dbslmmfit.cpp:56-244)
 *                         and DBSLMMFIT::est (small only, dbslmmfit.hpp:55-66, :247-363):
 *                         l_ptr == NULL selects the LMM-only overload.  Called where
 *                         DBSLMM::BatchRun calls est (dbslmm.cpp:334-348, 375-386).
 *   dbslmm_plan_*         the same call split into upload / run / download so the solve can be
 *                         repeated with inputs resident in HBM (bench, h2f tuning).
 *   dbslmm_bed_maf        the MAF pass of IO::readBim (dtpr.cpp:93-102) = readSNPIm over every
 *                         reference SNP, maf only.
 *   dbslmm_read_snp_std   IO::readSNPIm + SNPPROC::nomalizeVec (dtpr.cpp:285-364, 375-380) for a
 *                         list of bed rows: standardised fp64 columns (parity / diagnostics).
 *
 * Conventions: plain pointers and sizes, no C++ types, no exceptions across the boundary.
 * Every call returns 0 on success or a negative DBSLMM_E* code; dbslmm_last_error(ctx) then
 * holds a message.  The caller owns every buffer; inputs are read-only for the call.  One call
 * at a time per context; distinct contexts are independent.  A context drives one GPU
 * (dbslmm_ctx_create) or several (dbslmm_ctx_create_multi: the LD blocks of every plan are
 * sharded over the devices).
 */
#ifndef DBSLMM_HIP_H_
#define DBSLMM_HIP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DBSLMM_ABI_VERSION 15

enum {
    DBSLMM_OK = 0,
    DBSLMM_E_ARG = -1,      /* invalid argument (sizes, NULL, ranges) */
    DBSLMM_E_HIP = -2,      /* HIP runtime error (no device, OOM, launch failure) */
    DBSLMM_E_STATE = -3     /* call sequence error (plan not run, ...) */
};

/* Per-block status written by dbslmm_est / dbslmm_plan_download. */
enum {
    DBSLMM_BLOCK_OK = 0,
    DBSLMM_BLOCK_EMPTY = 1,        /* no SNP in this block */
    DBSLMM_BLOCK_NOT_PD = 2,       /* joint LD matrix not positive definite -> beta = NaN
                                      (reference: PCG "Matrix is Singular!", dbslmmfit.cpp:664) */
    DBSLMM_BLOCK_MONOMORPHIC = 3,  /* a SNP with zero variance -> NaN column in the reference
                                      (dtpr.cpp:375-380); beta = NaN for the whole block */
    DBSLMM_BLOCK_NOT_CONVERGED = 4 /* an iterative solve stopped at its iteration cap without
                                      meeting its error bound: beta = the last iterate (the
                                      reference's PCG prints "Matrix is Singular!" at maxiter and
                                      returns its iterate, dbslmmfit.cpp:664-666).  The PCG route
                                      (solver, pcg_maxit) and the h2f copies iterated on a base
                                      factor (h2f_iter: CG / Chebyshev at their caps) report it. */
};

typedef struct dbslmm_ctx dbslmm_ctx;
typedef struct dbslmm_plan dbslmm_plan;

/* Path selection of a plan (the product has ONE numerical path per block size class; these
 * fields only move the size thresholds, e.g. so tests can drive every kernel class at small
 * sizes).  Zero-initialise for the defaults; every field's 0 means "default".
 *
 * tiled_min      blocks with m >= tiled_min take the multi-workgroup tiled factorisation
 *                (default 384, or 256 when no block reaches 512; minimum 64)
 * gram_big_min   blocks with m >= this use the 128 x 128-tile Gram kernel (default 96)
 * gram_huge_min  ... and the 256 x 256-tile one from here (default 384, 768 when n_ref < 4096)
 * h2f_mode       plan_run_multi: 0 = tiled blocks factored once, the other sigmas solved by
 *                Chebyshev iteration on that factor when the bound allows (tau in (0, 1],
 *                <= 60 iterations); 1 = one factorisation per sigma (the merged sequence)
 * cheb_tol       relative error target of the h2f copies iterated on the base copy's factor (default
 *                1e-9: four orders below the 1e-5 parity bar on beta, one below the reference PCG's
 *                own deviation from the exact solution (~1e-8)).  CG (the default h2f_iter) stops a
 *                block once |r| <= cheb_tol lambda_min(M_c) |x| (5.03 iterations per tiled block at
 *                config 4); Chebyshev runs its a priori count (7 at h2f 0.8 / 1 / 1.2), which is
 *                also CG's cap
 * lead_min       tiled blocks with m >= lead_min form the lead group: their Gram tiles run first
 *                and their factorisation (the longest dependency chains) starts right after
 *                them, beside the rest of the Gram and the other blocks' factorisation (default
 *                max(1536, m_max / 8) when tiled blocks lie on both sides of it; < 0: no lead
 *                group, and the tiled sequence starts after the whole Gram instead of right
 *                after the tiled blocks' Gram tiles).  Scheduling only: the results are
 *                bit-identical either way.
 * large_cheb     plan_run_multi with Chebyshev h2f: the single-workgroup blocks (64 <= m+1, m
 *                below tiled_min) iterate on the base copy's factor too (0 = on when every such
 *                block fits the iteration kernel, ld <= 512; -1 = off: every copy factored)
 * cheb_fused     1 = all Chebyshev passes of a copy group in one persistent launch over every tiled
 *                block (experimental, bit-identical, slower at config 4; turns sub_split off);
 *                0 = one launch per pass
 * debug_delay_us testing only: a spin kernel of this many microseconds at the head of every
 *                concurrently running stream segment (the bulk trailing launches of each tiled
 *                sequence, the rest sequence, the main stream after the lead fork, the lead
 *                sequence), so a missing cross-stream dependency fails deterministically
 *                instead of by timing.  Results must be bit-identical to a run without it.
 * debug_stop     testing only: 1 = stop every run after the Gram (the block matrices then hold
 *                Sigma, dbslmm_plan_block_matrix); 0 = the full solve
 * sub_split      scheduling, plans with a lead group: 0 / 1 = the substitutions (backward solve and
 *                h2f Chebyshev passes) run per group -- the rest group's right after its own
 *                factorisation, beside the lead group's, on sub_grid_rest / sub_grid_lead
 *                persistent workgroups (default); -1 = one launch sequence over all tiled blocks
 *                after both factorisations.  Scheduling only: bit-identical results.
 *                2 = as 0 / 1, but the rest group's h2f copies iterate with one workgroup per
 *                block (every Chebyshev pass in one launch, dbslmm_tcheb; blocks up to 4096 SNPs,
 *                otherwise as 0): results within cheb_tol, not bit-identical to 0 / 1.
 * sub_grid_lead, sub_grid_rest   their persistent grids (0 = default: 5/16 of the CUs for
 *                the lead group, the other three quarters for the rest)
 * shard_copies   multi-device plans (dbslmm_ctx_create_multi): the number of h2f solves each
 *                run_multi call will request (0 / 1: single solves).  With K >= 2 and at least K
 *                devices the shard plan may split the K copies of the blocks whose dependency chain
 *                exceeds the fair share of the step into K (block, copy) units on distinct devices
 *                (dbslmm_shard_plan).  Any n_sigma still works: with n_sigma != K a split block is
 *                solved whole on the device of its copy 0.  Ignored by single-device plans.
 * h2f_iter       h2f_mode 0, the iterated copies (tiled and single-workgroup blocks): 1 = Chebyshev
 *                (a priori coefficients and iteration count), 2 = preconditioned CG on the same
 *                factor (Chronopoulos-Gear form, dbslmm_cg_update / dbslmm_chol_cheb): stops per
 *                block once |r| <= cheb_tol lambda_min(M_c) |x|,
 *                capped at the Chebyshev count (a copy still above the bound there is reported
 *                DBSLMM_BLOCK_NOT_CONVERGED); 0 = the default (2).  Both within cheb_tol; the
 *                base copy is bit-identical either way.  (cheb_fused = 1 and the whole-block rest
 *                group of sub_split = 2 iterate by Chebyshev.)
 * solver         how a run solves its blocks (ABI 12): 1 = factorisation (fp64 Cholesky of every
 *                block, the paths above); 2 = PCG: the reference's own algorithm (Jacobi-PCG,
 *                dbslmmfit.cpp:629-678) on the joint matrix of every block, all h2f copies as
 *                right-hand sides of one iteration, the LD matrix streamed from the Gram as exact
 *                integers (uint16; fp64 Sigma for blocks with missing calls or n_ref > 16383);
 *                0 = auto: PCG when every copy is well conditioned by its prior shift
 *                (1/(sigma_s n) >= 2, so that kappa <= ~6 and <= ~35 iterations), 0 < tau < 1
 *                (or no large SNPs), at most 4 copies and no debug_stop; the factorisation
 *                otherwise.  dbslmm_plan_variance needs the factor: after a PCG run it
 *                re-solves the latest sigma by factorisation first.
 * pcg_tol        PCG: relative error bound per block and copy, |x - x*| <= pcg_tol |x*| in the
 *                2-norm, enforced as |r| <= pcg_tol lambda |x| with lambda = 1/(sigma_s n) + 1 - tau
 *                (blocks without large SNPs) or 1 - tau, lower bounds of lambda_min that hold for
 *                any data (0 = default 1e-12)
 * pcg_maxit      PCG: iteration cap (0 = default 1000, the reference's maxiter); a copy still
 *                above its bound there is reported DBSLMM_BLOCK_NOT_CONVERGED with its iterate.
 *                Also lowers the cap of the factorisation route's h2f CG (h2f_iter 2) below its
 *                default, the Chebyshev count.
 * pcg_whole      PCG (ABI 15): blocks of at most 8 tile rows (1024 SNPs) on the uint16 Gram are
 *                solved whole by one workgroup per Krylov sequence (dbslmm_pcg_block) beside the
 *                chip-wide iterations of the others; 0 = default (on), -1 = off (every block on
 *                the chip-wide kernels: A/B and parity tests).  Results agree within pcg_tol.
 */
typedef struct dbslmm_options {
    int32_t tiled_min;
    int32_t gram_big_min;
    int32_t gram_huge_min;
    int32_t h2f_mode;
    double cheb_tol;
    int32_t lead_min;
    int32_t large_cheb;
    int32_t cheb_fused;
    int32_t debug_delay_us;
    int32_t debug_stop;
    int32_t sub_split;
    int32_t sub_grid_lead;
    int32_t sub_grid_rest;
    int32_t shard_copies;
    int32_t h2f_iter;
    int32_t solver;
    double pcg_tol;
    int32_t pcg_maxit;
    int32_t pcg_whole;
} dbslmm_options;

/* One LD-block problem set, the arguments of DBSLMMFIT::est in flat form.
 *
 * bed       the whole PLINK .bed image INCLUDING its 3 magic bytes (host memory); row r of
 *           SNP-major data starts at byte 3 + r*ceil(n_ref/4) (dtpr.cpp:302).
 * n_ref     individuals in the reference .fam (getRow, dbslmm.cpp:232).
 * n_obs     GWAS sample size (-n).
 * sigma_s   h / nsnp (dbslmm.cpp:332).
 * tau       LD shrinkage; the reference hard-codes 0.8 (dbslmmfit.cpp:697,751).
 * num_block number of LD blocks (addBlock's return, dtpr.cpp:455-481).
 * s_ptr     num_block+1 offsets; small SNPs of block b are s_pos[s_ptr[b]..s_ptr[b+1]) (bed
 *           rows, INFO::pos) with z-scores z_s[...] (INFO::z); order = the reference's
 *           info_s order.
 * l_ptr     same for large SNPs, or NULL for the LMM-only path.
 * opts      path-selection thresholds (dbslmm_options), or NULL for the defaults.
 */
typedef struct dbslmm_problem {
    const uint8_t* bed;
    int64_t bed_len;
    int32_t n_ref;
    int32_t n_obs;
    double sigma_s;
    double tau;
    int32_t num_block;
    const int64_t* s_ptr;
    const int32_t* s_pos;
    const double* z_s;
    const int64_t* l_ptr;
    const int32_t* l_pos;
    const double* z_l;
    const dbslmm_options* opts;
} dbslmm_problem;

/* Kernel timing slots reported by dbslmm_plan_kernel_ms. */
enum {
    DBSLMM_K_UNPACK = 0,      /* dbslmm_unpack_stats: 2-bit .bed rows -> 2-bit dosage codes + stats */
    DBSLMM_K_GRAM = 1,        /* dbslmm_gram_i8 / _big / _huge: FP4-MFMA grouped syrk of the exact
                                 integer dosages (2-bit codes expanded on the fly) + fp64
                                 standardising epilogue (PCG route: the integer Gram as uint16) */
    DBSLMM_K_CHOL_LARGE = 2,  /* dbslmm_chol_large: blocks with 64 <= m+1 and m below the tiled
                                 threshold, one workgroup each */
    DBSLMM_K_CHOL_SMALL = 3,  /* dbslmm_chol_small: blocks with <= 63 SNPs, one wave each
                                 (concurrent with CHOL_LARGE when there are no tiled blocks) */
    DBSLMM_K_CHOL_TILED = 4,  /* dbslmm_tchol_*: blocks with m >= the tiled threshold
                                 (dbslmm_options.tiled_min; default 384, or 256 when no block
                                 reaches 512), many workgroups per block,
                                 one launch per panel phase (third stream); the whole sequence */
    DBSLMM_K_TRSV = 5,        /* dbslmm_trsv_fwd/bwd: h2f tuning's CG / Chebyshev iterations of the
                                 tiled blocks on the base copy's factor (run_multi; 0 otherwise) */
    DBSLMM_K_PCG = 6,         /* dbslmm_pcg_*: the PCG route's iterations (init to final; 0 on the
                                 factorisation route) */
    DBSLMM_K_PCG_BLOCK = 7,   /* dbslmm_pcg_block: the small blocks solved whole (ABI 14; runs on a
                                 second stream inside the K_PCG span) */
    DBSLMM_K_COUNT = 8
};

int dbslmm_abi_version(void);

/* Create a context on HIP device `device` (ordinal as seen by this process). */
int dbslmm_ctx_create(int device, dbslmm_ctx** out);

/* Create a context over n_dev HIP devices (ordinals; a device may repeat: several shards on one
 * GPU).  Replaces the reference's only parallelism, OpenMP over LD blocks
 * (scr/dbslmmfit.cpp:191-220), with one GPU per shard: plan_create assigns the work units --
 * (LD block, h2f copy) pairs, dbslmm_shard_plan with dbslmm_options.shard_copies -- to the devices,
 * uploads to each device only the .bed rows of its blocks, and every plan / est call then drives
 * all devices concurrently (one host thread per job) and returns beta, status and variance columns
 * in the caller's original order.  dbslmm_bed_maf splits its rows over the devices; read_snp_std
 * and valid_blocks run on the first device.  n_dev == 1 is dbslmm_ctx_create(device_ids[0]). */
int dbslmm_ctx_create_multi(int32_t n_dev, const int32_t* device_ids, dbslmm_ctx** out);
/* Shard plan (ABI 10): assign the work units of a problem -- (LD block, h2f copy) pairs -- to n_dev
 * devices.  m[b] = SNPs of block b (small + large), n_copies = h2f solves per run (1: single solves).
 * A block's copies stay on one device (one Gram, one factorisation, the other copies iterated on
 * it) unless the block's dependency chain exceeds the fair share of the step and n_dev >= n_copies:
 * then each copy is a unit of its own, factored directly, copy c on device c of a group of n_copies
 * devices (several split blocks may share a group: a device's split units are all of one copy and
 * are solved as one job, their chains together).  Whole blocks go to devices
 * longest-first by a time model of one MI355X (per-block chip time of each kernel class and the
 * block's chain alone).  Out: unit_device[b * n_copies + c] = the device index
 * of copy c of block b (-1: empty block); dev_ms (optional, n_dev entries) = the model's predicted
 * step of each device in ms.  Host-only (no GPU needed); deterministic.  Replaces the reference's
 * OpenMP schedule(dynamic) over blocks (scr/dbslmmfit.cpp:189-220). */
int dbslmm_shard_plan(int32_t num_block, const int32_t* m, int32_t n_ref, int32_t n_dev, int32_t n_copies,
                      int32_t* unit_device, double* dev_ms);
/* Shard plan of a problem (ABI 13): as dbslmm_shard_plan, for the route the problem's plans take
 * with these n_sigma sigmas (dbslmm_options.solver and the prior shift, as dbslmm_plan_run_multi
 * decides).  Factorisation route: dbslmm_shard_plan's model and units.  PCG route: whole blocks
 * only (every copy of a block on one device: one Krylov sequence serves the copies of a block
 * without large SNPs), longest first onto the least-loaded device by the PCG model (unpack + Gram
 * at the measured kernel rates, then per iteration the block's tiles and tile rows; a priori
 * iteration counts).  Outputs as dbslmm_shard_plan, n_copies = n_sigma.
 * Host-only; deterministic. */
int dbslmm_shard_plan_problem(const dbslmm_problem* p, const double* sigma_s, int32_t n_sigma, int32_t n_dev,
                              int32_t* unit_device, double* dev_ms);
/* A plan over ONE device's units of a shard plan (ABI 10), on a single-device context: the same
 * problem as dbslmm_plan_create (the whole .bed image and CSR arrays), solving only the units with
 * unit_device[b * n_copies + c] == device_index (its split units -- all of one h2f copy -- as one
 * job on a context of its own on the same GPU, so they run beside the device's whole blocks).  run_multi / download / variance write only
 * those units' entries of the caller's full-size arrays; everything else is left untouched, so
 * one process per GPU (bench.py under torch.distributed) solves its part and gathers the rest.
 * Run it with n_sigma == n_copies (otherwise a split block is solved whole by the device of its
 * copy 0). */
int dbslmm_plan_create_units(dbslmm_ctx* ctx, const dbslmm_problem* p, int32_t n_copies,
                             const int32_t* unit_device, int32_t device_index, dbslmm_plan** out);
/* Devices a context drives (1 for dbslmm_ctx_create). */
int dbslmm_ctx_num_devices(const dbslmm_ctx* ctx);
/* block_device[b] (num_block entries) = the device index (0 .. n_dev-1, in device_ids order) that
 * solves block b (its h2f copy 0 when the shard plan split its copies), -1 for an empty block (or,
 * on a units plan, a block none of whose units it solves); all 0 on a single-device context. */
int dbslmm_plan_shard_info(const dbslmm_plan* plan, int32_t* block_device);
void dbslmm_ctx_destroy(dbslmm_ctx* ctx);
const char* dbslmm_last_error(const dbslmm_ctx* ctx);
/* Keep a device copy of the caller's .bed image on the context (staged upload through pinned
 * buffers): dbslmm_bed_maf and dbslmm_plan_create calls that pass the same host range (bed,
 * bed_len) then read it instead of uploading again -- the reference reads the .bed once for the
 * MAF pass (IO::readBim, dtpr.cpp:93-102) and again per block in calcBlock (dbslmmfit.cpp:
 * 384-387).  The cached image is matched by host pointer and length only: the caller must not
 * modify the buffer, or free it and pass a new one at the same address, while it is cached
 * (call this again, or with bed == NULL, after any change).  A plan created from the cached image
 * reads it in place (no second device copy) and keeps it alive until the plan is destroyed, even
 * if the context releases or replaces it.  bed == NULL releases the context's reference.  A
 * multi-device context ignores the call (each device holds only its shard's rows). */
int dbslmm_ctx_cache_bed(dbslmm_ctx* ctx, const uint8_t* bed, int64_t bed_len);
/* dbslmm_ctx_cache_bed with the image read from an open file descriptor (pread straight into the
 * pinned staging buffers: the caller's pages of the file are never touched, so a caller that maps
 * the file pays no page faults and no page-table teardown for it).  `key` -- typically the
 * caller's mmap of the same file, never dereferenced here -- identifies the image: dbslmm_bed_maf
 * and dbslmm_plan_create calls that pass (key, bed_len) as their .bed read the cached copy.  The
 * file must not change while cached.  (ABI 8; the dbslmm CLI uses it.) */
int dbslmm_ctx_cache_bed_fd(dbslmm_ctx* ctx, int fd, int64_t bed_len, const uint8_t* key);

/* DBSLMMFIT::est replacement: upload, solve, download, free.  beta_s has s_ptr[num_block]
 * entries, beta_l l_ptr[num_block] (ignored when l_ptr == NULL); block_status (optional) has
 * num_block entries.  Blocking. */
int dbslmm_est(dbslmm_ctx* ctx, const dbslmm_problem* p, double* beta_s, double* beta_l,
               int32_t* block_status);

/* Split form.  plan_create copies the .bed image and block metadata into HBM and sizes the
 * workspace; plan_run enqueues the three kernels on the context's stream (asynchronous);
 * plan_sync waits; plan_download copies beta / status to the caller. */
int dbslmm_plan_create(dbslmm_ctx* ctx, const dbslmm_problem* p, dbslmm_plan** out);
int dbslmm_plan_run(dbslmm_plan* plan);
int dbslmm_plan_sync(dbslmm_plan* plan);
int dbslmm_plan_download(dbslmm_plan* plan, double* beta_s, double* beta_l, int32_t* block_status);
/* h2f tuning (replaces the three dbslmm runs of software/DBSLMM.R:204-219, -h = h2 * h2f):
 * one unpack + Gram, then for each sigma_s[i] one factorisation + solve; outputs are
 * n_sigma consecutive slices: beta_s[i * n_s ..], beta_l[i * n_l ..], block_status[i * num_block ..]
 * (NULL skips).  Synchronous.  The plan's own sigma_s is unchanged. */
int dbslmm_plan_run_multi(dbslmm_plan* plan, const double* sigma_s, int32_t n_sigma,
                          double* beta_s, double* beta_l, int32_t* block_status);

/* Change sigma_s (h2f tuning, software/DBSLMM.R:205-219) without re-uploading. */
int dbslmm_plan_set_sigma(dbslmm_plan* plan, double sigma_s);
void dbslmm_plan_destroy(dbslmm_plan* plan);

/* Kernel timing (HIP events recorded around each launch on the plan's stream).  Enable before
 * plan_run; after plan_sync, ms_out[k] = average duration in ms of kernel k over the runs since
 * enabling, launches_out = number of runs averaged. */
int dbslmm_plan_enable_timing(dbslmm_plan* plan, int enable);
int dbslmm_plan_kernel_ms(dbslmm_plan* plan, double* ms_out /*[DBSLMM_K_COUNT]*/, int32_t* launches_out);

/* Workload figures of the plan (for rooflines): [0] SNPs, [1] packed bytes read by the unpack,
 * [2] Gram operand (2-bit dosage code) bytes written by the unpack, [3] Gram ops (2 per MAC, algorithmic
 * sum_b n_ref*m_b*(m_b+1)), [4] Gram ops as executed on padded tiles, [5] Cholesky+solve fp64
 * flops of the large blocks (sum_b m_b^3/3 + 2 m_b^2), [6] non-empty blocks, [7] gram tiles,
 * [8] the same fp64 flops for the small blocks, [9] large blocks, [10] the same fp64 flops for
 * the tiled blocks, [11] tiled blocks, [12] launches of the tiled sequence per run, [13] bytes of
 * the factor read by one substitution launch over the tiled blocks (64-row tiles), [14] Chebyshev
 * iterations of the latest run_multi (0: none; with CG their cap), [15] its base copy (-1: none),
 * [16] factor bytes its h2f passes read (CG: each tiled block's own iteration count),
 * [17] 1 when the latest run took the PCG route, [18] its iterations (the slowest block),
 * [19] the lower-triangle LD matrix bytes the chip-wide PCG kernels streamed in that run (in their
 * storage: uint16 integer Gram / fp64 Sigma; every block times its own iterations), [20] their
 * partial-sum bytes (written + read once), [21] the same matrix bytes of the blocks
 * dbslmm_pcg_block solved whole (ABI 14; before: per-iteration figures). */
#define DBSLMM_WORKLOAD_LEN 22
int dbslmm_plan_workload(const dbslmm_plan* plan, double* out /*[DBSLMM_WORKLOAD_LEN]*/);
/* PCG iterations of each block in the latest run (ABI 13): iters[b] (num_block entries) = the
 * iterations block b ran before its every copy met the stopping rule (pcg_maxit at the cap), 0 for
 * empty blocks and after a run on the factorisation route.  Waits for the run. */
int dbslmm_plan_block_iters(dbslmm_plan* plan, int32_t* iters);

/* Diagnostics (parity tests): after plan_sync, the working matrix of block `block` (original
 * block id) in factorisation copy `copy`: ld x ld fp64, row-major, ld = *ld_out (out == NULL:
 * only ld).  Layout: rows / columns [small | large | z row m | padding];
 * after a debug_stop = 1 run the lower triangle (i < m, j <= i) holds Sigma (no 1/(sigma_s n)
 * shift); after a full run of a block on the multi-workgroup path (m >= tiled_min) the strict
 * lower triangle holds L (M = L L^T), row m holds y = L^{-1} z, and each 64 x 64 diagonal tile's
 * diagonal and upper triangle hold its inverse transposed.  Synchronous.  (ABI 9) */
int dbslmm_plan_block_matrix(dbslmm_plan* plan, int32_t block, int32_t copy, double* out,
                             int32_t* ld_out);

/* Test-set variance (the `diags` matrix DBSLMMFIT::est saves to variance.txt,
 * scr/dbslmmfit.cpp:116,191-214,242; calcBlock :366-626 with calc_nt_by_nt_matrix,
 * scr/calc_asymptotic_variance.cpp:22-137).  The test panel is a PLINK .bed image of n_total
 * individuals; indicator[0..n_total) selects the test individuals (nonzero; readSNPIm,
 * dtpr.cpp:285-364); s_pos / l_pos give each small / large SNP of the plan (same order and
 * length as the problem's s_pos / l_pos, l_pos NULL when the plan has no large SNPs) its row
 * in the test .bed (calcBlock's positional test_info_s_block[i].pos).
 */
typedef struct dbslmm_test_panel {
    const uint8_t* bed;
    int64_t bed_len;
    int32_t n_total;
    const int32_t* indicator;
    const int32_t* s_pos;
    const int32_t* l_pos;
} dbslmm_test_panel;

/* After plan_run / plan_run_multi (uses the factorisation of the most recent sigma_s):
 * diags is n_test x num_block column-major, n_test = number of indicator entries equal to 1;
 * column b = diag(X_l var_bl X_l^T + X_s var_bs X_s^T) of block b, zeros for a block without
 * SNPs, NaN for a block whose status is NOT_PD / MONOMORPHIC.  Synchronous; host buffers.
 * n_test_out (optional) receives n_test. */
int dbslmm_plan_variance(dbslmm_plan* plan, const dbslmm_test_panel* test, double* diags,
                         int32_t* n_test_out);

/* MAF pass: maf[r] for every bed row r < n_snp (readSNPIm with an all-ones indicator). */
int dbslmm_bed_maf(dbslmm_ctx* ctx, const uint8_t* bed, int64_t bed_len, int32_t n_ref,
                   int64_t n_snp, double* maf);

/* readSNPIm + nomalizeVec for rows pos[0..n_rows): out is n_ref x n_rows column-major fp64
 * (column j = standardised dosages of bed row pos[j]); maf (optional) n_rows entries. */
int dbslmm_read_snp_std(dbslmm_ctx* ctx, const uint8_t* bed, int64_t bed_len, int32_t n_ref,
                        const int32_t* pos, int32_t n_rows, double* out, double* maf);

/* External-validation R^2 terms: the per-block loop of the `valid` tool (replaces the
 * Armadillo products of scr/validate.cpp:221-257).  Block b owns .bed rows pos[ptr[b]..ptr[b+1])
 * with weights z1 (DBSLMM beta) and z2 (external z):
 *   nume[b] = z1 . z2,   deno[b] = z1^T (X^T X / n_ref) z1 = |X z1|^2 / n_ref
 * X = the nomalizeVec-standardised reference genotypes (N-1 sd, missing calls at the mean);
 * a monomorphic SNP gives NaN, as the reference's 0/0 column.  Synchronous; host buffers. */
int dbslmm_valid_blocks(dbslmm_ctx* ctx, const uint8_t* bed, int64_t bed_len, int32_t n_ref,
                        int32_t num_block, const int64_t* ptr, const int32_t* pos,
                        const double* z1, const double* z2, double* nume, double* deno);

#ifdef __cplusplus
}
#endif
#endif /* DBSLMM_HIP_H_ */
