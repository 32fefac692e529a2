// multi.hip -- multi-GPU contexts and plans (included at the end of plan.hip: same translation
// unit, so the single-device plan functions are called directly).
//
// The reference parallelises only over LD blocks (OpenMP schedule(dynamic) over batches of 60,
// scr/dbslmmfit.cpp:191-220): blocks are independent, so a multi-GPU solve needs no exchange during
// compute.  The unit of work here is an (LD block, h2f copy) pair -- the reference itself runs the
// h2f solves as independent dbslmm processes (software/DBSLMM.R:204-219):
//   1. dbslmm_shard_plan assigns the units to devices with a time model of one device (below):
//      a block's h2f copies stay together (one Gram, one factorisation, Chebyshev iterations for the
//      other copies on that factor) unless its dependency chain alone exceeds the fair share of the
//      step; then each copy is a unit of its own, factored directly on a different device, so the
//      largest blocks' chains run side by side instead of bounding the step;
//   2. a plan over a device's units is a set of JOBS on that device: one plan over its whole blocks
//      (all copies) plus one single-copy plan per split unit, each on its own context (streams) so
//      they run concurrently; the sub-problems carry COMPACT .bed images holding only their rows;
//   3. every call (run / run_multi / sync / download / variance / timing) fans out over the jobs,
//      one host thread each, and scatters the job outputs into the caller's arrays (beta, status,
//      variance columns) in the original order -- the only "exchange", straight from each device's
//      HBM to the caller's host buffers.  (The ABI's outputs are host memory, so a device-side gather
//      over xGMI before the copy-out would only add a hop)
// A multi-device context (dbslmm_ctx_create_multi) builds the jobs of every device;
// dbslmm_plan_create_units builds those of one device on a single-device context (one process per
// GPU: bench.py under torch.distributed, whose ranks gather the betas with RCCL).
#include <thread>

// ---------------------------------------------------------------- time model of one device
// Calibrated on config 4 (1M SNPs x 10k): chip-time of each kernel class from a
// serialised SQ_WAVE_CYCLES pass (round 4: trailing 13.2, substitutions 12.0, panels 3.2, Gram 2.9,
// regions 1.75, unpack 1.4, chol_large 1.0 chip-ms) over its algorithmic work, the Gram's rate by
// block size from the uniform-block probes (profiles/r05/gram), the block chains from the 9.6k-SNP
// block alone (tools/micro/tchol_alone.py: 14.7 ms); the remaining constants (busy fraction, chain
// drags, pipeline rates, download) fitted to the round-5 one-GPU rehearsal (bench.py --predict
// 2,4,8: 14 per-device steps, profiles/r05/shard/README).
namespace shard {
constexpr double kUnpackBps = 3.1e12;       // unpack: packed + operand bytes per second (alone)
constexpr double kGramOpsSmall = 1.7e15;    // Gram ops (2 per MAC) per second, m <= 600 ...
constexpr double kGramOpsBig = 3.4e15;      // ... m >= 4096 (log-linear between)
constexpr double kTrailFlops = 62e12;       // tiled factorisation bulk (trailing update)
constexpr double kPanelFlops = 68e12;       // panels: 2 x 128 x m^2 flops per block
constexpr double kRegionChipUs = 0.17;      // regions: chip-us per 128 columns (86 us on half a CU)
constexpr double kCholLargeFlops = 2e12;    // single-workgroup blocks (latency-bound)
constexpr double kSubBps = 4.3e12;          // substitution passes: factor bytes per second
// factorisation chain per 128 columns of a block alone: 128 us up to 4000 SNPs, then growing with
// the far updates the chain's launches wait beside (+0.0107 us per SNP above 4000): one block alone,
// unpack to beta, 1.71 / 2.74 / 4.21 / 6.75 / 10.05 / 14.60 ms at 1.6k / 2.6k / 4k / 5.5k / 7.5k /
// 9.6k SNPs (profiles/r05/chain/alone_by_size.txt)
constexpr double kChainRegionUs = 128.0, kChainRegionGrow = 0.0107, kChainRegionKnee = 4000.0;
constexpr double kChainSubUs = 4.5;         // substitution chain per 64-row tile, per pass (in situ)
constexpr double kBusy = 0.9;               // fraction of the chip the overlapped phases keep busy
constexpr double kDragWhole = 0.63;         // a whole block's chain: slow-down per chip-ms beside it
constexpr double kDragSplit = 1.06;         // a split unit's chain (its own context, no priority)
// the device's phases in sequence: unpack + Gram of everything, then the factorisations, then the
// substitution passes (each group's passes wait for its factorisation), then the result download
constexpr double kFrontRate = 0.79, kFacRate = 1.39, kSubRate = 0.73;
constexpr double kDownloadMsPerM = 0.95;    // per million (SNP, h2f copy) results
constexpr int kH2fIters = 6;               // h2f {0.8, 1, 1.2} at cheb_tol 1e-9 by CG (dbslmm_cg_update:
                                            // 5.03 iterations per block byte-weighted, 6-7 for blocks with
                                            // large SNPs; Chebyshev's a priori count is 7).  6 against the
                                            // rates fitted before CG: the rehearsal's devices within
                                            // 21.5-22.1 (N = 4) / 15.0-15.8 ms (N = 8) where 5 left the
                                            // whole-block devices 1.1-1.3 ms behind (profiles/r05/cg)
constexpr int kTiledMin = 384;              // plan.hip kTiledMinDefault

struct Cost {
    double work = 0.0;    // chip-ms
    double chain = 0.0;   // ms: the block's dependency chain when it runs alone
    double front = 0.0, fac = 0.0, sub = 0.0;   // chip-ms of the unpack + Gram / factorisation / passes
    double results = 0.0;                       // (SNP, copy) results downloaded
};

static double gram_ops(double m) {
    if (m <= 600.0) return kGramOpsSmall;
    if (m >= 4096.0) return kGramOpsBig;
    return kGramOpsSmall + std::log(m / 600.0) / std::log(4096.0 / 600.0) * (kGramOpsBig - kGramOpsSmall);
}

// Block of m SNPs, `copies` h2f solves; direct = every copy factored (a split unit is one direct
// copy), else one factorisation + CG iterations for the other copies
static Cost block_cost(double m, double n_ref, int copies, bool direct) {
    Cost c;
    if (m <= 0) return c;
    const double kp = std::ceil(n_ref / 128.0) * 128.0;
    const double unpack = m * (std::ceil(n_ref / 4.0) + kp / 4.0) / kUnpackBps * 1e3;
    const double gram = n_ref * m * (m + 1.0) / gram_ops(m) * 1e3;
    const int nfac = direct ? copies : 1;
    const double T = std::ceil(m / 64.0);
    const double pass_bytes = T * (T + 1.0) / 2.0 * 64.0 * 64.0 * 8.0;
    const int passes = direct ? copies : 1 + (copies > 1 ? 2 * kH2fIters : 0);
    c.front = unpack + gram;
    c.results = m * copies;
    if (m >= kTiledMin) {
        c.fac = nfac * (m * m * m / 3.0 / kTrailFlops * 1e3 + 256.0 * m * m / kPanelFlops * 1e3 +
                        m / 128.0 * kRegionChipUs * 1e-3);
        c.sub = passes * pass_bytes / kSubBps * 1e3;
        const double region_us = kChainRegionUs + kChainRegionGrow * std::max(0.0, m - kChainRegionKnee);
        c.chain = gram + m / 128.0 * region_us * 1e-3 + (direct ? 1 : passes) * T * kChainSubUs * 1e-3;
    } else {
        c.fac = (direct ? copies : 1) * m * m * m / 3.0 / kCholLargeFlops * 1e3;
        c.chain = gram + m * 0.2e-3;   // ~0.2 us per column of the single-workgroup factorisation
    }
    c.work = c.front + c.fac + c.sub;
    return c;
}

// One device's load: total work, the longest whole-block chain of its main job, its split units
// (contexts of their own: on the shared hardware queues their chains run one after the other) and
// its phase totals.  Predicted step = the largest of work / busy, each kind of chain + drag x the
// other work, and the phases in sequence.
struct Dev {
    double work = 0.0, whole_chain = 0.0, whole_chain_work = 0.0, split_chain = 0.0, split_work = 0.0;
    double front = 0.0, fac = 0.0, sub = 0.0, results = 0.0;
    int n_split = 0;
    double time() const {
        double t = work / kBusy;
        if (whole_chain > 0) t = std::max(t, whole_chain + kDragWhole * std::max(0.0, work - whole_chain_work));
        if (split_chain > 0) t = std::max(t, split_chain + kDragSplit * std::max(0.0, work - split_work));
        return std::max(t, front / kFrontRate + fac / kFacRate + sub / kSubRate + kDownloadMsPerM * results * 1e-6);
    }
    void add(const Cost& k, bool split) {
        work += k.work;
        front += k.front;
        fac += k.fac;
        sub += k.sub;
        results += k.results;
        if (split) {
            // a device's split units share one h2f copy (plan_units) and so one job: their chains
            // advance together in the same launches, each slowed by the others' work (the drag)
            if (k.chain > split_chain) {
                split_chain = k.chain;
                split_work = k.work;
            }
            ++n_split;
        } else if (k.chain > whole_chain) {
            whole_chain = k.chain;
            whole_chain_work = k.work;
        }
    }
};

// Units -> devices.  unit_device[b * K + c] (K = copies per run) = device of copy c of block b, -1
// for an empty block; dev_ms[d] = predicted step of device d.  Deterministic.
static void plan_units(int32_t nb, const int32_t* m, int32_t n_ref, int32_t G, int32_t K,
                       std::vector<int32_t>& unit_device, std::vector<double>& dev_ms) {
    K = std::max(1, K);
    unit_device.assign(static_cast<size_t>(nb) * K, -1);
    dev_ms.assign(G, 0.0);
    std::vector<char> split(nb, 0);
    std::vector<Cost> whole(nb), unit(nb);
    double total = 0.0;
    for (int b = 0; b < nb; ++b) {
        whole[b] = block_cost(m[b], n_ref, K, false);
        unit[b] = block_cost(m[b], n_ref, 1, true);
        total += whole[b].work;
    }
    // Split the h2f copies of a block (copy c on device t K + c of a K-device group t) when its whole
    // chain exceeds both the fair share of the step and the chains already decided; longest chain
    // first.  A new group while K devices remain; after that a split block joins the group whose
    // devices' predicted step grows least, if that beats its whole chain: the units of one copy on
    // one device form ONE job (one plan, one launch sequence), so their chains run together --
    // split units of different copies on one device would be separate jobs sharing the hardware
    // queues, their chains one after the other, which the groups rule out.  Every split adds its
    // extra factorisations to the total.
    std::vector<int32_t> byc;
    for (int b = 0; b < nb; ++b)
        if (m[b] > 0) byc.push_back(b);
    std::stable_sort(byc.begin(), byc.end(), [&](int32_t x, int32_t y) { return whole[x].chain > whole[y].chain; });
    std::vector<Dev> dev(G);
    int n_grp = 0;
    double bound = 0.0;
    auto place = [&](int32_t b, int t) {
        for (int c = 0; c < K; ++c) {
            dev[t * K + c].add(unit[b], true);
            unit_device[static_cast<size_t>(b) * K + c] = t * K + c;
        }
        split[b] = 1;
        total += K * unit[b].work - whole[b].work;
    };
    for (int32_t b : byc) {
        const double share = total / (kBusy * G);
        if (whole[b].chain <= std::max(share, bound)) break;
        if (K == 1 || unit[b].chain >= whole[b].chain) {
            bound = std::max(bound, whole[b].chain);
            continue;
        }
        if ((n_grp + 1) * K <= G) {
            place(b, n_grp++);
            bound = std::max(bound, unit[b].chain);
            continue;
        }
        int best = -1;
        double bt = 0.0;
        for (int t = 0; t < n_grp; ++t) {
            double v = 0.0;
            for (int c = 0; c < K; ++c) {
                Dev x = dev[t * K + c];
                x.add(unit[b], true);
                v = std::max(v, x.time());
            }
            if (best < 0 || v < bt - 1e-12) { best = t; bt = v; }
        }
        if (best >= 0 && bt < whole[b].chain) {
            place(b, best);
            bound = std::max(bound, bt);
        } else {
            bound = std::max(bound, whole[b].chain);
        }
    }
    // whole blocks: LPT by the predicted device step, longest first
    std::vector<int32_t> rest;
    for (int32_t b : byc)
        if (!split[b]) rest.push_back(b);
    std::stable_sort(rest.begin(), rest.end(), [&](int32_t x, int32_t y) {
        return std::max(whole[x].work / kBusy, whole[x].chain) > std::max(whole[y].work / kBusy, whole[y].chain);
    });
    for (int32_t b : rest) {
        int best = -1;
        double bt = 0.0;
        for (int d = 0; d < G; ++d) {
            Dev t = dev[d];
            t.add(whole[b], false);
            const double v = t.time();
            if (best < 0 || v < bt - 1e-12) { best = d; bt = v; }
        }
        dev[best].add(whole[b], false);
        for (int c = 0; c < K; ++c) unit_device[static_cast<size_t>(b) * K + c] = best;
    }
    for (int d = 0; d < G; ++d) dev_ms[d] = dev[d].time();
}

// ---------------------------------------------------------------- time model, PCG route
// On the PCG route (pcg.hip) a device runs one sequence: unpack + Gram of its blocks, then two
// concurrent paths -- dbslmm_pcg_block solving its blocks of <= 8 tile rows whole (one workgroup per
// Krylov sequence: its time is the larger of the chip's throughput over all of them, the longest
// sequence on one CU, and the sequences packed onto the CUs) and the chip-wide iterations of the
// others (per tile and per tile row and copy column, plus a floor per iteration: three dependent
// launches) -- then the result download.  No block needs splitting: the largest (9.7k SNPs) is
// ~1 ms of work.  Rates fitted to the round-6 one-GPU rehearsals of configs 3-5 at N = 1, 2, 4, 8
// (tools/fit_shard_model2.py, the model's own structure; 45 devices), iteration counts a priori
// (pcg_iters_model), DESIGN.md section 6.
constexpr double kPcgUnpackMs0 = 0.0102, kPcgUnpackBps = 4.581e12;    // dwordx4 unpack
constexpr double kPcgGramMs0 = 0.0840;                               // Gram launches
constexpr double kPcgGramOpsHuge = 3.379e15, kPcgGramOpsBig = 1.508e15;   // 256- / 128-tile kernels
constexpr double kPcgFusedQuadNs = 1.502;    // dbslmm_pcg_block, chip throughput: per 64 x 64 quadrant and iteration
constexpr double kPcgSeqQuadUs = 0.2594;     // ... one sequence on its CU: per quadrant and iteration
constexpr double kPcgCUs = 256.0;            // (the sequences packed onto the CUs)
constexpr double kPcgTileNs = 12.35;         // chip-wide product: per 128 x 128 tile and iteration (+50 % per extra column)
constexpr double kPcgRowNs = 1.21;            // rows + update: per tile row, copy column and iteration
constexpr double kPcgIterFloorUs = 20.37;    // per chip-wide iteration (launch chain)
constexpr double kPcgShare = 0.741;          // both paths at once: this share of their summed times
constexpr double kPcgRunMs = 0.0692;         // per run: memsets, init, final, read-back, host
constexpr double kPcgDownloadMsPerM = 0.753; // per million (SNP, copy) results downloaded + scattered
constexpr int kPcgFusedTb = 8;               // pcg::kFTb

// a priori iterations of a block at relative tolerance tol: CG's bound at kappa = 1 + 10 /
// (d + 1 - tau) (fitted to the measured counts: 15.7 / 13.9 / 12.9 mean at d = 10 / 16.7 / 20),
// + 2 for the outlying eigenvalues of large SNPs
static int pcg_iters_model(double dmin, double tau, double tol, bool large) {
    const double kap = 1.0 + 10.0 / std::max(1e-3, dmin + 1.0 - tau);
    const double q = (std::sqrt(kap) - 1.0) / (std::sqrt(kap) + 1.0);
    return static_cast<int>(std::ceil(std::log(2.0 / tol) / -std::log(q))) + (large ? 2 : 0);
}

// a device's PCG-route work, accumulated block by block
struct PcgDev {
    double front = 0.0, fq = 0.0, seq_max = 0.0, chip = 0.0, results = 0.0;   // fq: quadrant-iterations
    int chip_iters = 0;
    double time() const {
        if (front == 0.0 && results == 0.0) return 0.0;
        const double fused = std::max({fq * kPcgFusedQuadNs * 1e-6, seq_max * kPcgSeqQuadUs * 1e-3,
                                       fq * kPcgSeqQuadUs * 1e-3 / kPcgCUs});
        const double p = std::max({chip, fused, kPcgShare * (chip + fused)}) + chip_iters * kPcgIterFloorUs * 1e-3;
        return kPcgUnpackMs0 + kPcgGramMs0 + front + p + kPcgRunMs + kPcgDownloadMsPerM * results * 1e-6;
    }
};
struct PcgCost {
    double front = 0.0, fq = 0.0, seq = 0.0, chip = 0.0, results = 0.0;   // seq: one sequence's quadrant-iterations
    int chip_iters = 0;
    double ms() const { return front + fq * kPcgFusedQuadNs * 1e-6 + chip; }   // (the ordering key)
};
static PcgCost pcg_block_cost(double m, double ml, double n_ref, int copies, int iters) {
    PcgCost c;
    if (m <= 0) return c;
    const double kp = std::ceil(n_ref / 128.0) * 128.0;
    const double huge_min = kp >= 4096 ? 384.0 : 768.0;
    c.front = m * (std::ceil(n_ref / 4.0) + kp / 4.0) / kPcgUnpackBps * 1e3 +
              n_ref * m * (m + 1.0) / (m >= huge_min ? kPcgGramOpsHuge : kPcgGramOpsBig) * 1e3;
    const double Tb = std::ceil(m / 128.0), Q = std::ceil(m / 64.0);
    const int nc = (copies > 1 && ml > 0) ? copies : 1;   // multi-shift: one column without large SNPs
    if (Tb <= kPcgFusedTb) {   // one sequence per product column, each its own workgroup
        c.seq = iters * Q * (Q + 1.0) / 2.0;
        c.fq = nc * c.seq;
    } else {
        c.chip = iters * (Tb * (Tb + 1.0) / 2.0 * (1.0 + 0.5 * (nc - 1)) * kPcgTileNs + Tb * nc * kPcgRowNs) * 1e-6;
        c.chip_iters = iters;
    }
    c.results = m * copies;
    return c;
}

// Whole blocks -> devices, longest first onto the device whose predicted step grows least.
static void plan_units_pcg(int32_t nb, const int32_t* m, const int32_t* ml, int32_t n_ref, int32_t G, int32_t K,
                           const std::vector<int>& iters, std::vector<int32_t>& unit_device,
                           std::vector<double>& dev_ms) {
    K = std::max(1, K);
    unit_device.assign(static_cast<size_t>(nb) * K, -1);
    std::vector<PcgCost> cost(nb);
    std::vector<int32_t> order;
    for (int b = 0; b < nb; ++b) {
        cost[b] = pcg_block_cost(m[b], ml ? ml[b] : 0, n_ref, K, iters[b]);
        if (m[b] > 0) order.push_back(b);
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return cost[x].ms() > cost[y].ms(); });
    std::vector<PcgDev> dev(G);
    auto with = [&](PcgDev d, const PcgCost& c) {
        d.front += c.front;
        d.fq += c.fq;
        d.seq_max = std::max(d.seq_max, c.seq);
        d.chip += c.chip;
        d.results += c.results;
        d.chip_iters = std::max(d.chip_iters, c.chip_iters);
        return d;
    };
    for (int32_t b : order) {
        int best = 0;
        double bt = 0.0;
        for (int d = 0; d < G; ++d) {
            const double v = with(dev[d], cost[b]).time();
            if (d == 0 || v < bt - 1e-12) { best = d; bt = v; }
        }
        dev[best] = with(dev[best], cost[b]);
        for (int c = 0; c < K; ++c) unit_device[static_cast<size_t>(b) * K + c] = best;
    }
    dev_ms.assign(G, 0.0);
    for (int d = 0; d < G; ++d) dev_ms[d] = dev[d].time();
}
}  // namespace shard

// Does a plan of this problem take the PCG route for these sigmas?  (plan.hip pcg_route at the
// problem level: the same options, tau, large-SNP and prior-shift rules.)
static bool problem_pcg_route(const dbslmm_problem* pr, const double* sig, int n, bool has_large) {
    const dbslmm_options* o = pr->opts;
    const int solver = o ? o->solver : 0;
    if (solver == 1 || (o && o->debug_stop) || n < 1) return false;
    if (n > pcg::kMaxNC || !(pr->tau > 0.0 && pr->tau <= 1.0) || (pr->tau >= 1.0 && has_large)) return false;
    if (solver == 2) return true;
    for (int c = 0; c < n; ++c)
        if (1.0 / (sig[c] * static_cast<double>(pr->n_obs)) < kPcgDmin) return false;
    return true;
}

// The shard plan of a problem: the PCG model when its runs take the PCG route, else the
// factorisation model (shard::plan_units).  m / ml: SNPs / large SNPs per block.
static void plan_problem(const dbslmm_problem* pr, const double* sig, int n, int32_t G,
                         const std::vector<int32_t>& m, const std::vector<int32_t>& ml,
                         std::vector<int32_t>& ud, std::vector<double>& dev_ms) {
    bool has_large = false;
    for (int32_t x : ml) has_large |= x > 0;
    if (!problem_pcg_route(pr, sig, n, has_large)) {
        shard::plan_units(pr->num_block, m.data(), pr->n_ref, G, n, ud, dev_ms);
        return;
    }
    double dmin = INFINITY;
    for (int c = 0; c < n; ++c) dmin = std::min(dmin, 1.0 / (sig[c] * static_cast<double>(pr->n_obs)));
    const double tol = pr->opts && pr->opts->pcg_tol > 0.0 ? std::max(1e-15, pr->opts->pcg_tol) : 1e-12;
    std::vector<int> it(pr->num_block);
    for (int b = 0; b < pr->num_block; ++b) it[b] = shard::pcg_iters_model(dmin, pr->tau, tol, ml[b] > 0);
    shard::plan_units_pcg(pr->num_block, m.data(), ml.data(), pr->n_ref, G, n, it, ud, dev_ms);
}

// SNPs and large SNPs per block of a problem (checked CSR offsets)
static int block_sizes(dbslmm_ctx* ctx, const dbslmm_problem* pr, std::vector<int32_t>& m, std::vector<int32_t>& ml) {
    const bool has_l = pr->l_ptr != nullptr;
    m.assign(pr->num_block, 0);
    ml.assign(pr->num_block, 0);
    for (int b = 0; b < pr->num_block; ++b) {
        const int64_t ms = pr->s_ptr[b + 1] - pr->s_ptr[b], l = has_l ? pr->l_ptr[b + 1] - pr->l_ptr[b] : 0;
        if (ms < 0 || l < 0) {
            if (ctx) ctx->err = "CSR offsets not monotone";
            return DBSLMM_E_ARG;
        }
        m[b] = static_cast<int32_t>(ms + l);
        ml[b] = static_cast<int32_t>(l);
    }
    return DBSLMM_OK;
}

// ---------------------------------------------------------------- jobs
// Run f(i) for every job index on its own host thread; the first failing rc wins and its job's
// context message is copied to the parent context.
template <typename F>
static int fan_out(dbslmm_plan* p, F f) {
    auto& S = p->mp->shards;
    const int n = static_cast<int>(S.size());
    std::vector<int> rc(n, DBSLMM_OK);
    if (n == 1) {
        rc[0] = f(0);   // one job (a units plan of one device): no thread to spawn per call
    } else {
        std::vector<std::thread> th;
        th.reserve(n);
        for (int i = 0; i < n; ++i) th.emplace_back([&, i] { rc[i] = f(i); });
        for (auto& t : th) t.join();
    }
    for (int i = 0; i < n; ++i)
        if (rc[i] != DBSLMM_OK) {
            dbslmm_ctx* jc = S[i].plan ? S[i].plan->ctx : S[i].ctx;
            p->ctx->err = "device " + std::to_string(jc ? jc->device : -1) + ": " + (jc ? jc->err : std::string("?"));
            return rc[i];
        }
    return DBSLMM_OK;
}

// The jobs of the devices in `devs` (device index d -> context dev_ctx[d]) for a shard plan.
static int mp_build(dbslmm_ctx* ctx, const dbslmm_problem* pr, int32_t K, const std::vector<int32_t>& unit_device,
                    const std::vector<int>& devs, const std::vector<dbslmm_ctx*>& dev_ctx, bool partial,
                    dbslmm_plan** out) {
    ARG_CHECK(ctx, pr && out, "null problem/out");
    *out = nullptr;
    ARG_CHECK(ctx, pr->bed && pr->n_ref > 1 && pr->n_obs > 0 && pr->num_block >= 0, "bad sizes");
    ARG_CHECK(ctx, pr->s_ptr && (pr->s_ptr[pr->num_block] == 0 || (pr->s_pos && pr->z_s)), "bad small CSR");
    const bool has_l = pr->l_ptr != nullptr;
    if (has_l) ARG_CHECK(ctx, pr->l_ptr[pr->num_block] == 0 || (pr->l_pos && pr->z_l), "bad large CSR");
    const int64_t bps = pr->n_ref / 4 + (pr->n_ref % 4 ? 1 : 0);
    ARG_CHECK(ctx, pr->bed_len >= 3 + bps, "bed image shorter than one SNP row");
    const int64_t n_rows = (pr->bed_len - 3) / bps;
    auto* p = new dbslmm_plan();
    p->ctx = ctx;
    p->n_ref = pr->n_ref;
    p->n_obs = pr->n_obs;
    p->num_block = pr->num_block;
    p->sigma_s = pr->sigma_s;
    p->tau = pr->tau;
    p->n_s = pr->s_ptr[pr->num_block];
    p->n_l = has_l ? pr->l_ptr[pr->num_block] : 0;
    p->mp = new dbslmm_mplan();
    p->mp->n_copies = K;
    p->mp->partial = partial;
    p->mp->unit_device = unit_device;
    // jobs: per device its whole blocks (copy -1), then one job per h2f copy c holding the device's
    // split units of that copy (shard::plan_units gives a device split units of one copy only)
    auto& J = p->mp->shards;
    for (int d : devs) {
        DeviceShard main_job;
        main_job.device_index = d;
        main_job.ctx = dev_ctx[d];
        for (int b = 0; b < pr->num_block; ++b) {
            const int32_t* ud = unit_device.data() + static_cast<size_t>(b) * K;
            bool whole = ud[0] == d;
            for (int c = 1; c < K; ++c) whole &= ud[c] == d;
            if (whole) main_job.blocks.push_back(b);
        }
        J.push_back(std::move(main_job));
        for (int c = 0; c < K; ++c) {
            DeviceShard u;
            u.device_index = d;
            u.copy = c;
            for (int b = 0; b < pr->num_block; ++b) {
                const int32_t* ud = unit_device.data() + static_cast<size_t>(b) * K;
                bool whole = true;
                for (int e = 1; e < K; ++e) whole &= ud[e] == ud[0];
                if (!whole && ud[c] == d) u.blocks.push_back(b);
            }
            if (!u.blocks.empty()) J.push_back(std::move(u));
        }
    }
    // sub-problems with compact .bed images (rows renumbered in first-use order)
    struct Sub {
        std::vector<uint8_t> bed;
        std::vector<int64_t> s_ptr, l_ptr;
        std::vector<int32_t> s_pos, l_pos;
        std::vector<double> z_s, z_l;
        dbslmm_problem prob{};
    };
    std::vector<Sub> subs(J.size());
    for (size_t j = 0; j < J.size(); ++j) {
        DeviceShard& sh = J[j];
        Sub& su = subs[j];
        std::unordered_map<int32_t, int32_t> remap;
        std::vector<int32_t> rows;
        auto local = [&](int32_t r) -> int32_t {
            auto it = remap.find(r);
            if (it != remap.end()) return it->second;
            const int32_t k = static_cast<int32_t>(rows.size());
            remap.emplace(r, k);
            rows.push_back(r);
            return k;
        };
        su.s_ptr.push_back(0);
        su.l_ptr.push_back(0);
        for (int32_t b : sh.blocks) {
            for (int64_t i = pr->s_ptr[b]; i < pr->s_ptr[b + 1]; ++i) {
                const int32_t r = pr->s_pos[i];
                if (r < 0 || r >= n_rows) { ctx->err = "small SNP bed row out of range"; dbslmm_plan_destroy(p); return DBSLMM_E_ARG; }
                su.s_pos.push_back(local(r));
                su.z_s.push_back(pr->z_s[i]);
                sh.s_idx.push_back(i);
            }
            su.s_ptr.push_back(static_cast<int64_t>(su.s_pos.size()));
            if (has_l) {
                for (int64_t i = pr->l_ptr[b]; i < pr->l_ptr[b + 1]; ++i) {
                    const int32_t r = pr->l_pos[i];
                    if (r < 0 || r >= n_rows) { ctx->err = "large SNP bed row out of range"; dbslmm_plan_destroy(p); return DBSLMM_E_ARG; }
                    su.l_pos.push_back(local(r));
                    su.z_l.push_back(pr->z_l[i]);
                    sh.l_idx.push_back(i);
                }
                su.l_ptr.push_back(static_cast<int64_t>(su.l_pos.size()));
            }
        }
        su.bed.assign(3 + std::max<size_t>(1, rows.size()) * bps, 0);
        std::memcpy(su.bed.data(), pr->bed, 3);
        for (size_t k = 0; k < rows.size(); ++k)
            std::memcpy(su.bed.data() + 3 + k * bps, pr->bed + 3 + static_cast<int64_t>(rows[k]) * bps, bps);
        dbslmm_problem& q = su.prob;
        q.bed = su.bed.data();
        q.bed_len = static_cast<int64_t>(su.bed.size());
        q.n_ref = pr->n_ref;
        q.n_obs = pr->n_obs;
        q.sigma_s = pr->sigma_s;
        q.tau = pr->tau;
        q.num_block = static_cast<int32_t>(sh.blocks.size());
        q.s_ptr = su.s_ptr.data();
        q.s_pos = su.s_pos.data();
        q.z_s = su.z_s.data();
        if (has_l) {
            q.l_ptr = su.l_ptr.data();
            q.l_pos = su.l_pos.data();
            q.z_l = su.z_l.data();
        }
        q.opts = pr->opts;
    }
    // job plans, one host thread each; a split unit runs on a context of its own on its device
    // (own streams: it runs beside the device's other jobs, its chain on high-priority streams)
    const int rc = fan_out(p, [&](int j) -> int {
        DeviceShard& sh = J[j];
        if (sh.copy >= 0) {
            const int r = dbslmm_ctx_create(dev_ctx[sh.device_index]->device, &sh.own_ctx);
            if (r != DBSLMM_OK) return r;
            sh.ctx = sh.own_ctx;
        }
        if (sh.blocks.empty()) return DBSLMM_OK;   // an idle device (more devices than blocks)
        return dbslmm_plan_create(sh.ctx, &subs[j].prob, &sh.plan);
    });
    if (rc != DBSLMM_OK) { dbslmm_plan_destroy(p); return rc; }
    // jobs without blocks hold no plan: dropped
    J.erase(std::remove_if(J.begin(), J.end(), [](const DeviceShard& s) { return s.plan == nullptr; }), J.end());
    p->ran = false;
    *out = p;
    return DBSLMM_OK;
}

static int mp_create(dbslmm_ctx* ctx, const dbslmm_problem* pr, dbslmm_plan** out) {
    ARG_CHECK(ctx, pr && out && pr->s_ptr && pr->num_block >= 0, "null problem/out");
    std::vector<int32_t> m, ml;
    if (const int rc = block_sizes(ctx, pr, m, ml)) return rc;
    const int G = static_cast<int>(ctx->subs.size());
    const int32_t K = pr->opts && pr->opts->shard_copies > 1 ? pr->opts->shard_copies : 1;
    ARG_CHECK(ctx, K <= 64, "shard_copies must be <= 64");
    // the route is decided per run from its sigmas; the plan assumes K copies at the problem's sigma_s
    std::vector<double> sig(K, pr->sigma_s);
    std::vector<int32_t> ud;
    std::vector<double> dev_ms;
    plan_problem(pr, sig.data(), K, G, m, ml, ud, dev_ms);
    std::vector<int> devs(G);
    std::iota(devs.begin(), devs.end(), 0);
    return mp_build(ctx, pr, K, ud, devs, ctx->subs, false, out);
}

static void mp_destroy(dbslmm_plan* p) {
    for (DeviceShard& sh : p->mp->shards) {
        dbslmm_plan_destroy(sh.plan);
        dbslmm_ctx_destroy(sh.own_ctx);
    }
    delete p->mp;
    p->mp = nullptr;
}

// job j's plan copy holding the caller's h2f copy c in the last run (-1: none)
static int job_copy(const DeviceShard& sh, int c) {
    for (size_t k = 0; k < sh.run_copies.size(); ++k)
        if (sh.run_copies[k] == c) return static_cast<int>(k);
    return -1;
}

// beta / status of one solve, scattered from every job into the caller's arrays
static int mp_download(dbslmm_plan* p, int copy, double* beta_s, double* beta_l, int32_t* block_status) {
    auto& S = p->mp->shards;
    if (block_status && !p->mp->partial)
        for (int32_t b = 0; b < p->num_block; ++b) block_status[b] = DBSLMM_BLOCK_EMPTY;
    return fan_out(p, [&](int d) -> int {
        DeviceShard& sh = S[d];
        const int jc = job_copy(sh, copy);
        if (jc < 0) return DBSLMM_OK;
        std::vector<double> bs(sh.s_idx.size()), bl(sh.l_idx.size());
        std::vector<int32_t> st(sh.blocks.size());
        const int rc = download_copy(sh.plan, jc, bs.data(), bl.data(), st.data());
        if (rc != DBSLMM_OK) return rc;
        if (beta_s) for (size_t i = 0; i < bs.size(); ++i) beta_s[sh.s_idx[i]] = bs[i];
        if (beta_l) for (size_t i = 0; i < bl.size(); ++i) beta_l[sh.l_idx[i]] = bl[i];
        if (block_status) for (size_t i = 0; i < st.size(); ++i) block_status[sh.blocks[i]] = st[i];
        return DBSLMM_OK;
    });
}

// every solve of the last run (n = its sigmas), from every job in ONE pass: each job's copies come
// down in one pipelined download (download_copies) into its reused staging, then each copy is
// scattered into the caller's arrays at the caller's copy index (beta_s / beta_l / block_status:
// n consecutive arrays of n_s / n_l / num_block, as dbslmm_plan_run_multi's outputs)
static int mp_download_all(dbslmm_plan* p, int n, double* beta_s, double* beta_l, int32_t* block_status) {
    auto& S = p->mp->shards;
    if (block_status && !p->mp->partial)
        for (int64_t i = 0; i < static_cast<int64_t>(n) * p->num_block; ++i) block_status[i] = DBSLMM_BLOCK_EMPTY;
    return fan_out(p, [&](int d) -> int {
        DeviceShard& sh = S[d];
        const int nr = static_cast<int>(sh.run_copies.size());
        if (nr == 0) return DBSLMM_OK;
        const size_t ns = sh.s_idx.size(), nl = sh.l_idx.size(), nb = sh.blocks.size();
        if (sh.dl_s.size() < nr * ns) sh.dl_s.resize(nr * ns);
        if (sh.dl_l.size() < nr * nl) sh.dl_l.resize(nr * nl);
        if (sh.dl_st.size() < nr * nb) sh.dl_st.resize(nr * nb);
        const int rc = download_copies(sh.plan, 0, nr, sh.dl_s.data(), sh.dl_l.data(), sh.dl_st.data());
        if (rc != DBSLMM_OK) return rc;
        for (int k = 0; k < nr; ++k) {
            const int64_t c = sh.run_copies[k];
            if (c >= n) continue;
            const double* bs = sh.dl_s.data() + k * ns;
            const double* bl = sh.dl_l.data() + k * nl;
            const int32_t* st = sh.dl_st.data() + k * nb;
            if (beta_s) {
                double* o = beta_s + c * p->n_s;
                for (size_t i = 0; i < ns; ++i) o[sh.s_idx[i]] = bs[i];
            }
            if (beta_l) {
                double* o = beta_l + c * p->n_l;
                for (size_t i = 0; i < nl; ++i) o[sh.l_idx[i]] = bl[i];
            }
            if (block_status) {
                int32_t* o = block_status + c * p->num_block;
                for (size_t i = 0; i < nb; ++i) o[sh.blocks[i]] = st[i];
            }
        }
        return DBSLMM_OK;
    });
}

// n solves: with n == the plan's copies every job solves its own copies (a split unit: its copy
// alone, factored directly); otherwise a split block is solved whole by the job of its copy 0
static int mp_run(dbslmm_plan* p, const double* sigmas, int n, bool wait) {
    auto& S = p->mp->shards;
    const int K = p->mp->n_copies;
    const int rc = fan_out(p, [&](int d) -> int {
        DeviceShard& sh = S[d];
        sh.run_copies.clear();
        if (sh.copy >= 0 && n == K) {
            sh.run_copies.push_back(sh.copy);
        } else if (sh.copy <= 0) {
            for (int c = 0; c < n; ++c) sh.run_copies.push_back(c);
        } else {
            return DBSLMM_OK;     // another job solves this block's copies
        }
        std::vector<double> sg;
        for (int c : sh.run_copies) sg.push_back(sigmas[c]);
        int r = run_impl(sh.plan, true, sg.data(), static_cast<int>(sg.size()));
        if (r == DBSLMM_OK && wait) r = dbslmm_plan_sync(sh.plan);
        return r;
    });
    if (rc == DBSLMM_OK) {
        p->ran = true;
        p->stopped = false;
        p->var_copy = n - 1;
        p->sigma_run = sigmas[n - 1];
    }
    return rc;
}

static int mp_sync(dbslmm_plan* p) {
    auto& S = p->mp->shards;
    return fan_out(p, [&](int d) -> int { return S[d].run_copies.empty() ? DBSLMM_OK : dbslmm_plan_sync(S[d].plan); });
}

// per-block PCG iterations of the latest run, from every job (a block's max over its jobs)
static int mp_block_iters(dbslmm_plan* p, int32_t* iters) {
    auto& S = p->mp->shards;
    if (!p->mp->partial) std::fill(iters, iters + p->num_block, 0);
    std::vector<std::vector<int32_t>> sub(S.size());
    const int rc = fan_out(p, [&](int j) -> int {
        if (S[j].run_copies.empty()) return DBSLMM_OK;
        sub[j].assign(std::max<size_t>(1, S[j].blocks.size()), 0);
        return dbslmm_plan_block_iters(S[j].plan, sub[j].data());
    });
    if (rc != DBSLMM_OK) return rc;
    for (size_t j = 0; j < S.size(); ++j)
        for (size_t i = 0; i < S[j].blocks.size() && i < sub[j].size(); ++i) {
            int32_t& o = iters[S[j].blocks[i]];
            o = std::max(o, sub[j][i]);
        }
    return DBSLMM_OK;
}

static int mp_variance(dbslmm_plan* p, const dbslmm_test_panel* tp, double* diags, int32_t* n_test_out) {
    dbslmm_ctx* ctx = p->ctx;
    ARG_CHECK(ctx, tp && tp->indicator && tp->n_total > 0, "bad test panel");
    ARG_CHECK(ctx, p->n_s == 0 || tp->s_pos, "test panel s_pos missing");
    ARG_CHECK(ctx, p->n_l == 0 || tp->l_pos, "test panel l_pos missing");
    int32_t n_test = 0;
    for (int32_t i = 0; i < tp->n_total; ++i) n_test += tp->indicator[i] != 0;
    if (n_test_out) *n_test_out = n_test;
    if (n_test == 0 || p->num_block == 0) return DBSLMM_OK;
    ARG_CHECK(ctx, diags, "null diags");
    auto& S = p->mp->shards;
    if (!p->mp->partial) std::fill(diags, diags + static_cast<size_t>(n_test) * p->num_block, 0.0);
    // the jobs holding the last solve's factorisation (the caller's copy var_copy is their last)
    auto holds = [&](const DeviceShard& sh) { return !sh.run_copies.empty() && sh.run_copies.back() == p->var_copy; };
    // every job's pending single-sigma re-run (graph captures) first, drained, then the variances
    const int rc0 = fan_out(p, [&](int d) -> int {
        dbslmm_plan* q = S[d].plan;
        if (!holds(S[d]) || !q->cheb_pending_var) return DBSLMM_OK;
        const int r = variance_factor(q);
        return r == DBSLMM_OK ? dbslmm_plan_sync(q) : r;
    });
    if (rc0 != DBSLMM_OK) return rc0;
    return fan_out(p, [&](int d) -> int {
        DeviceShard& sh = S[d];
        if (!holds(sh)) return DBSLMM_OK;
        std::vector<int32_t> sp(sh.s_idx.size()), lp(sh.l_idx.size());
        for (size_t i = 0; i < sp.size(); ++i) sp[i] = tp->s_pos[sh.s_idx[i]];
        for (size_t i = 0; i < lp.size(); ++i) lp[i] = tp->l_pos[sh.l_idx[i]];
        dbslmm_test_panel t = *tp;
        t.s_pos = sp.data();
        t.l_pos = p->n_l ? lp.data() : nullptr;
        std::vector<double> dg(static_cast<size_t>(n_test) * sh.blocks.size());
        const int rc = dbslmm_plan_variance(sh.plan, &t, dg.data(), nullptr);
        if (rc != DBSLMM_OK) return rc;
        for (size_t j = 0; j < sh.blocks.size(); ++j)
            std::memcpy(diags + static_cast<size_t>(sh.blocks[j]) * n_test, dg.data() + j * n_test,
                        n_test * sizeof(double));
        return DBSLMM_OK;
    });
}

// MAF pass over contiguous row ranges, one per device.  A range [r0, r1) is handed over as the
// image starting at bed + r0 * bps: its first 3 bytes stand in for the magic (never read) and row
// r0 is its row 0, so no copy is needed.
static int mp_bed_maf(dbslmm_ctx* ctx, const uint8_t* bed, int32_t n_ref, int64_t n_snp, double* maf) {
    const int64_t bps = n_ref / 4 + (n_ref % 4 ? 1 : 0);
    const int G = static_cast<int>(ctx->subs.size());
    std::vector<int> rc(G, DBSLMM_OK);
    std::vector<std::thread> th;
    for (int d = 0; d < G; ++d)
        th.emplace_back([&, d] {
            const int64_t r0 = n_snp * d / G, r1 = n_snp * (d + 1) / G;
            if (r1 > r0) rc[d] = dbslmm_bed_maf(ctx->subs[d], bed + r0 * bps, 3 + (r1 - r0) * bps, n_ref, r1 - r0, maf + r0);
        });
    for (auto& t : th) t.join();
    for (int d = 0; d < G; ++d)
        if (rc[d] != DBSLMM_OK) {
            ctx->err = "device " + std::to_string(ctx->subs[d]->device) + ": " + ctx->subs[d]->err;
            return rc[d];
        }
    return DBSLMM_OK;
}

extern "C" {

int dbslmm_ctx_create_multi(int32_t n_dev, const int32_t* device_ids, dbslmm_ctx** out) {
    if (!out || n_dev <= 0 || !device_ids) return DBSLMM_E_ARG;
    *out = nullptr;
    if (n_dev == 1) return dbslmm_ctx_create(device_ids[0], out);
    auto* c = new dbslmm_ctx();
    c->device = -1;
    for (int i = 0; i < n_dev; ++i) {
        dbslmm_ctx* s = nullptr;
        const int rc = dbslmm_ctx_create(device_ids[i], &s);
        if (rc != DBSLMM_OK) {
            dbslmm_ctx_destroy(c);
            return rc;
        }
        c->subs.push_back(s);
    }
    *out = c;
    return DBSLMM_OK;
}

int dbslmm_ctx_num_devices(const dbslmm_ctx* ctx) {
    if (!ctx) return DBSLMM_E_ARG;
    return ctx->subs.empty() ? 1 : static_cast<int>(ctx->subs.size());
}

int dbslmm_plan_shard_info(const dbslmm_plan* p, int32_t* block_device) {
    if (!p || !block_device) return DBSLMM_E_ARG;
    if (!p->mp) {
        for (int32_t b = 0; b < p->num_block; ++b) block_device[b] = 0;
        return DBSLMM_OK;
    }
    const int K = p->mp->n_copies;
    for (int32_t b = 0; b < p->num_block; ++b) block_device[b] = -1;   // empty blocks
    for (const DeviceShard& sh : p->mp->shards)
        for (int32_t b : sh.blocks)
            if (sh.copy <= 0) block_device[b] = p->mp->unit_device[static_cast<size_t>(b) * K];
    return DBSLMM_OK;
}

int dbslmm_shard_plan(int32_t num_block, const int32_t* m, int32_t n_ref, int32_t n_dev, int32_t n_copies,
                      int32_t* unit_device, double* dev_ms) {
    if (num_block < 0 || (num_block > 0 && !m) || n_ref <= 1 || n_dev <= 0 || n_copies < 1 || n_copies > 64 ||
        !unit_device)
        return DBSLMM_E_ARG;
    for (int32_t b = 0; b < num_block; ++b)
        if (m[b] < 0) return DBSLMM_E_ARG;
    std::vector<int32_t> ud;
    std::vector<double> ms;
    shard::plan_units(num_block, m, n_ref, n_dev, n_copies, ud, ms);
    std::copy(ud.begin(), ud.end(), unit_device);
    if (dev_ms) std::copy(ms.begin(), ms.end(), dev_ms);
    return DBSLMM_OK;
}

int dbslmm_shard_plan_problem(const dbslmm_problem* pr, const double* sigma_s, int32_t n_sigma, int32_t n_dev,
                              int32_t* unit_device, double* dev_ms) {
    if (!pr || !pr->s_ptr || pr->num_block < 0 || !sigma_s || n_sigma < 1 || n_sigma > 64 || n_dev <= 0 ||
        !unit_device || pr->n_ref <= 1 || pr->n_obs <= 0)
        return DBSLMM_E_ARG;
    for (int c = 0; c < n_sigma; ++c)
        if (!(sigma_s[c] > 0.0)) return DBSLMM_E_ARG;
    std::vector<int32_t> m, ml;
    if (const int rc = block_sizes(nullptr, pr, m, ml)) return rc;
    std::vector<int32_t> ud;
    std::vector<double> ms;
    plan_problem(pr, sigma_s, n_sigma, n_dev, m, ml, ud, ms);
    std::copy(ud.begin(), ud.end(), unit_device);
    if (dev_ms) std::copy(ms.begin(), ms.end(), dev_ms);
    return DBSLMM_OK;
}

int dbslmm_plan_create_units(dbslmm_ctx* ctx, const dbslmm_problem* pr, int32_t n_copies, const int32_t* unit_device,
                             int32_t device_index, dbslmm_plan** out) {
    if (!ctx) return DBSLMM_E_ARG;
    ARG_CHECK(ctx, ctx->subs.empty(), "dbslmm_plan_create_units takes a single-device context");
    ARG_CHECK(ctx, pr && out && unit_device && n_copies >= 1 && n_copies <= 64 && device_index >= 0,
              "null problem/out/unit_device, or n_copies / device_index out of range");
    if (const int rc = ctx_ready(ctx)) return rc;
    ARG_CHECK(ctx, pr->num_block >= 0 && pr->s_ptr, "bad sizes");
    const bool has_l = pr->l_ptr != nullptr;
    std::vector<int32_t> ud(unit_device, unit_device + static_cast<size_t>(pr->num_block) * n_copies);
    for (int b = 0; b < pr->num_block; ++b) {
        const bool empty = pr->s_ptr[b + 1] == pr->s_ptr[b] && (!has_l || pr->l_ptr[b + 1] == pr->l_ptr[b]);
        for (int c = 0; c < n_copies; ++c) {
            const int32_t d = ud[static_cast<size_t>(b) * n_copies + c];
            ARG_CHECK(ctx, empty ? d == -1 || d >= 0 : d >= 0, "unit_device: a non-empty block's unit without a device");
            if (empty) ud[static_cast<size_t>(b) * n_copies + c] = -1;
        }
    }
    std::vector<dbslmm_ctx*> dev_ctx(device_index + 1, nullptr);
    dev_ctx[device_index] = ctx;
    return mp_build(ctx, pr, n_copies, ud, {device_index}, dev_ctx, true, out);
}

}  // extern "C"
