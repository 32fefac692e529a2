// multi.hip -- multi-GPU contexts and plans (included at the end of plan.hip: same translation
// unit, so the single-device plan functions are called directly).
//
// The reference parallelises only over LD blocks (OpenMP schedule(dynamic) over batches of 60,
// scr/dbslmmfit.cpp:191-220): blocks are independent, so a multi-GPU solve needs no exchange during
// compute.  A multi-device context (dbslmm_ctx_create_multi) holds one single-device context per
// device; plan_create on it:
//   1. shards the non-empty LD blocks over the devices, longest-processing-time first on
//      cost_b = n_ref m_b (m_b + 1) + m_b^3 / 3 (Gram + factorisation), deterministic;
//   2. builds each shard's sub-problem: its blocks in block order and a COMPACT .bed image holding
//      only their rows (each device receives only the packed rows it needs: 1/G of the upload);
//   3. creates the shard plans concurrently, one host thread per device (the uploads overlap on
//      the devices' own PCIe links).
// Every later call (run / run_multi / sync / download / variance / timing) fans out over the
// shards, one host thread each, and scatters the shard outputs into the caller's arrays (beta,
// status, variance columns) in the original order -- the only "exchange", straight from each
// device's HBM to the caller's host buffers.  (The ABI's outputs are host memory, so a device-side
// gather over xGMI before the copy-out would only add a hop)
#include <thread>

// Run f(i) for every shard index on its own host thread; the first failing rc wins and its
// sub-context message is copied to the parent context.
template <typename F>
static int fan_out(dbslmm_ctx* ctx, int n, F f) {
    std::vector<int> rc(n, DBSLMM_OK);
    std::vector<std::thread> th;
    th.reserve(n);
    for (int i = 0; i < n; ++i) th.emplace_back([&, i] { rc[i] = f(i); });
    for (auto& t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rc[i] != DBSLMM_OK) {
            ctx->err = "device " + std::to_string(ctx->subs[i]->device) + ": " + ctx->subs[i]->err;
            return rc[i];
        }
    return DBSLMM_OK;
}

static int mp_create(dbslmm_ctx* ctx, const dbslmm_problem* pr, dbslmm_plan** out) {
    ARG_CHECK(ctx, pr && out, "null problem/out");
    *out = nullptr;
    ARG_CHECK(ctx, pr->bed && pr->n_ref > 1 && pr->n_obs > 0 && pr->num_block >= 0, "bad sizes");
    ARG_CHECK(ctx, pr->s_ptr && (pr->s_ptr[pr->num_block] == 0 || (pr->s_pos && pr->z_s)), "bad small CSR");
    const bool has_l = pr->l_ptr != nullptr;
    if (has_l) ARG_CHECK(ctx, pr->l_ptr[pr->num_block] == 0 || (pr->l_pos && pr->z_l), "bad large CSR");
    const int64_t bps = pr->n_ref / 4 + (pr->n_ref % 4 ? 1 : 0);
    ARG_CHECK(ctx, pr->bed_len >= 3 + bps, "bed image shorter than one SNP row");
    const int64_t n_rows = (pr->bed_len - 3) / bps;
    const int G = static_cast<int>(ctx->subs.size());
    // 1. LPT shard of the non-empty blocks
    std::vector<double> cost(pr->num_block, 0.0);
    std::vector<int32_t> order;
    for (int b = 0; b < pr->num_block; ++b) {
        const int64_t ms = pr->s_ptr[b + 1] - pr->s_ptr[b], ml = has_l ? pr->l_ptr[b + 1] - pr->l_ptr[b] : 0;
        ARG_CHECK(ctx, ms >= 0 && ml >= 0, "CSR offsets not monotone");
        const double m = static_cast<double>(ms + ml);
        cost[b] = pr->n_ref * m * (m + 1.0) + m * m * m / 3.0;
        if (ms + ml > 0) order.push_back(b);
    }
    std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return cost[a] > cost[b]; });
    std::vector<double> load(G, 0.0);
    std::vector<std::vector<int32_t>> own(G);
    for (int32_t b : order) {
        const int d = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
        own[d].push_back(b);
        load[d] += cost[b];
    }
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
    p->mp->shards.resize(G);
    // 2. sub-problems with compact .bed images (rows renumbered in first-use order)
    struct Sub {
        std::vector<uint8_t> bed;
        std::vector<int64_t> s_ptr, l_ptr;
        std::vector<int32_t> s_pos, l_pos;
        std::vector<double> z_s, z_l;
        dbslmm_problem prob{};
    };
    std::vector<Sub> subs(G);
    for (int d = 0; d < G; ++d) {
        DeviceShard& sh = p->mp->shards[d];
        Sub& su = subs[d];
        std::sort(own[d].begin(), own[d].end());   // block order within the shard
        sh.blocks = own[d];
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
    // 3. shard plans, one host thread per device
    const int rc = fan_out(ctx, G, [&](int d) -> int {
        return dbslmm_plan_create(ctx->subs[d], &subs[d].prob, &p->mp->shards[d].plan);
    });
    if (rc != DBSLMM_OK) { dbslmm_plan_destroy(p); return rc; }
    p->ran = false;
    *out = p;
    return DBSLMM_OK;
}

static void mp_destroy(dbslmm_plan* p) {
    for (DeviceShard& sh : p->mp->shards) dbslmm_plan_destroy(sh.plan);
    delete p->mp;
    p->mp = nullptr;
}

// beta / status of one solve, scattered from every shard into the caller's arrays
static int mp_download(dbslmm_plan* p, int copy, double* beta_s, double* beta_l, int32_t* block_status) {
    dbslmm_ctx* ctx = p->ctx;
    auto& S = p->mp->shards;
    if (block_status)
        for (int32_t b = 0; b < p->num_block; ++b) block_status[b] = DBSLMM_BLOCK_EMPTY;
    return fan_out(ctx, static_cast<int>(S.size()), [&](int d) -> int {
        DeviceShard& sh = S[d];
        std::vector<double> bs(sh.s_idx.size()), bl(sh.l_idx.size());
        std::vector<int32_t> st(sh.blocks.size());
        const int rc = download_copy(sh.plan, copy, bs.data(), bl.data(), st.data());
        if (rc != DBSLMM_OK) return rc;
        if (beta_s) for (size_t i = 0; i < bs.size(); ++i) beta_s[sh.s_idx[i]] = bs[i];
        if (beta_l) for (size_t i = 0; i < bl.size(); ++i) beta_l[sh.l_idx[i]] = bl[i];
        if (block_status) for (size_t i = 0; i < st.size(); ++i) block_status[sh.blocks[i]] = st[i];
        return DBSLMM_OK;
    });
}

static int mp_run(dbslmm_plan* p, const double* sigmas, int n, bool wait) {
    auto& S = p->mp->shards;
    const int rc = fan_out(p->ctx, static_cast<int>(S.size()), [&](int d) -> int {
        dbslmm_plan* q = S[d].plan;
        int r = run_impl(q, true, sigmas, n);
        if (r == DBSLMM_OK && wait) r = dbslmm_plan_sync(q);
        return r;
    });
    if (rc == DBSLMM_OK) {
        p->ran = true;
        p->var_copy = n - 1;
        p->sigma_run = sigmas[n - 1];
    }
    return rc;
}

static int mp_sync(dbslmm_plan* p) {
    auto& S = p->mp->shards;
    return fan_out(p->ctx, static_cast<int>(S.size()), [&](int d) -> int { return dbslmm_plan_sync(S[d].plan); });
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
    std::fill(diags, diags + static_cast<size_t>(n_test) * p->num_block, 0.0);
    auto& S = p->mp->shards;
    // every shard's pending single-sigma re-run (graph captures) first, drained, then the variances
    const int rc0 = fan_out(ctx, static_cast<int>(S.size()), [&](int d) -> int {
        dbslmm_plan* q = S[d].plan;
        if (S[d].blocks.empty() || !q->cheb_pending_var) return DBSLMM_OK;
        const int r = variance_factor(q);
        return r == DBSLMM_OK ? dbslmm_plan_sync(q) : r;
    });
    if (rc0 != DBSLMM_OK) return rc0;
    return fan_out(ctx, static_cast<int>(S.size()), [&](int d) -> int {
        DeviceShard& sh = S[d];
        if (sh.blocks.empty()) return DBSLMM_OK;
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
    return fan_out(ctx, G, [&](int d) -> int {
        const int64_t r0 = n_snp * d / G, r1 = n_snp * (d + 1) / G;
        if (r1 == r0) return DBSLMM_OK;
        return dbslmm_bed_maf(ctx->subs[d], bed + r0 * bps, 3 + (r1 - r0) * bps, n_ref, r1 - r0, maf + r0);
    });
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
    for (int32_t b = 0; b < p->num_block; ++b) block_device[b] = -1;   // empty blocks
    for (size_t d = 0; d < p->mp->shards.size(); ++d)
        for (int32_t b : p->mp->shards[d].blocks) block_device[b] = static_cast<int32_t>(d);
    return DBSLMM_OK;
}

}  // extern "C"
