#!/usr/bin/env python3
"""Benchmark of the per-LD-block effect-size solver (DBSLMMFIT::est hot path) on MI355X.

One "step" = one full solve of the workload with the packed genotypes already resident in HBM:
2-bit unpack + per-SNP stats -> joint i8-MFMA Gram per LD block -> fp64 Cholesky + solves ->
beta in HBM.  Default workload = the configuration BASELINE.json's metric is quoted on
("1M SNP x 10k indiv"), configs[3]: synthetic 1M SNPs x 10k individuals over the 22-chromosome
EUR LD blocks, DBSLMM (large + small effects), h2 = 0.5 tuned over h2f in {0.8, 1.0, 1.2} (one
Gram + three factorisations and solves per step).  --config 2 is the small configs[1] case.

    python bench.py [--gpus N --steps K --warmup W] [--devices 0,0]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Multi-GPU (strong scaling, the default): ONE problem -- the same workload as N=1 -- with its LD
blocks sharded over the GPUs (longest processing time first on n_ref m(m+1) + m^3/3, each GPU
holding only its blocks' .bed rows).  Two launch modes:

* one process (`python bench.py --gpus N`, no WORLD_SIZE): the product's own multi-device context
  (dbslmm_ctx_create_multi through dbslmm_amd.Context(list of devices)): one host thread per
  device, every shard's betas copied straight into the caller's arrays.  --devices a,b,.. names
  the device list (repeats allowed: `--gpus 2 --devices 0,0` rehearses two shards on one GPU);
* one process per GPU under torch.distributed.run (WORLD_SIZE = N; implied --dist): each rank
  solves its shard (dbslmm_amd/dist.py) and the betas are gathered to rank 0 with one RCCL
  `gather` per step (the path's only exchange); value uses the max-over-ranks time.

value = the problem's SNPs x steps / time.  For N > 1 the merged betas of the last step are checked
against the oracle's direct solve on every block >= 2000 SNPs (max_dbeta_vs_cpu_ref.big_blocks).
--replicas (torchrun): N independent copies of the workload (seed = 1 + rank, no exchange) -> weak
scaling.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
PEAK_HBM_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_FP4_TOPS = 10000.0      # dense FP4 MFMA (MI355X_MICROARCH.md: ~10 PF dense; the Gram's instruction)
PEAK_I8_TOPS = 5000.0        # dense i8 MFMA (the natural roof of exact integer work; reported beside)
PEAK_F64_TFLOPS = 78.6       # fp64 (vector = matrix rate on gfx950)

# BASELINE.json configs (1-based): synthetic panels; 3-5 are the scale configs
CONFIGS = {
    # configs[0]: the reference's own example (test_dat chr1, DBSLMM, EUR chr1 blocks) through the
    # drop-in CLI; the CPU leg times the C restatement on 1 thread (config1_main)
    1: dict(snps=None, n_ref=None, pop="EUR", lmm_only=False, gen=None),
    2: dict(snps=50000, n_ref=2000, pop="EUR", lmm_only=False, gen="numpy"),
    3: dict(snps=500000, n_ref=5000, pop="EUR", lmm_only=False, gen="gpu"),
    4: dict(snps=1000000, n_ref=10000, pop="EUR", lmm_only=False, gen="gpu", h2f="0.8,1,1.2"),
    5: dict(snps=1000000, n_ref=10000, pop="AFR", lmm_only=True, gen="gpu"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--devices", default=None,
                    help="one process, N > 1: device ordinals of the multi-device context, e.g. 0,1 or "
                         "0,0 (a rehearsal on one GPU); default 0..gpus-1")
    ap.add_argument("--dist", action="store_true",
                    help="one process per GPU over torch.distributed (implied by a torchrun launch, "
                         "WORLD_SIZE > 1)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=4, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i-1] preset (4 = the metric's 1M x 10k workload)")
    ap.add_argument("--snps", type=int, default=None)
    ap.add_argument("--n-ref", type=int, default=None)
    ap.add_argument("--pop", default=None)
    ap.add_argument("--lmm-only", action="store_true", default=None)
    ap.add_argument("--h2f", default=None,
                    help="h2 factors, e.g. 0.8,1,1.2: one Gram + one solve per factor per step "
                         "(DBSLMM tuning, config 4)")
    ap.add_argument("--gen", choices=("numpy", "gpu"), default=None,
                    help="synthetic panel generator (default: numpy for config 2, gpu above)")
    ap.add_argument("--opt", action="append", default=[], metavar="KEY=VALUE",
                    help="dbslmm_options field (path thresholds; experiments), repeatable")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true",
                    help="N > 1: skip the big-block beta check of the merged betas")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the untimed lead-group-off run that times the Gram without overlap")
    ap.add_argument("--e2e-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end leg (PLINK files in page cache -> the dbslmm CLI -> <eff>.txt)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = all host threads (OMP_NUM_THREADS, else the affinity mask)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="process group backend (nccl = RCCL over xGMI; gloo only for rehearsals)")
    ap.add_argument("--rank-device", type=int, default=None,
                    help="rehearsal on a 1-GPU box: every rank on this device instead of LOCAL_RANK")
    ap.add_argument("--predict", default="auto", metavar="N[,N..]",
                    help="N = 1 only: one-GPU rehearsal of an N-GPU strong-scaling step -- each device's "
                         "units of the N-device shard plan timed alone on this GPU; predicted step = the "
                         "slowest device (reported beside the line, never as value).  auto (default) = "
                         "2,4,8 for the metric's workload (config 4), none elsewhere; none = off")
    ap.add_argument("--replicas", action="store_true",
                    help="N>1: independent replicas of the workload per rank (weak scaling) instead "
                         "of one problem sharded over the ranks (strong scaling)")
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.h2f = [float(x) for x in a.h2f.split(",")] if a.h2f else None
    if a.predict == "auto":
        a.predict = "2,4,8" if a.config == 4 and a.snps == CONFIGS[4]["snps"] else None
    elif a.predict == "none":
        a.predict = None
    return a


def kernel_roofline(name, ms, wl, n_solve=1):
    """ms = the kernel's time per step; n_solve = solves per step (h2f factors)."""
    s = ms * 1e-3
    if name == "dbslmm_unpack_stats":
        b = wl["unpack_read_bytes"] + wl["unpack_write_bytes"]
        a = b / s / 1e9
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms)
    if name == "dbslmm_pcg":
        # the PCG route (pcg.hip): the chip-wide iterations -- every block it iterates streams its
        # lower-triangle LD matrix (uint16 integer Gram) once per iteration, plus the product's
        # partial sums; every block its own iteration count (plan workload [19], [20])
        b = wl.get("pcg_chip_bytes", 0.0) + wl.get("pcg_partial_bytes", 0.0)
        a = b / s / 1e9 if s > 0 else 0.0
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms, iterations=wl.get("pcg_iters", 0.0),
                    matrix_bytes=wl.get("pcg_chip_bytes", 0.0), partial_bytes=wl.get("pcg_partial_bytes", 0.0),
                    note="Jacobi-PCG (the reference's PCGv) on every block's joint matrix, all h2f copies "
                         "together; ms = init to final (the rows / update launches included), a span that also "
                         "holds dbslmm_pcg_block on the second stream: its bytes count there, not here")
    if name == "dbslmm_pcg_block":
        # the small one-column blocks solved whole, one workgroup each: their lower-triangle matrices
        # streamed once per iteration of each block (plan workload [21])
        b = wl.get("pcg_block_bytes", 0.0)
        a = b / s / 1e9 if s > 0 else 0.0
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms,
                    note="one launch per run (HIP events on its stream), beside the chip-wide iterations of "
                         "the other blocks; algorithmic = sum over its blocks of iterations x the lower "
                         "triangle's uint16 bytes")
    if name == "dbslmm_gram":
        a = wl["gram_ops_alg"] / s / 1e12
        return dict(kernel=name, bound="mfma", achieved=a, peak=PEAK_FP4_TOPS, unit="TFLOP/s",
                    frac=a / PEAK_FP4_TOPS, frac_vs_i8_peak=a / PEAK_I8_TOPS,
                    algorithmic=wl["gram_ops_alg"], ms=ms,
                    executed_tops=wl["gram_ops_exec"] / s / 1e12,
                    note="ops (2/MAC) of the exact integer Gram, algorithmic sum_b n_ref*m_b*(m_b+1), vs "
                         "the dense FP4 peak of the instruction it issues (v_mfma_scale_f32_32x32x64_f8f6f4, "
                         "dosages as e2m1); executed = padded tiles x padded individuals")
    if name == "dbslmm_trsv":
        # h2f iterations (CG by default): per iteration one forward + one backward substitution,
        # each streaming the base copy's factor once (HBM-bound; chained over 64-row tiles); the
        # plan counts each tiled block's own passes (a converged block's later items are skipped)
        b = wl.get("h2f_pass_bytes") or 2.0 * wl["trsv_bytes"] * wl["cheb_iters"]
        a = b / s / 1e9 if s > 0 else 0.0
        it = b / (2.0 * wl["trsv_bytes"]) if wl["trsv_bytes"] > 0 else 0.0
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms,
                    note="factor bytes read by the h2f iterations' forward + backward substitutions on the "
                         "base copy's factor: %.2f iterations per tiled block on average (byte-weighted; cap %d); "
                         "chain- and streaming-bound, ~5.7 us per 64-row step of the largest block" % (it, wl["cheb_iters"]))
    if name in ("dbslmm_tchol", "dbslmm_chol_large") and wl["cheb_iters"] > 0:
        n_solve = 1     # h2f: only the base copy of the tiled and single-workgroup blocks is factored
    fl = n_solve * {"dbslmm_chol_large": wl["chol_flops_large"], "dbslmm_chol_small": wl["chol_flops_small"],
                    "dbslmm_tchol": wl["chol_flops_tiled"]}[name]
    a = fl / s / 1e12 if s > 0 else 0.0
    return dict(kernel=name, bound="mfma", achieved=a, peak=PEAK_F64_TFLOPS, unit="TFLOP/s",
                frac=a / PEAK_F64_TFLOPS, algorithmic=fl, ms=ms,
                note="fp64 flops sum_b m^3/3 + 2m^2 over its blocks vs the fp64 MFMA peak"
                     + ("; multi-workgroup sequence, %d launches; wall span from the first tiled launch (the "
                        "lead group's sequence starts during the Gram and overlaps it)" % wl["tiled_launches"]
                        if name == "dbslmm_tchol" else "; latency-bound (sequential column chain)"))


def pmc_traffic(kernel, args, n_solve):
    """HBM bytes per step of `kernel` from the latest committed rocprofv3 PMC passes (FETCH_SIZE x2
    + WRITE_SIZE, tools/pmc_traffic.py) of this same preset workload (profiles/r*/
    pmc_traffic_c<N>.json), or None.  The tiled sequence is counted per solve x n_solve."""
    import glob
    preset = CONFIGS[args.config]
    same = all(getattr(args, k) == (v if k != "h2f" else [float(x) for x in v.split(",")])
               for k, v in preset.items()) and (args.h2f is None) == ("h2f" not in preset)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"pmc_traffic_c{args.config}.json")))
    if not same or not files:
        return None, None
    d = json.load(open(files[-1]))
    k = d.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    if "hbm_bytes_per_step" in k:             # composite phases (tiled sequence, h2f substitutions)
        per = k["hbm_bytes_per_step"]
    else:
        per = k["hbm_bytes"] * (n_solve if kernel.startswith("dbslmm_chol") else 1)
    return per, os.path.relpath(files[-1], ROOT)


def host_info():
    """CPU model, logical CPUs of the machine and the threads this process may use (the GPU box
    shows the whole machine in nproc; its CPU share is OMP_NUM_THREADS)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    share = int(os.environ.get("OMP_NUM_THREADS") or aff)
    return dict(cpu_model=model, nproc=nproc, affinity=aff, threads_all=max(1, min(share, aff)))


def cpu_leg(args, prob, res, sigmas, wl):
    """cpu_baseline (the C restatement of the reference, timed on this host) and the beta check.

    Timing: blocks drawn SNP-uniformly (a block with probability ~ its SNP count, so big blocks
    appear as often as their share of SNPs) until ~args.cpu_seconds of CPU work, once with all
    host threads (OpenMP over blocks, 1 BLAS thread each -- the reference's -t N build) and once
    with 1 thread.  The sample's throughput in cost units (block_cost = n_ref m(m+1) + m^3/3) is
    applied to the whole workload's cost, bounded below by the largest block's single-thread time
    (a block never spans threads in the reference): value = workload SNPs / that time.
    Beta check: every block with >= 2000 SNPs against the oracle's direct (Cholesky) solve on all
    host cores, plus the timed sample against the reference-faithful PCG."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ref_numpy as R
    from dbslmm_amd.dist import block_cost, sub_problem
    blas = O.use_blas(True)
    hi = host_info()
    thr = args.cpu_threads or hi["threads_all"]
    nblk = len(prob.s_ptr) - 1
    m_b = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    cost = block_cost(m_b, prob.n_ref)
    sig_list = sigmas if sigmas else [prob.sigma_s]
    rng = np.random.default_rng(0)
    nz = np.flatnonzero(m_b > 0)
    order = rng.choice(nz, size=nz.size, replace=False, p=m_b[nz] / m_b[nz].sum())

    def timed(threads, seconds):
        """Blocks in `order` (skipping those whose own cost exceeds the call budget) until the
        budget: returns (SNPs, cost, seconds, blocks, outs)."""
        done_snps, done_cost, tc, used, outs = 0, 0.0, 0.0, [], []
        rate = 2e9 * threads            # cost units / s, refined after every call
        i = 0
        while tc < seconds and i < order.size:
            # next call: ~1 s of work at the measured rate; a block whose single-thread time
            # would exceed 40 % of the budget is left out (the reference never splits a block)
            budget = rate * max(0.2, min(1.0, seconds - tc))
            cur, acc = [], 0.0
            while i < order.size and acc < budget:
                b = order[i]
                i += 1
                if cost[b] / (rate / threads) > 0.4 * seconds:
                    continue
                cur.append(b)
                acc += cost[b]
            if not cur:
                continue
            blocks = np.sort(np.array(cur))
            sub, s_idx, l_idx = sub_problem(prob, blocks)
            c0 = time.perf_counter()
            o = [O.est(sub.bed, sub.n_ref, sub.n_obs, sg, sub.s_ptr, sub.s_pos, sub.z_s,
                       sub.l_ptr, sub.l_pos, sub.z_l, tau=prob.tau, method="pcg", threads=threads)
                 for sg in sig_list]       # the reference runs dbslmm once per h2f factor
            tc += time.perf_counter() - c0
            done_snps += len(s_idx) + len(l_idx)
            done_cost += acc
            rate = done_cost / tc
            used.append(blocks)
            outs.append((s_idx, l_idx, o))
        return done_snps, done_cost, tc, used, outs

    snps_t, cost_t, sec_t, used_t, outs_t = timed(thr, args.cpu_seconds)
    snps_1, cost_1, sec_1, used_1, _ = timed(1, max(2.0, args.cpu_seconds / 2)) if thr > 1 else \
        (snps_t, cost_t, sec_t, used_t, None)
    rate_t, rate_1 = cost_t / sec_t, cost_1 / sec_1          # cost units per second
    total, cmax, m_all = float(cost.sum()), float(cost.max()), float(m_b.sum())
    t_all = max(total / rate_t, cmax / rate_1)
    t_one = total / rate_1
    nb_t = int(sum(len(u) for u in used_t))
    cpu = dict(
        value=m_all / t_all, unit="SNPs/s", cores=thr, kind="port",
        sample=(f"{nb_t} of {nblk} blocks ({snps_t} SNPs, {cost_t / total:.1%} of the workload's "
                f"cost) drawn SNP-uniformly, {sec_t:.1f} s on {thr} threads (OpenMP over blocks, "
                f"1 BLAS thread each, {len(sig_list)} solve(s) per SNP as on the GPU); value = "
                f"workload SNPs / (workload cost at the sample's cost rate, >= the largest block "
                f"at the 1-thread rate): C restatement of the reference (byte-wise readSNPIm, N-1 "
                f"standardise, {'OpenBLAS dsyrk/dgemm/dgemv' if blas else 'plain-loop Gram'}, "
                f"Jacobi-PCG tol 1e-7)"),
        sample_snps_per_s=snps_t / sec_t,
        t1=dict(value=m_all / t_one, cores=1, sample_snps=snps_1, seconds=sec_1,
                sample_snps_per_s=snps_1 / sec_1),
        host=hi, est_seconds_per_step=t_all,
        cores_note=(f"{thr} threads = this GPU box's CPU share: the pool exports OMP_NUM_THREADS="
                    f"{os.environ.get('OMP_NUM_THREADS', '?')} for one GPU and asks jobs to size worker "
                    f"pools to it; the affinity mask ({hi['affinity']} threads) spans the whole host, "
                    f"which other jobs share, so it is not this job's to use"),
        node_linear_estimate=dict(
            value=m_all / t_all * (hi["nproc"] / 2) / thr, cores=hi["nproc"] // 2,
            note="upper bound for the reference on every physical core of this host: the measured "
                 "rate scaled linearly from the threads used (not measured)"))
    # beta check 1: the timed sample vs the reference-faithful PCG (every h2f solve)
    mx, nw, ncmp = 0.0, 0.0, 0
    for s_idx, l_idx, o in outs_t:
        for c, (rs, rl, _, _) in enumerate(o):
            ref = np.concatenate([rs, rl])
            got = np.concatenate([res[c][0][s_idx], res[c][1][l_idx]])
            ok = np.isfinite(ref)
            if ok.any():
                mx = max(mx, float(np.max(np.abs(got[ok] - ref[ok]))))
                nw = max(nw, float(np.max(np.abs(got[ok] - ref[ok])) / np.max(np.abs(ref[ok]))))
            ncmp += int(ok.sum())
    dbeta = dict(max_abs=mx, normwise=nw, snps_compared=ncmp,
                 vs="CPU reference-faithful PCG (oracle) on the timed sample" +
                    (", every h2f solve" if sigmas else ""))
    dbeta["big_blocks"] = big_block_check(prob, res, sigmas)
    return cpu, dbeta


def big_block_check(prob, res, sigmas):
    """beta check on every block >= 2000 SNPs vs the oracle's direct fp64 solve of the reference
    equations (all host cores per block), every h2f solve; res = the full problem's results."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ref_numpy as R
    O.use_blas(True)
    hi = host_info()
    sig_list = sigmas if sigmas else [prob.sigma_s]
    m_b = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    big = np.flatnonzero(m_b >= 2000)
    O.blas_threads(hi["threads_all"])
    bmx, bnw, bsn = 0.0, 0.0, 0
    t0 = time.perf_counter()
    try:
        for b in big:
            b = int(b)
            s0, s1 = int(prob.s_ptr[b]), int(prob.s_ptr[b + 1])
            Xs = O.read_block_std(prob.bed, prob.n_ref, prob.s_pos[s0:s1], threads=hi["threads_all"])
            Xl = None
            if prob.l_ptr is not None and prob.l_ptr[b + 1] > prob.l_ptr[b]:
                l0, l1 = int(prob.l_ptr[b]), int(prob.l_ptr[b + 1])
                Xl = O.read_block_std(prob.bed, prob.n_ref, prob.l_pos[l0:l1], threads=hi["threads_all"])
            Sss, Sls, Sll = R.block_sigmas_tau(Xs, Xl, prob.n_ref, prob.tau)
            del Xs, Xl
            for c, sg in enumerate(sig_list):
                if Sls is None:
                    ref = R.est_block_s_sigma(Sss, prob.n_obs, sg, prob.z_s[s0:s1], "chol")
                    got = res[c][0][s0:s1]
                else:
                    rs, rl = R.est_block_ls_sigma(Sss, Sls, Sll, prob.n_obs, sg, prob.z_s[s0:s1],
                                                  prob.z_l[l0:l1], "chol")
                    ref = np.concatenate([rs, rl])
                    got = np.concatenate([res[c][0][s0:s1], res[c][1][l0:l1]])
                d = float(np.max(np.abs(got - ref)))
                bmx, bnw = max(bmx, d), max(bnw, d / float(np.max(np.abs(ref))))
                bsn += ref.size
    finally:
        O.blas_threads(1)
    return dict(blocks=int(big.size), max_m=int(m_b.max()), snps_compared=bsn,
                max_abs=bmx, normwise_per_block_max=bnw, seconds=time.perf_counter() - t0,
                vs="oracle direct fp64 solve (Cholesky) of the reference equations, "
                   "every block >= 2000 SNPs" + (", every h2f solve" if sigmas else ""))


def predict_leg(args, full, sigmas, m_b, ctx):
    """One-GPU rehearsal of the N-GPU strong-scaling step: for each N the
    library's shard plan (dbslmm_shard_plan_problem) splits the problem into N devices' units;
    each device's units plan (dbslmm_plan_create_units, exactly what rank d of
    `torch.distributed.run --nproc-per-node N bench.py` runs) is timed ALONE on this GPU -- 2
    warm-up, then the median of five batches of `k` synchronous solves, like the timed step --
    and the predicted step is the slowest device (plus the
    time model's own prediction beside it).  The RCCL gather of <= 3 x 8 MB over xGMI is not
    included (~0.1 ms)."""
    import numpy as np
    from dbslmm_amd import Plan
    from dbslmm_amd.dist import shard_units_problem
    K = len(sigmas) if sigmas else 1
    sig = sigmas if sigmas else [full.sigma_s]
    k = 5
    out = {}
    for N in [int(x) for x in args.predict.split(",")]:
        ud, model = shard_units_problem(full, sig, N)
        split = np.flatnonzero(~np.all(ud == ud[:, :1], axis=1))
        per = []
        for d in range(N):
            plan = Plan.units(ctx, full, ud, d)
            o = (np.zeros((K, full.n_s)), np.zeros((K, full.n_l)), np.zeros((K, full.num_block), dtype=np.int32))
            for _ in range(2):
                plan.run_multi(sig, out=o)
            batches = []
            for _ in range(5):          # the median of five batches of k (host noise: tools/r06_dev.py)
                t0 = time.perf_counter()
                for _ in range(k):
                    plan.run_multi(sig, out=o)
                batches.append((time.perf_counter() - t0) / k * 1e3)
            per.append(float(np.median(batches)))
            plan.close()
        step = max(per)
        out[str(N)] = dict(step_ms=step, value=float(m_b.sum()) / (step * 1e-3), per_device_ms=per,
                           model_ms=model.tolist(),
                           split_blocks=[dict(block=int(b), snps=int(m_b[b]), devices=ud[b].tolist()) for b in split])
    return dict(results=out, unit="SNPs/s", note=(
        "one-GPU rehearsal: each device's units plan of the N-device shard plan timed alone (2 warm-up, "
        f"the median of 5 batches of {k} synchronous solves); predicted N-GPU step = the slowest device; value = the problem's SNPs / "
        "that step.  Excludes the per-step RCCL gather of the betas to rank 0."))


def e2e_leg(args, panel):
    """End to end through the drop-in CLI: the workload's synthetic panel written as PLINK
    ref.{bed,bim,fam} + GEMMA summaries + block file (page cache), then `dbslmm` (mmap'd .bed ->
    one staged upload -> GPU MAF pass -> parse/match -> plan -> solve -> <eff>.txt per h2f) in a
    fresh process, twice; the second run is reported.  SNPs/s = solved SNPs / the process's wall
    time (HIP initialisation included; `ctx` is that part)."""
    import shutil
    import subprocess
    import tempfile
    from dbslmm_amd import synth
    d = tempfile.mkdtemp(prefix="dbslmm_e2e_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        f = synth.write_plink(panel, d)
        t_files = time.perf_counter() - t0
        cmd = [os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm"), "-s", f["s"], "-r", f["ref"], "-b", f["b"],
               "-n", str(f["n"]), "-nsnp", str(f["nsnp"]), "-h", "0.5", "-mafMax", "0.2",
               "-eff", os.path.join(d, "eff"), "--timing"]
        if not args.lmm_only:
            cmd += ["-l", f["l"]]
        if args.h2f:
            cmd += ["-h2f", ",".join("%g" % x for x in args.h2f)]
        runs = []
        for _ in range(2):
            t1 = time.perf_counter()
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            wall = time.perf_counter() - t1
            if r.returncode != 0:
                return dict(error=f"dbslmm CLI rc={r.returncode}: {r.stderr[-400:]}")
            line = [x for x in r.stderr.splitlines() if x.startswith("TIMING ")]
            ph = json.loads(line[-1][7:]) if line else {}
            runs.append((wall, ph))
        wall, ph = runs[-1]
        n = ph.get("snps", 0)
        return dict(value=n / wall, unit="SNPs/s", seconds=wall, snps=n, phases_s=ph,
                    value_after_init=n / max(1e-9, wall - ph.get("ctx", 0.0)),
                    files_written_s=t_files, solves_per_snp=len(args.h2f) if args.h2f else 1,
                    note="page-cached PLINK files -> dbslmm CLI -> <eff>.txt, one process on GPU 0 "
                         "(HIP init, .bed upload, GPU MAF pass, host parse/match, plan, solve, writer)")
    finally:
        shutil.rmtree(d, ignore_errors=True)


def config1_main(args):
    """BASELINE configs[0]: test_dat chr1 (tests/golden/test_dat: ref_chr1 400 individuals, the
    GEMMA summary split into small / large SNPs by the clumped list tests/golden/l_snps.txt), EUR
    chr1 blocks, DBSLMM tau 0.8, -n 2400 -nsnp 996 -h 0.5 -mafMax 0.2 -- the reference's own
    example.  GPU: the drop-in CLI (HIP init, parse, plan, solve, writer), run twice; the second
    run also re-solves the resident problem `steps` times (--repeat): ms_per_step = their mean,
    value = SNPs per second of it.  CPU: the C restatement of the reference (readSNPIm, N-1
    standardise, Gram, Jacobi-PCG 1e-7) on 1 thread -- the reference's -t 1 -- on the same
    problem, repeated for ~2 s; the betas are compared with the CLI's --precise-out file."""
    import subprocess
    import tempfile
    import numpy as np
    td = os.path.join(ROOT, "tests", "golden", "test_dat")
    blocks_f = os.path.join(ROOT, "dbslmm_amd", "data", "block_data", "EUR", "chr1.bed")
    lset = {l.strip() for l in open(os.path.join(ROOT, "tests", "golden", "l_snps.txt")) if l.strip()}
    d = tempfile.mkdtemp(prefix="dbslmm_c1_", dir=os.environ.get("TMPDIR", "/tmp"))
    s_f, l_f = os.path.join(d, "s.txt"), os.path.join(d, "l.txt")
    with open(os.path.join(td, "summary_gemma_chr1.assoc.txt")) as f, open(s_f, "w") as fs, open(l_f, "w") as fl:
        for line in f:
            (fl if line.split("\t")[1] in lset else fs).write(line)
    eff = os.path.join(d, "eff")
    cmd = [os.path.join(ROOT, "dbslmm_amd", "bin", "dbslmm"), "-s", s_f, "-l", l_f, "-r", os.path.join(td, "ref_chr1"),
           "-b", blocks_f, "-n", "2400", "-nsnp", "996", "-h", "0.5", "-mafMax", "0.2", "-t", "1",
           "-eff", eff, "--precise-out", "--timing", "--repeat", str(args.warmup + args.steps)]
    runs = []
    for _ in range(2):
        t1 = time.perf_counter()
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        wall = time.perf_counter() - t1
        if r.returncode != 0:
            raise SystemExit(f"dbslmm CLI rc={r.returncode}: {r.stderr[-400:]}")
        line = [x for x in r.stderr.splitlines() if x.startswith("TIMING ")]
        runs.append((wall, json.loads(line[-1][7:])))
    wall, ph = runs[-1]
    rep = ph["solve_repeat"][args.warmup:]
    step_s = float(np.mean(rep))
    n_snp = int(ph["snps"])
    rows = [x.split() for x in open(eff + ".txt").read().splitlines() if x.strip()]
    got = np.array([float(x[2]) for x in rows])

    # CPU leg (the oracle = the C restatement of the reference; bench's cpu_baseline leg)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    import ref_numpy as R
    blas = O.use_blas(True)
    n_ref = R.get_row(os.path.join(td, "ref_chr1.fam"))
    bim = R.read_bim(os.path.join(td, "ref_chr1"), n_ref, True)
    blocks = R.read_block(blocks_f)
    info_s = R.add_block(R.match_ref(R.read_summ(s_f), bim, 0.2)[0], blocks)
    info_l = R.add_block(R.match_ref(R.read_summ(l_f), bim, 0.2)[0], blocks)
    nb = len(blocks)

    def csr(infos):
        ptr = np.zeros(nb + 1, dtype=np.int64)
        for x in infos:
            ptr[x["block"] + 1] += 1
        return (np.cumsum(ptr), np.array([x["pos"] for x in infos], dtype=np.int32),
                np.array([x["z"] for x in infos], dtype=np.float64))

    s_ptr, s_pos, z_s = csr(info_s)
    l_ptr, l_pos, z_l = csr(info_l)
    bed = np.fromfile(os.path.join(td, "ref_chr1.bed"), dtype=np.uint8)
    outs, k, t0 = None, 0, time.perf_counter()
    while True:
        outs = {m: O.est(bed, n_ref, 2400, 0.5 / 996, s_ptr, s_pos, z_s, l_ptr, l_pos, z_l, tau=0.8,
                         method=m, threads=1) for m in ("pcg",)}
        k += 1
        if time.perf_counter() - t0 > 2.0:
            break
    cpu_s = (time.perf_counter() - t0) / k
    direct = O.est(bed, n_ref, 2400, 0.5 / 996, s_ptr, s_pos, z_s, l_ptr, l_pos, z_l, tau=0.8,
                   method="direct", threads=1)
    res = {}

    def eff_order(bs, bl):   # <eff>.txt rows: large then small, rows with an infinite beta_noscl dropped
        v = []
        for info, beta in ((info_l, bl), (info_s, bs)):
            for e, b in zip(info, beta):
                if e["maf"] in (0.0, 1.0) and b != 0:
                    continue
                v.append(b)
        return np.array(v)

    for name, o in (("pcg", outs["pcg"]), ("direct", direct)):
        exp = eff_order(o[0], o[1])
        res[name] = dict(max_abs=float(np.max(np.abs(got - exp))),
                         normwise=float(np.max(np.abs(got - exp)) / np.max(np.abs(exp))))
    m_b = np.diff(s_ptr) + np.diff(l_ptr)
    flops = float(np.sum(n_ref * m_b * (m_b + 1.0) + m_b.astype(float) ** 3 / 3 + 2.0 * m_b ** 2))
    ach = flops / step_s / 1e12
    out = {
        "metric": "SNPs solved/sec (whole node) + max-|\u0394\u03b2| vs CPU ref, test_dat chr1",
        "value": n_snp / step_s, "unit": "SNPs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": step_s * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "the reference's test_dat chr1 example (tests/golden/test_dat, 400 individuals)",
        "config": {"workload": "test_dat chr1, DBSLMM tau 0.8, -n 2400 -nsnp 996 -h 0.5 -mafMax 0.2, EUR chr1 "
                               "blocks (BASELINE configs[0])", "snps": n_snp, "n_ref": n_ref, "blocks": nb,
                   "parallelism": "1 GPU (drop-in CLI)"},
        "roofline": {"bound": "mfma", "achieved": ach, "peak": 78.6, "unit": "TFLOP/s", "frac": ach / 78.6,
                     "traffic": None, "kernel": "whole solve (Gram + factorisation + substitution)",
                     "note": "algorithmic fp64-equivalent flops n_ref m(m+1) + m^3/3 + 2m^2 per block over "
                             "the CLI's re-solve time (launch-bound at this size)"},
        "cpu_baseline": {"value": n_snp / cpu_s, "unit": "SNPs/s", "cores": 1, "kind": "port",
                         "sample": f"the whole workload, {k} repetitions in {k * cpu_s:.2f} s: C restatement of "
                                   f"the reference (byte-wise readSNPIm, N-1 standardise, "
                                   f"{'OpenBLAS' if blas else 'plain-loop'} Gram, Jacobi-PCG tol 1e-7), "
                                   f"1 thread = the reference's -t 1", "seconds": cpu_s},
        "end_to_end": {"value": n_snp / wall, "unit": "SNPs/s", "seconds": wall, "phases_s": ph,
                       "note": "dbslmm CLI process wall time, HIP init included (second of two runs)"},
        "max_dbeta_vs_cpu_ref": {"vs_pcg": res["pcg"], "vs_direct": res["direct"], "snps_compared": int(got.size)},
    }
    print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.config == 1:
        return config1_main(args)
    if args.e2e_only:   # child of the N = 1 run below: fresh process, GPU otherwise idle
        from dbslmm_amd import synth
        panel = synth.simulate(args.snps, args.n_ref, pop=args.pop, seed=1, engine=args.gen, device=0)
        print(json.dumps(e2e_leg(args, panel)), flush=True)
        return
    e2e_pre = None
    if (int(os.environ.get("WORLD_SIZE", "1")) == 1 and not args.no_e2e and not args.devices
            and args.gpus == 1 and args.rank_device is None):
        # The end-to-end CLI leg runs first, in a child process, before this process initialises
        # the GPU: measured beside this process's resident plans the CLI's solve phase took 0.6-0.9 s
        # instead of 0.07-0.10 s (tools/e2e_probe.py), which is this process's state, not the CLI's.
        import subprocess
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--e2e-only"] + sys.argv[1:],
                           capture_output=True, text=True, timeout=900)
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        e2e_pre = json.loads(lines[-1]) if r.returncode == 0 and lines else \
            dict(error=f"e2e child rc={r.returncode}: {r.stderr[-400:]}")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    dist = None
    if args.rank_device is not None:
        local = args.rank_device
    # one process: the product's multi-device context over `devices` (N = len(devices))
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    if world > 1:
        devices = [local]
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(devices[0])
    in_proc = world == 1 and len(devices) > 1
    n_gpus = world if world > 1 else len(devices)
    cdev = "cuda" if args.dist_backend == "nccl" else "cpu"    # collective tensors

    from dbslmm_amd import Context, KERNEL_NAMES, Plan, synth
    from dbslmm_amd.dist import UnitGather, shard_units_problem

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    sharded = world > 1 and not args.replicas
    panel = synth.simulate(args.snps, args.n_ref, pop=args.pop, seed=1 if sharded else 1 + rank,
                           engine=args.gen, device=devices[0])
    full = synth.make_problem(panel, lmm_only=args.lmm_only)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        full.opts[k] = float(v) if k in ("cheb_tol", "pcg_tol") else int(v)
    del panel   # (the end-to-end leg generated its own copy in its child process)
    sigmas = [full.sigma_s * f for f in args.h2f] if args.h2f else None
    n_copies = len(sigmas) if sigmas else 1
    m_b = np.diff(full.s_ptr) + (np.diff(full.l_ptr) if full.l_ptr is not None else 0)
    if n_copies > 1:
        full.opts["shard_copies"] = n_copies   # multi-device context: h2f copies may be split
    gather = None
    prob = full
    sig_run = sigmas if sigmas else [full.sigma_s]
    ctx = Context(devices if in_proc else devices[0])
    if sharded:
        # this rank's (block, h2f copy) units of the library's shard plan (dbslmm_shard_plan),
        # gathered to rank 0 by one RCCL gather per step
        ud, _ = shard_units_problem(full, sig_run, world)
        plan = Plan.units(ctx, full, ud, rank)
        gather = UnitGather(full, ud, device=cdev)
    else:
        plan = Plan(ctx, prob)
    wl = plan.workload()

    outs = None
    if sigmas or sharded:   # the caller's result buffers, reused every step (as an application would)
        outs = (np.zeros((n_copies, prob.n_s)), np.zeros((n_copies, prob.n_l)),
                np.zeros((n_copies, prob.num_block), dtype=np.int32))

    def step():
        if sigmas or sharded:
            res = plan.run_multi(sig_run, out=outs)   # one Gram, len(sigmas) solves (synchronous)
            if gather:
                return gather(outs[0], outs[1])
            return res
        plan.run()
        return None

    for _ in range(args.warmup):
        step()
    plan.sync()
    sync_all()
    barrier()
    sync_all()
    plan.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    plan.sync()
    sync_all()
    barrier()
    sync_all()
    elapsed = time.perf_counter() - t0
    wl = plan.workload()                      # + the h2f iteration count of the runs
    kms, nlaunch = plan.kernel_ms()
    kms = kms * nlaunch / args.steps          # per step (a tuning step is len(h2f) runs)
    # the results of one more step, compared with the CPU reference below (every h2f solve)
    if sigmas or sharded:
        res = plan.run_multi(sig_run, out=outs)
        res = [(a.copy(), b.copy(), c.copy()) for a, b, c in res]
    else:
        plan.run()
        res = [plan.download()]
    status = res[0][2]
    if sharded:   # this rank's units only: the other blocks' status entries are not its own
        status = status[np.any(ud == rank, axis=1)]
    full_res = res if world == 1 else None    # the full problem's betas (rank 0)
    if gather:
        merged = gather(np.stack([r[0] for r in res]), np.stack([r[1] for r in res]))
        if rank == 0:
            full_res = [(bs, bl, None) for bs, bl in merged]
    st = torch.tensor([int(np.sum((status != 0) & (status != 1)))], dtype=torch.int64, device=cdev)
    if dist is not None:
        dist.all_reduce(st, op=dist.ReduceOp.SUM)

    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    snps = torch.tensor([wl["snps"]], dtype=torch.float64, device=cdev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(snps, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    total_snps = float(snps.item())
    value = total_snps * args.steps / elapsed

    n_solve = len(sigmas) if sigmas else 1
    kernels = [kernel_roofline(KERNEL_NAMES[k], float(kms[k]), wl, n_solve) for k in range(len(KERNEL_NAMES))]
    if n_gpus == 1 and not args.no_isolated and not wl.get("pcg_route"):   # (no lead group on PCG)
        # The lead group's unpack, Gram and factorisation overlap the others', so the phase spans
        # above include that contention.  One untimed plan with the lead group off times every
        # phase without it (outside the timed region; reported beside the spans, never as `value`).
        import dataclasses
        iso = Plan(ctx, dataclasses.replace(prob, opts=dict(prob.opts, lead_min=-1)))
        run_iso = (lambda: iso.run_multi(sigmas)) if sigmas else iso.run
        run_iso()
        iso.sync()
        iso.enable_timing(True)
        for _ in range(3):
            run_iso()
        iso.sync()
        iso_ms, iso_n = iso.kernel_ms()
        del iso
        for k in range(len(KERNEL_NAMES)):
            alone = kernel_roofline(KERNEL_NAMES[k], float(iso_ms[k]) * iso_n / 3, wl, n_solve)
            kernels[k].update(alone_ms=alone["ms"], alone_achieved=alone["achieved"], alone_frac=alone["frac"],
                              span_note="ms = the phase's wall span in the timed (overlapped) schedule; "
                                        "alone_* = the same phase with the lead group off (untimed run)")
    # the dominant kernel: the longest single launch class.  On the PCG route the chip-wide span
    # (init to final: hundreds of product / rows / update launches, dbslmm_pcg_block running beside
    # them on the second stream) is a composite and stays in `kernels` only.
    pcg_split = any(k["kernel"] == "dbslmm_pcg_block" and k["ms"] > 0 for k in kernels)
    dom = max((k for k in kernels if not (pcg_split and k["kernel"] == "dbslmm_pcg")), key=lambda r: r["ms"])
    traffic, tsrc = pmc_traffic(dom["kernel"], args, n_solve) if n_gpus == 1 else (None, None)
    roof = dict(bound=dom["bound"], achieved=dom["achieved"], peak=dom["peak"], unit=dom["unit"],
                frac=dom["frac"], traffic=traffic, kernel=dom["kernel"], traffic_source=tsrc,
                ms=dom["ms"], alone_ms=dom.get("alone_ms"), alone_achieved=dom.get("alone_achieved"),
                alone_frac=dom.get("alone_frac"),
                note="achieved / frac on the phase's wall span in the timed schedule (overlapped with "
                     "other phases); alone_* = the same phase timed without the lead-group overlap")

    cpu = None
    dbeta = None
    if rank == 0 and n_gpus == 1 and not args.no_cpu_baseline:
        cpu, dbeta = cpu_leg(args, prob, res, sigmas, wl)
    elif rank == 0 and full_res is not None and not args.replicas and not args.no_check:
        dbeta = dict(big_blocks=big_block_check(full, full_res, sigmas),
                     note=f"merged betas of the {n_gpus}-GPU solve (cpu_baseline is timed at N = 1 only)")
    e2e = e2e_pre
    pred = None
    if args.predict and n_gpus == 1 and rank == 0:
        pred = predict_leg(args, full, sigmas, m_b, ctx)

    if rank == 0:
        if in_proc:
            par = (f"(LD block, h2f copy) units of one problem sharded over {n_gpus} GPU(s) {devices} by the "
                   f"product's multi-device context (dbslmm_ctx_create_multi: time-model shard plan, one host "
                   f"thread per job, betas copied from each device to the caller's arrays)")
        elif args.replicas:
            par = f"{world} independent replicas (no exchange)"
        elif world > 1:
            par = (f"(LD block, h2f copy) units of one problem sharded over {world} GPU(s) by the time-model "
                   f"shard plan (dbslmm_shard_plan, one process per GPU), "
                   f"betas gathered to rank 0 by one {'RCCL' if args.dist_backend == 'nccl' else 'gloo'} "
                   f"gather per step")
        else:
            par = "1 GPU"
        line = {
            "metric": METRIC, "value": value, "unit": "SNPs/s", "n_gpus": n_gpus,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak" if args.replicas else "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (AR(1)-LD PLINK panel, seed = %s)" % ("1 + rank" if args.replicas else "1"),
            "config": {"workload": f"synthetic {args.snps} SNP x {args.n_ref} indiv, 22 chr "
                                   f"{args.pop} LD blocks, {'LMM-only' if args.lmm_only else 'DBSLMM large+small'}, "
                                   f"h2=0.5 (BASELINE configs[{args.config - 1}])", "generator": args.gen,
                       "h2f": args.h2f, "options": dict(full.opts),
                       "snps_rank0": wl["snps"], "snps_total": total_snps, "n_ref": args.n_ref,
                       "blocks_rank0": wl["blocks"], "devices": devices if world == 1 else None,
                       "gram": "exact integer dosages as FP4 (e2m1, unit block scales) on "
                               "v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation exact below 2^24, "
                               "fp64 epilogue",
                       "solve": ("Jacobi-PCG (the reference's PCGv, scr/dbslmmfit.cpp:629-678) on the joint "
                                 "per-block matrix streamed from the exact integer Gram, every h2f copy a "
                                 "right-hand side, each block and copy until |r| <= %g lambda_min |x| "
                                 "(%d iterations for the slowest block)" % (1e-12, wl["pcg_iters"]))
                       if wl.get("pcg_route") else "fp64 Cholesky of the joint per-block matrix" + (
                           "; h2f: tiled blocks factored once (base h2f), the other h2f solves by "
                           + ("%d Chebyshev iterations on that factor" % wl["cheb_iters"]
                              if "h2f_iter=1" in [o.replace(" ", "") for o in args.opt] else
                              "CG preconditioned by that factor, each block until |r| <= cheb_tol "
                              "lambda_min |x| (at most %d iterations)" % wl["cheb_iters"])
                           if wl["cheb_iters"] > 0 else ""),
                       "parallelism": par},
            "roofline": roof,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "predicted_multi_gpu": pred,
            "max_dbeta_vs_cpu_ref": dbeta,
            "status_nonzero_blocks": int(st.item()),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
