#!/usr/bin/env python3
"""Benchmark of the per-LD-block effect-size solver (DBSLMMFIT::est hot path) on MI355X.

One "step" = one full solve of the workload with the packed genotypes already resident in HBM:
2-bit unpack + per-SNP stats -> joint i8-MFMA Gram per LD block -> fp64 Cholesky + solves ->
beta in HBM.  Default workload = the configuration BASELINE.json's metric is quoted on
("1M SNP x 10k indiv"), configs[3]: synthetic 1M SNPs x 10k individuals over the 22-chromosome
EUR LD blocks, DBSLMM (large + small effects), h2 = 0.5 tuned over h2f in {0.8, 1.0, 1.2} (one
Gram + three factorisations and solves per step).  --config 2 is the small configs[1] case.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Multi-GPU: LD blocks are independent, so each rank solves its own shard (its own synthetic
panel of the same shape, seed = rank) with no data-path collective -> weak scaling; the job
value is the SNPs of all ranks / the max-over-ranks time.  Rank 0 prints ONE JSON line.
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
PEAK_I8_TOPS = 5000.0        # dense i8 MFMA = 2x the ~2.5 PF dense bf16 rate
PEAK_F64_TFLOPS = 78.6       # fp64 (vector = matrix rate on gfx950)

# BASELINE.json configs (1-based): synthetic panels; 3-5 are the scale configs
CONFIGS = {
    2: dict(snps=50000, n_ref=2000, pop="EUR", lmm_only=False, gen="numpy"),
    3: dict(snps=500000, n_ref=5000, pop="EUR", lmm_only=False, gen="gpu"),
    4: dict(snps=1000000, n_ref=10000, pop="EUR", lmm_only=False, gen="gpu", h2f="0.8,1,1.2"),
    5: dict(snps=1000000, n_ref=10000, pop="AFR", lmm_only=True, gen="gpu"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    a = ap.parse_args()
    for k, v in CONFIGS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    a.h2f = [float(x) for x in a.h2f.split(",")] if a.h2f else None
    return a


def kernel_roofline(name, ms, wl, n_solve=1):
    """ms = the kernel's time per step; n_solve = solves per step (h2f factors)."""
    s = ms * 1e-3
    if name == "dbslmm_unpack_stats":
        b = wl["unpack_read_bytes"] + wl["unpack_write_bytes"]
        a = b / s / 1e9
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms)
    if name == "dbslmm_gram_i8":
        a = wl["gram_ops_alg"] / s / 1e12
        return dict(kernel=name, bound="mfma", achieved=a, peak=PEAK_I8_TOPS, unit="TFLOP/s",
                    frac=a / PEAK_I8_TOPS, algorithmic=wl["gram_ops_alg"], ms=ms,
                    executed_tops=wl["gram_ops_exec"] / s / 1e12,
                    note="int8 ops (2/MAC), algorithmic sum_b n_ref*m_b*(m_b+1); executed = "
                         "padded tiles x padded individuals")
    if name == "dbslmm_trsv":
        # h2f Chebyshev iterations: per iteration one forward + one backward substitution, each
        # streaming the base copy's factor once (HBM-bound; chained over 64-row tiles)
        b = 2.0 * wl["trsv_bytes"] * wl["cheb_iters"]
        a = b / s / 1e9 if s > 0 else 0.0
        return dict(kernel=name, bound="hbm", achieved=a, peak=PEAK_HBM_GBS, unit="GB/s",
                    frac=a / PEAK_HBM_GBS, algorithmic=b, ms=ms,
                    note="factor bytes read by the %d forward + backward substitutions of h2f tuning "
                         "(iterations on the base copy's factor; chain- and streaming-bound, ~5.7 us per 64-row step of the largest block)"
                         % wl["cheb_iters"])
    if name == "dbslmm_tchol" and wl["cheb_iters"] > 0:
        n_solve = 1     # h2f: only the base copy of the tiled blocks is factored
    fl = n_solve * {"dbslmm_chol_large": wl["chol_flops_large"], "dbslmm_chol_small": wl["chol_flops_small"],
                    "dbslmm_tchol": wl["chol_flops_tiled"]}[name]
    a = fl / s / 1e12 if s > 0 else 0.0
    return dict(kernel=name, bound="mfma", achieved=a, peak=PEAK_F64_TFLOPS, unit="TFLOP/s",
                frac=a / PEAK_F64_TFLOPS, algorithmic=fl, ms=ms,
                note="fp64 flops sum_b m^3/3 + 2m^2 over its blocks vs the fp64 MFMA peak"
                     + ("; multi-workgroup sequence, %d launches" % wl["tiled_launches"]
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


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world)
    else:
        torch.cuda.set_device(0)

    from dbslmm_amd import Context, KERNEL_NAMES, Plan, synth

    def barrier():
        if dist is not None:
            dist.barrier()

    panel = synth.simulate(args.snps, args.n_ref, pop=args.pop, seed=1 + rank, engine=args.gen,
                           device=local if world > 1 else 0)
    prob = synth.make_problem(panel, lmm_only=args.lmm_only)
    ctx = Context(local if world > 1 else 0)
    plan = Plan(ctx, prob)
    wl = plan.workload()

    sigmas = [prob.sigma_s * f for f in args.h2f] if args.h2f else None

    def step():
        if sigmas:
            plan.run_multi(sigmas)      # one Gram, len(sigmas) solves (synchronous)
        else:
            plan.run()

    for _ in range(args.warmup):
        step()
    plan.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    plan.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    plan.sync()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    wl = plan.workload()                      # + the h2f iteration count of the runs
    kms, nlaunch = plan.kernel_ms()
    kms = kms * nlaunch / args.steps          # per step (a tuning step is len(h2f) runs)
    if sigmas:   # every h2f solve of the last step is compared with the CPU reference
        res = plan.run_multi(sigmas)
    else:
        res = [plan.download()]
    status = res[0][2]

    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    snps = torch.tensor([wl["snps"]], dtype=torch.float64, device="cuda")
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(snps, op=dist.ReduceOp.SUM)
    elapsed = float(t.item())
    total_snps = float(snps.item())
    value = total_snps * args.steps / elapsed

    n_solve = len(sigmas) if sigmas else 1
    kernels = [kernel_roofline(KERNEL_NAMES[k], float(kms[k]), wl, n_solve) for k in range(len(KERNEL_NAMES))]
    dom = max(kernels, key=lambda r: r["ms"])
    traffic, tsrc = pmc_traffic(dom["kernel"], args, n_solve)
    roof = dict(bound=dom["bound"], achieved=dom["achieved"], peak=dom["peak"], unit=dom["unit"],
                frac=dom["frac"], traffic=traffic, kernel=dom["kernel"], traffic_source=tsrc)

    cpu = None
    dbeta = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        blas = O.use_blas(True)
        thr = args.cpu_threads or min(16, os.cpu_count() or 1)
        from dbslmm_amd.dist import sub_problem
        # bounded sample: whole workload repeated if it fits the budget, else blocks in a fixed
        # random order until the budget is spent (beta compared on exactly those blocks)
        from dbslmm_amd.dist import block_cost
        nblk = len(prob.s_ptr) - 1
        m_b = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
        cost = block_cost(m_b, prob.n_ref)
        order = np.random.default_rng(0).permutation(nblk)
        target = min(cost.sum(), 2e10)            # ~0.1-1 s of 16-thread CPU work per call
        chunks, cur, acc = [], [], 0.0
        skipped = int(np.sum(cost > 5 * target))
        for b in order:
            if cost[b] > 5 * target:           # keeps one call bounded (largest blocks skipped)
                continue
            cur.append(b)
            acc += cost[b]
            if acc >= target:
                chunks.append(np.sort(np.array(cur)))
                cur, acc = [], 0.0
        if cur:
            chunks.append(np.sort(np.array(cur)))
        reps, tc, snps_done = 0, 0.0, 0
        cmp_got, cmp_ref = [[] for _ in res], [[] for _ in res]
        sig_list = sigmas if sigmas else [prob.sigma_s]
        full_once = False
        i = 0
        while tc < args.cpu_seconds and reps < 50:
            if i >= len(chunks):
                full_once, i = True, 0
            blocks = chunks[i]
            i += 1
            sub, s_idx, l_idx = sub_problem(prob, blocks)
            c0 = time.perf_counter()
            outs = [O.est(sub.bed, sub.n_ref, sub.n_obs, sg, sub.s_ptr, sub.s_pos, sub.z_s,
                          sub.l_ptr, sub.l_pos, sub.z_l, tau=prob.tau, method="pcg", threads=thr)
                    for sg in sig_list]      # the reference runs dbslmm once per h2f factor
            tc += time.perf_counter() - c0
            snps_done += len(s_idx) + len(l_idx)
            if not full_once:
                for c, (rs, rl, _, _) in enumerate(outs):
                    cmp_ref[c].append(np.concatenate([rs, rl]))
                    cmp_got[c].append(np.concatenate([res[c][0][s_idx], res[c][1][l_idx]]))
            if i >= len(chunks):
                reps += 1
        what = (f"full workload x{reps}+" if reps else
                f"{snps_done} of {int(wl['snps'])} SNPs (random block subset"
                f"{f', {skipped} largest blocks excluded' if skipped else ''})")
        cpu = dict(value=snps_done / tc, unit="SNPs/s", cores=thr, kind="port",
                   sample=f"{what} in {tc:.1f} s, {len(sig_list)} solve(s) per SNP as on the GPU: "
                          f"C restatement of the reference "
                          f"(byte-wise readSNPIm, N-1 standardise, {'OpenBLAS dsyrk/dgemm/dgemv' if blas else 'plain-loop Gram'}, "
                          f"Jacobi-PCG tol 1e-7), OpenMP over blocks x{thr}, BLAS 1 thread")
        mx, nw, ncmp = 0.0, 0.0, 0
        for c in range(len(res)):
            ref = np.concatenate(cmp_ref[c])
            got = np.concatenate(cmp_got[c])
            ok = np.isfinite(ref)
            d = float(np.max(np.abs(got[ok] - ref[ok])))
            mx, nw = max(mx, d), max(nw, d / float(np.max(np.abs(ref[ok]))))
            ncmp += int(ok.sum())
        dbeta = dict(max_abs=mx, normwise=nw, snps_compared=ncmp,
                     vs="CPU reference-faithful PCG (oracle), every h2f solve" if sigmas else
                        "CPU reference-faithful PCG (oracle)")

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "SNPs/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (AR(1)-LD PLINK panel, seed = 1 + rank)",
            "config": {"workload": f"synthetic {args.snps} SNP x {args.n_ref} indiv, 22 chr "
                                   f"{args.pop} LD blocks, {'LMM-only' if args.lmm_only else 'DBSLMM large+small'}, "
                                   f"h2=0.5 (BASELINE configs[{args.config - 1}])", "generator": args.gen,
                       "h2f": args.h2f,
                       "snps_per_gpu": wl["snps"], "n_ref": args.n_ref, "blocks": wl["blocks"],
                       "gram": "exact int8 dosages on v_mfma_i32_32x32x32_i8, fp64 epilogue",
                       "solve": "fp64 Cholesky of the joint per-block matrix" + (
                           "; h2f: tiled blocks factored once (base h2f), the other h2f solves by "
                           "%d Chebyshev iterations on that factor" % wl["cheb_iters"]
                           if wl["cheb_iters"] > 0 else ""),
                       "parallelism": f"ld-block shards x{world}"},
            "roofline": roof,
            "kernels": kernels,
            "cpu_baseline": cpu,
            "max_dbeta_vs_cpu_ref": dbeta,
            "status_nonzero_blocks": int(np.sum((status != 0) & (status != 1))),
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
