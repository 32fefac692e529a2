"""Determinism / ordering probe (round 4): does a config's solve change between runs?

The pipeline is deterministic (fixed k order in every reduction, no atomics on values), so every
run of one problem must give bit-identical betas.  A missing dependency between streams, or a
null-stream memset of plan_create still running under the first run, shows up as a run whose
betas differ from the steady state.  Prints one JSON line per phase; mismatching blocks are
named with their size and normwise difference.

  python tools/race_probe.py --config 3 --fresh 6 --reruns 100
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {2: (50_000, 2_000, "EUR", False), 3: (500_000, 5_000, "EUR", False),
           4: (1_000_000, 10_000, "EUR", False), 5: (1_000_000, 10_000, "AFR", True)}


def memset_probe(gib: float) -> dict:
    """Host time of hipMemset on a large buffer: ~0 means asynchronous to the host."""
    hip = C.CDLL("libamdhip64.so")
    p = C.c_void_p()
    n = int(gib * (1 << 30))
    assert hip.hipMalloc(C.byref(p), C.c_size_t(n)) == 0
    hip.hipMemset(p, 1, C.c_size_t(n))     # (first use: runtime / blit kernel set-up)
    hip.hipDeviceSynchronize()
    t0 = time.perf_counter()
    hip.hipMemset(p, 0, C.c_size_t(n))
    t1 = time.perf_counter()
    hip.hipDeviceSynchronize()
    t2 = time.perf_counter()
    hip.hipFree(p)
    return {"memset_gib": gib, "host_return_ms": (t1 - t0) * 1e3, "until_sync_ms": (t2 - t0) * 1e3}


def diff_blocks(prob, ref, got):
    bs0, bl0, _ = ref
    bs1, bl1, _ = got
    m_s = np.diff(prob.s_ptr)
    m_l = np.diff(prob.l_ptr) if prob.l_ptr is not None else np.zeros_like(m_s)
    out = []
    for b in range(prob.num_block):
        s0, s1 = prob.s_ptr[b], prob.s_ptr[b + 1]
        a = [bs0[s0:s1]]
        c = [bs1[s0:s1]]
        if prob.l_ptr is not None:
            l0, l1 = prob.l_ptr[b], prob.l_ptr[b + 1]
            a.append(bl0[l0:l1])
            c.append(bl1[l0:l1])
        a = np.concatenate(a)
        c = np.concatenate(c)
        if a.size and not np.array_equal(a, c, equal_nan=True):
            d = float(np.max(np.abs(a - c)) / max(np.max(np.abs(a)), 1e-300))
            out.append((b, int(m_s[b] + m_l[b]), d))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--fresh", type=int, default=6)
    ap.add_argument("--reruns", type=int, default=100)
    ap.add_argument("--memset-gib", type=float, default=4.0)
    ap.add_argument("--opts", default="{}")
    ap.add_argument("--lib", default=None, help="another build of the library (A/B)")
    ap.add_argument("--abi", type=int, default=None, help="its ABI version")
    args = ap.parse_args()
    if args.memset_gib > 0:
        print(json.dumps(memset_probe(args.memset_gib)), flush=True)
    from dbslmm_amd import _lib
    if args.lib:
        if args.abi is not None:
            _lib.ABI_VERSION = args.abi
        _lib.load(os.path.abspath(args.lib))
    print(json.dumps({"lib": args.lib or _lib.LIB_PATH}), flush=True)
    from dbslmm_amd import Context, Plan, synth
    snps, n_ref, pop, lmm = CONFIGS[args.config]
    panel = synth.simulate(snps, n_ref, pop=pop, seed=1, engine="gpu")
    prob = synth.make_problem(panel, lmm_only=lmm)
    prob.opts = json.loads(args.opts)
    del panel
    ctx = Context(0)
    # steady state: the second run of one plan
    plan = Plan(ctx, prob)
    plan.run()
    first = plan.download()
    plan.run()
    ref = plan.download()
    d = diff_blocks(prob, ref, first)
    print(json.dumps({"phase": "first_vs_second", "mismatch_blocks": len(d), "worst": d[:8]}), flush=True)
    bad = []
    for r in range(args.reruns):
        plan.run()
        got = plan.download()
        d = diff_blocks(prob, ref, got)
        if d:
            bad.append((r, d[:4]))
    print(json.dumps({"phase": "reruns", "runs": args.reruns, "bad_runs": len(bad), "first_bad": bad[:4]}),
          flush=True)
    plan.close()
    badf = []
    for r in range(args.fresh):
        pl = Plan(ctx, prob)
        pl.run()
        got = pl.download()
        pl.close()
        d = diff_blocks(prob, ref, got)
        if d:
            badf.append((r, len(d), d[:4]))
    print(json.dumps({"phase": "fresh_plans", "plans": args.fresh, "bad": len(badf), "first_bad": badf[:4]}),
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
