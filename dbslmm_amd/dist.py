"""Multi-GPU solve of one problem: (LD block, h2f copy) units sharded across ranks, beta gathered
to rank 0.

The reference parallelises only over LD blocks (OpenMP `schedule(dynamic)` over batches of 60,
scr/dbslmmfit.cpp:189-220) and runs each h2f factor as its own dbslmm process
(software/DBSLMM.R:204-219); both are independent, so a multi-GPU solve needs no exchange during
compute.  One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI):

1. every rank computes the same shard plan (`shard_units`: the library's dbslmm_shard_plan, a time
   model of one MI355X -- per-block chip time of each kernel class plus the block's dependency
   chain alone; a block's h2f copies are split over devices only when its chain exceeds the fair
   share of the step);
2. each rank solves its units on its own GPU (`Plan.units`: its whole blocks in one plan, its split
   units -- all of one h2f copy -- in a single-copy plan on its own streams beside it);
3. the betas (fp64, <= 8 MB per h2f solve at 1M SNPs) are gathered to rank 0 in the original order
   -- the only collective, one `gather` of this rank's unit values per step.
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def block_cost(m: np.ndarray, n_ref: int) -> np.ndarray:
    """Cost of a block for the REFERENCE's CPU path (Gram n_ref m (m+1) + factorisation m^3 / 3):
    bench.py's CPU baseline samples blocks with it.  (The GPU shard plan uses the library's time
    model instead: shard_units.)"""
    m = np.asarray(m, dtype=np.float64)
    return n_ref * m * (m + 1) + m ** 3 / 3.0


def shard_units(m_per_block, n_ref: int, world: int, n_copies: int = 1):
    """The library's shard plan (dbslmm_shard_plan; host only, deterministic): returns
    unit_device [num_block, n_copies] (device of copy c of block b, -1 for an empty block) and the
    model's predicted step of every device in ms."""
    from . import _lib
    L = _lib.load()
    m = np.ascontiguousarray(m_per_block, dtype=np.int32)
    ud = np.zeros((m.size, n_copies), dtype=np.int32)
    ms = np.zeros(world, dtype=np.float64)
    rc = L.dbslmm_shard_plan(m.size, m.ctypes.data_as(C.c_void_p), int(n_ref), int(world), int(n_copies),
                             ud.ctypes.data_as(C.c_void_p), ms.ctypes.data_as(C.c_void_p))
    if rc != 0:
        raise _lib.DbslmmError(f"dbslmm_shard_plan failed rc={rc}")
    return ud, ms


def shard_units_problem(prob, sigmas, world: int):
    """The route-aware shard plan of a problem (dbslmm_shard_plan_problem; host only,
    deterministic): on the PCG route every block whole on one device by the PCG time model, on
    the factorisation route shard_units' plan.  Returns unit_device [num_block, len(sigmas)] and
    the model's predicted step of every device in ms."""
    from . import _lib
    L = _lib.load()
    sig = np.ascontiguousarray(sigmas, dtype=np.float64).reshape(-1)
    ud = np.zeros((prob.num_block, sig.size), dtype=np.int32)
    ms = np.zeros(world, dtype=np.float64)
    cs = prob.c_struct()
    rc = L.dbslmm_shard_plan_problem(C.byref(cs), sig.ctypes.data_as(C.c_void_p), sig.size, int(world),
                                     ud.ctypes.data_as(C.c_void_p), ms.ctypes.data_as(C.c_void_p))
    if rc != 0:
        raise _lib.DbslmmError(f"dbslmm_shard_plan_problem failed rc={rc}")
    return ud, ms


def shard_blocks(m_per_block: np.ndarray, n_ref: int, world: int) -> list[np.ndarray]:
    """Single-solve shard plan: the blocks of each rank (block order)."""
    ud, _ = shard_units(m_per_block, n_ref, world, 1)
    return [np.flatnonzero(ud[:, 0] == r).astype(np.int64) for r in range(world)]


def rank_jobs(unit_device: np.ndarray, rank: int):
    """The jobs of `rank` (the decomposition dbslmm_plan_create_units builds, multi.hip mp_build):
    [(blocks, copies)] -- first its whole blocks with every copy, then one job per h2f copy c
    holding the rank's split units of that copy."""
    ud = np.asarray(unit_device)
    K = ud.shape[1]
    whole = np.all(ud == ud[:, :1], axis=1)
    jobs = [(np.flatnonzero(whole & (ud[:, 0] == rank)), list(range(K)))]
    for c in range(K):
        jobs.append((np.flatnonzero(~whole & (ud[:, c] == rank)), [c]))
    return [j for j in jobs if j[0].size]


def unit_index(prob, unit_device: np.ndarray, rank: int):
    """Per copy c: the positions in the full [beta_s | beta_l] vector that `rank` solves."""
    ud = np.asarray(unit_device)
    n_s = prob.n_s
    out = []
    for c in range(ud.shape[1]):
        idx = []
        for b in np.flatnonzero(ud[:, c] == rank):
            idx.append(np.arange(prob.s_ptr[b], prob.s_ptr[b + 1]))
            if prob.l_ptr is not None:
                idx.append(n_s + np.arange(prob.l_ptr[b], prob.l_ptr[b + 1]))
        out.append(np.concatenate(idx).astype(np.int64) if idx else np.zeros(0, dtype=np.int64))
    return out


def sub_problem(prob, blocks: np.ndarray, compact: bool = False):
    """The BlockProblem restricted to `blocks` (kept in block order), plus the positions of its
    small / large SNPs in the full problem's beta_s / beta_l.  compact: the sub-problem gets its
    own .bed image holding only its rows (what one GPU of a sharded solve receives; the C-ABI's
    multi-device plans do the same, multi.hip)."""
    from . import BlockProblem
    s_idx = [np.arange(prob.s_ptr[b], prob.s_ptr[b + 1]) for b in blocks]
    s_idx = np.concatenate(s_idx) if s_idx else np.zeros(0, dtype=np.int64)
    s_ptr = np.concatenate([[0], np.cumsum(np.diff(prob.s_ptr)[blocks])]).astype(np.int64)
    kw = {}
    l_idx = np.zeros(0, dtype=np.int64)
    if prob.l_ptr is not None:
        li = [np.arange(prob.l_ptr[b], prob.l_ptr[b + 1]) for b in blocks]
        l_idx = np.concatenate(li) if li else np.zeros(0, dtype=np.int64)
        l_ptr = np.concatenate([[0], np.cumsum(np.diff(prob.l_ptr)[blocks])]).astype(np.int64)
        kw = dict(l_ptr=l_ptr, l_pos=prob.l_pos[l_idx], z_l=prob.z_l[l_idx])
    bed, s_pos = prob.bed, prob.s_pos[s_idx]
    if compact:
        bps = (prob.n_ref + 3) // 4
        rows = np.concatenate([s_pos, kw.get("l_pos", np.zeros(0, dtype=np.int32))])
        uniq, inv = np.unique(rows, return_inverse=True)
        body = prob.bed[3:3 + (int(uniq.max()) + 1 if uniq.size else 0) * bps].reshape(-1, bps)
        bed = np.concatenate([prob.bed[:3], body[uniq].reshape(-1)]) if uniq.size else prob.bed[:3 + bps]
        s_pos = inv[:s_pos.size].astype(np.int32)
        if "l_pos" in kw:
            kw["l_pos"] = inv[s_pos.size:].astype(np.int32)
    sub = BlockProblem(bed=bed, n_ref=prob.n_ref, n_obs=prob.n_obs, sigma_s=prob.sigma_s,
                       s_ptr=s_ptr, s_pos=s_pos, z_s=prob.z_s[s_idx], tau=prob.tau,
                       opts=dict(prob.opts), **kw)
    return sub, s_idx.astype(np.int64), l_idx.astype(np.int64)


class UnitGather:
    """Per-step gather of this rank's unit betas to rank 0 for a fixed shard plan: the index lists
    are built once; each call is ONE `gather` of a padded fp64 buffer holding, copy after copy,
    this rank's small-SNP values then its large-SNP values -- over RCCL/xGMI with the nccl backend.
    The host staging and rank 0's output arrays are allocated once and reused every step (fresh
    arrays page-faulted ~24 MB per step on rank 0); the returned arrays are views of them, valid
    until the next call."""

    def __init__(self, prob, unit_device, device="cpu"):
        import torch
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.n_s, self.n_l = prob.n_s, prob.n_l
        self.k = np.asarray(unit_device).shape[1]
        self.device = device

        def split(ixs):   # per copy: (small positions, large positions) in beta_s / beta_l
            return [(ix[ix < self.n_s], ix[ix >= self.n_s] - self.n_s) for ix in ixs]

        per_rank = [split(unit_index(prob, unit_device, r)) for r in range(self.world)]
        self.mine = per_rank[self.rank]
        self.idx = per_rank if self.rank == 0 else None
        self.width = max(1, max(sum(a.size + b.size for a, b in pr) for pr in per_rank))
        self.hbuf = torch.zeros(self.width, dtype=torch.float64)
        if device != "cpu":
            self.hbuf = self.hbuf.pin_memory()
        self.host = self.hbuf.numpy()
        self.buf = torch.zeros(self.width, dtype=torch.float64, device=device)
        self.out = None
        if self.rank == 0:
            self.out = [torch.empty_like(self.buf) for _ in range(self.world)]
            if device == "cpu":
                self.full_s = np.full((self.k, self.n_s), np.nan)
                self.full_l = np.full((self.k, self.n_l), np.nan)
            else:
                # on the GPU: the received segments are scattered on the device (one index_copy_
                # per rank and copy) and the whole result comes down in ONE copy into pinned memory,
                # instead of every rank's padded segment through the host
                self.dix = [[torch.from_numpy(np.concatenate([a, self.n_s + b])).to(device) for a, b in pr]
                            for pr in per_rank]
                self.full_dev = torch.full((self.k, self.n_s + self.n_l), float("nan"), dtype=torch.float64,
                                           device=device)
                self.full_host = torch.empty((self.k, self.n_s + self.n_l), dtype=torch.float64).pin_memory()
                fh = self.full_host.numpy()
                self.full_s, self.full_l = fh[:, :self.n_s], fh[:, self.n_s:]

    def __call__(self, beta_s, beta_l):
        """beta_s, beta_l: (k, n_s), (k, n_l) arrays holding this rank's units (the rest ignored)
        -> on rank 0 the full k pairs in the original order (None elsewhere)."""
        import torch.distributed as dist
        host, o = self.host, 0
        for c, (ixs, ixl) in enumerate(self.mine):
            host[o:o + ixs.size] = beta_s[c][ixs]
            o += ixs.size
            host[o:o + ixl.size] = beta_l[c][ixl]
            o += ixl.size
        self.buf.copy_(self.hbuf)
        dist.gather(self.buf, gather_list=self.out, dst=0)
        if self.rank != 0:
            return None
        if self.device != "cpu":
            for t, ixs in zip(self.out, self.dix):
                o = 0
                for c, ix in enumerate(ixs):
                    self.full_dev[c].index_copy_(0, ix, t[o:o + ix.numel()])
                    o += ix.numel()
            self.full_host.copy_(self.full_dev)
            return [(self.full_s[c], self.full_l[c]) for c in range(self.k)]
        for t, pr in zip(self.out, self.idx):
            v = t.numpy()
            o = 0
            for c, (ixs, ixl) in enumerate(pr):
                self.full_s[c, ixs] = v[o:o + ixs.size]
                o += ixs.size
                self.full_l[c, ixl] = v[o:o + ixl.size]
                o += ixl.size
        return [(self.full_s[c], self.full_l[c]) for c in range(self.k)]


def gather_beta(n_s: int, n_l: int, s_idx, l_idx, beta_s, beta_l, device="cpu"):
    """Gather every rank's (index, beta) to rank 0; returns the full beta_s, beta_l on rank 0
    (None elsewhere).  Shards are padded to the largest shard (one collective)."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    # encode small as index, large as n_s + index
    idx = np.concatenate([s_idx, n_s + np.asarray(l_idx, dtype=np.int64)]).astype(np.float64)
    val = np.concatenate([beta_s, beta_l]).astype(np.float64)
    cnt = torch.tensor([idx.size], dtype=torch.int64, device=device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    width = int(max(int(c.item()) for c in cnts))
    buf = torch.full((2, width), -1.0, dtype=torch.float64, device=device)
    buf[0, :idx.size] = torch.from_numpy(idx).to(device)
    buf[1, :val.size] = torch.from_numpy(val).to(device)
    out = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=out, dst=0)
    if rank != 0:
        return None, None
    full = np.full(n_s + n_l, np.nan)
    for r, t in enumerate(out):
        k = int(cnts[r].item())
        a = t[:, :k].cpu().numpy()
        full[a[0].astype(np.int64)] = a[1]
    return full[:n_s], full[n_s:]


def est_distributed(prob, solve=None, device=None, sigmas=None):
    """Solve `prob` across the ranks of the default process group; betas on rank 0.

    sigmas: h2f solves (default [prob.sigma_s]); the units are (block, copy) pairs of the shard plan.
    solve(sub_problem, sigma_list) -> [(beta_s, beta_l)] per sigma, for a test solver (the oracle);
    default = this rank's GPU through the C-ABI (one units plan, dbslmm_plan_create_units).
    Returns [(beta_s, beta_l)] per sigma on rank 0 (a single pair when sigmas is None), None
    elsewhere."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    sig = [prob.sigma_s] if sigmas is None else list(sigmas)
    K = len(sig)
    m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    ud, _ = shard_units(m, prob.n_ref, world, K)
    bs = np.zeros((K, prob.n_s))
    bl = np.zeros((K, prob.n_l))
    if solve is None:
        from . import Context, Plan
        import torch
        dev = torch.cuda.current_device() if device is None else device
        plan = Plan.units(Context(dev), prob, ud, rank)
        plan.run_multi(sig, out=(bs, bl, np.zeros((K, prob.num_block), dtype=np.int32)))
        plan.close()
    else:
        for blocks, copies in rank_jobs(ud, rank):
            sub, s_idx, l_idx = sub_problem(prob, blocks)
            for c, (s, l) in zip(copies, solve(sub, [sig[c] for c in copies])):
                bs[c, s_idx] = s
                bl[c, l_idx] = l
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    res = UnitGather(prob, ud, device=dev)(bs, bl)
    if res is None:
        return None
    return res if sigmas is not None else res[0]
