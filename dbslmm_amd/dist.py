"""Multi-GPU solve of one problem: LD blocks sharded across ranks, beta gathered to rank 0.

The reference parallelises only over LD blocks (OpenMP `schedule(dynamic)` over batches of 60,
scr/dbslmmfit.cpp:191-220); blocks are independent, so a multi-GPU solve needs no exchange
during compute.  One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI):

1. every rank computes the same longest-processing-time assignment of blocks to ranks
   (cost ~ n_ref*m^2 for the Gram + m^3/3 for the factorisation);
2. each rank solves its sub-problem on its own GPU (a BlockProblem restricted to its blocks);
3. the betas (fp64, <= 8 MB at 1M SNPs) are gathered to rank 0 in the original order -- the only
   collective, one padded `gather` of [index, beta] pairs.
"""
from __future__ import annotations

import heapq

import numpy as np


def block_cost(m: np.ndarray, n_ref: int) -> np.ndarray:
    m = np.asarray(m, dtype=np.float64)
    return n_ref * m * (m + 1) + m ** 3 / 3.0


def shard_blocks(m_per_block: np.ndarray, n_ref: int, world: int) -> list[np.ndarray]:
    """LPT: blocks sorted by cost, each to the least-loaded rank.  Deterministic."""
    cost = block_cost(m_per_block, n_ref)
    order = np.lexsort((np.arange(len(cost)), -cost))
    heap = [(0.0, r) for r in range(world)]
    owned = [[] for _ in range(world)]
    for b in order:
        if m_per_block[b] == 0:
            continue
        load, r = heapq.heappop(heap)
        owned[r].append(int(b))
        heapq.heappush(heap, (load + cost[b], r))
    return [np.array(sorted(o), dtype=np.int64) for o in owned]


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


class ShardGather:
    """Per-step gather of this rank's betas to rank 0 for a fixed shard layout: the counts and
    the padded width are exchanged once; each call is ONE `gather` of a [k, width] fp64 buffer
    (k = solves per step, e.g. the h2f factors) -- over RCCL/xGMI with the nccl backend."""

    def __init__(self, n_s, n_l, s_idx, l_idx, k=1, device="cpu"):
        import torch
        import torch.distributed as dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.n_s, self.n_l, self.k, self.device = n_s, n_l, k, device
        self.idx = np.concatenate([s_idx, n_s + np.asarray(l_idx, dtype=np.int64)]).astype(np.int64)
        cnt = torch.tensor([self.idx.size], dtype=torch.int64, device=device)
        cnts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(cnts, cnt)
        self.cnts = [int(c.item()) for c in cnts]
        self.width = max(1, max(self.cnts))
        self.buf = torch.zeros((k, self.width), dtype=torch.float64, device=device)
        self.out = [torch.empty_like(self.buf) for _ in range(self.world)] if self.rank == 0 else None
        idx = torch.full((self.width,), -1, dtype=torch.int64, device=device)
        idx[:self.idx.size] = torch.from_numpy(self.idx).to(device)
        self.idxs = [torch.empty_like(idx) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(idx, gather_list=self.idxs, dst=0)
        if self.rank == 0:
            self.idxs = [t[:c].cpu().numpy() for t, c in zip(self.idxs, self.cnts)]

    def __call__(self, betas):
        """betas: k pairs (beta_s, beta_l) of this rank's shard -> on rank 0 the full k pairs in
        the original order (None elsewhere)."""
        import torch
        import torch.distributed as dist
        host = np.zeros((self.k, self.width))
        for c, (bs, bl) in enumerate(betas):
            host[c, :self.idx.size] = np.concatenate([bs, bl])
        self.buf.copy_(torch.from_numpy(host))
        dist.gather(self.buf, gather_list=self.out, dst=0)
        if self.rank != 0:
            return None
        full = np.full((self.k, self.n_s + self.n_l), np.nan)
        for t, ix in zip(self.out, self.idxs):
            full[:, ix] = t[:, :ix.size].cpu().numpy()
        return [(full[c, :self.n_s], full[c, self.n_s:]) for c in range(self.k)]


def est_distributed(prob, solve=None, device=None):
    """Solve `prob` across the ranks of the default process group; beta on rank 0.

    solve(sub_problem) -> (beta_s, beta_l, status); default = this rank's GPU through the C-ABI.
    """
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    m = np.diff(prob.s_ptr) + (np.diff(prob.l_ptr) if prob.l_ptr is not None else 0)
    shards = shard_blocks(m, prob.n_ref, world)
    sub, s_idx, l_idx = sub_problem(prob, shards[rank])
    if solve is None:
        from . import DBSLMMFIT
        import torch
        dev = torch.cuda.current_device() if device is None else device
        solve = DBSLMMFIT(dev).est
    bs, bl, _ = solve(sub)
    dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
    return gather_beta(prob.n_s, prob.n_l, s_idx, l_idx, bs, bl, device=dev)
