"""Deterministic synthetic PLINK panels shaped like the BASELINE configs.

* SNPs per chromosome proportional to the summed LD-block span of the population's block file
  (data/block_data/<POP>/chr*.bed, the reference's Berisa-Pickrell blocks); bp positions uniform,
  unique and sorted inside [first start, last end), so every SNP falls in exactly one block.
* allele frequency p ~ U(0.05, 0.5); two haplotypes per individual from an AR(1) latent
  Gaussian along the SNPs of each block (rho = 0.9) thresholded at Phi^-1(p); dosage = h1 + h2.
* optional missing-call rate; z ~ N(0, 1) plus one large SNP (|z| = 8) in ~1 of 20 blocks.
* GWAS n_obs = 100000, se = 1/sqrt(n_obs), nsnp = M, h2 = 0.5 -> sigma_s = h2 / M.

``make_problem`` returns the in-memory BlockProblem (bench path); ``write_plink`` writes the
files the ``dbslmm`` CLI reads (.bed/.bim/.fam, GEMMA summary for small / large SNPs, blocks).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np
from scipy.signal import lfilter
from scipy.special import ndtri

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "block_data")
BED_MAGIC = bytes([0x6C, 0x1B, 0x01])


def read_blocks(pop: str = "EUR", chroms=range(1, 23)):
    """Block files as [(chrom, start, end)], in chromosome order then file order."""
    out = []
    for c in chroms:
        with open(os.path.join(DATA, pop, f"chr{c}.bed")) as f:
            for line in f:
                t = line.split()
                if len(t) >= 3:
                    out.append((c, int(t[1]), int(t[2])))
    return out


def pack_dosages(dos: np.ndarray) -> np.ndarray:
    """int8 dosages [m, n] (0,1,2; -1 = missing) -> packed SNP-major rows [m, ceil(n/4)].

    PLINK codes (low bit first): 2 -> 00, 1 -> 10, 0 -> 11, missing -> 01 (dtpr.cpp:329-350).
    """
    m, n = dos.shape
    nb = (n + 3) // 4
    code = np.zeros((m, nb * 4), dtype=np.uint8)
    lut = np.array([3, 2, 0, 1], dtype=np.uint8)      # dosage 0,1,2 / missing(3) -> code
    d = dos.astype(np.int16)
    idx = np.where(d < 0, 3, d)                        # 0->0,1->1,2->2,missing->3
    code[:, :n] = lut[idx]                             # 0->11(3), 1->10(2), 2->00(0), miss->01(1)
    c4 = code.reshape(m, nb, 4)
    return (c4[:, :, 0] | (c4[:, :, 1] << 2) | (c4[:, :, 2] << 4) | (c4[:, :, 3] << 6)).astype(np.uint8)


@dataclass
class SynthPanel:
    n_ref: int
    blocks: list            # [(chrom, start, end)]
    chrom: np.ndarray       # per SNP
    ps: np.ndarray          # bp positions
    block: np.ndarray       # block index per SNP
    af: np.ndarray          # A1 frequency used to simulate
    bed: np.ndarray         # uint8 image incl. magic
    z: np.ndarray           # z-scores
    large: np.ndarray       # bool per SNP
    n_obs: int = 100000
    h2: float = 0.5

    @property
    def m(self) -> int:
        return len(self.ps)


def _layout(m_total, pop, chroms, rng, block_limit=None):
    """SNP positions of a synthetic panel: per chromosome a share of m_total proportional to its
    summed block span, positions uniform in the span, each SNP in the block containing it."""
    blocks = read_blocks(pop, chroms)
    if block_limit is not None:
        blocks = blocks[:block_limit]
    spans = np.array([e - s for _, s, e in blocks], dtype=np.float64)
    # SNPs per chromosome proportional to summed block span; positions uniform in the span
    chrom_ids = sorted({c for c, _, _ in blocks})
    per_chr_span = {c: spans[[i for i, b in enumerate(blocks) if b[0] == c]].sum() for c in chrom_ids}
    tot = sum(per_chr_span.values())
    alloc = {c: int(math.floor(m_total * per_chr_span[c] / tot)) for c in chrom_ids}
    rem = m_total - sum(alloc.values())
    for c in sorted(chrom_ids, key=lambda c: -per_chr_span[c])[:rem]:
        alloc[c] += 1
    chrom, ps, blk = [], [], []
    for c in chrom_ids:
        bidx = [i for i, b in enumerate(blocks) if b[0] == c]
        lo = blocks[bidx[0]][1]
        hi = max(blocks[i][2] for i in bidx)
        k = alloc[c]
        cand = np.unique(rng.integers(lo, hi, size=int(k * 1.05) + 16))
        while len(cand) < k:
            cand = np.unique(np.concatenate([cand, rng.integers(lo, hi, size=k)]))
        pos = np.sort(cand[rng.choice(len(cand), size=k, replace=False)])
        starts = np.array([blocks[i][1] for i in bidx])
        ends = np.array([blocks[i][2] for i in bidx])
        bi = np.searchsorted(starts, pos, side="right") - 1
        ok = (bi >= 0) & (pos < ends[np.clip(bi, 0, None)])
        pos, bi = pos[ok], bi[ok]          # gaps between non-contiguous blocks are dropped
        chrom.append(np.full(len(pos), c))
        ps.append(pos)
        blk.append(np.array(bidx)[bi])
    chrom = np.concatenate(chrom)
    ps = np.concatenate(ps)
    blk = np.concatenate(blk)
    return blocks, chrom, ps, blk


def block_sizes(m_total: int, pop: str = "EUR", chroms=range(1, 23), seed: int = 1,
                block_limit: int | None = None) -> np.ndarray:
    """SNPs per LD block of simulate(m_total, ..., seed) without generating genotypes."""
    blocks, _, _, blk = _layout(m_total, pop, chroms, np.random.default_rng(seed), block_limit)
    return np.bincount(blk, minlength=len(blocks))


def simulate(m_total: int, n_ref: int, pop: str = "EUR", chroms=range(1, 23), seed: int = 1,
             rho: float = 0.9, miss_rate: float = 0.0, large_every: int = 20,
             large_z: float = 8.0, n_obs: int = 100000, h2: float = 0.5,
             block_limit: int | None = None, engine: str = "numpy", device: int = 0) -> SynthPanel:
    """engine "numpy" (CPU, used by the parity fixtures) or "gpu" (libdbslmm_synth.so, same model
    with a counter-hash RNG; for the 500k-1M SNP scale configs); "none": the "gpu" panel's blocks,
    z-scores and large SNPs without genotypes (zero .bed rows, never touched: shard-plan tests)."""
    rng = np.random.default_rng(seed)
    blocks, chrom, ps, blk = _layout(m_total, pop, chroms, rng, block_limit)
    m = len(ps)
    af = rng.uniform(0.05, 0.5, size=m)
    thr = ndtri(af).astype(np.float32)
    nb = (n_ref + 3) // 4
    bed = (np.zeros if engine == "none" else np.empty)(3 + m * nb, dtype=np.uint8)
    bed[:3] = np.frombuffer(BED_MAGIC, dtype=np.uint8)
    rows = bed[3:].reshape(m, nb)
    a = np.float32(math.sqrt(1.0 - rho * rho))
    # AR(1) along the SNPs of each block, 2 haplotypes per individual
    bounds = np.flatnonzero(np.diff(blk)) + 1
    starts = np.concatenate([[0], bounds])
    ends = np.concatenate([bounds, [m]])
    chunk = 4096
    if engine == "gpu":
        _gpu_rows(rows, starts, ends, thr, n_ref, seed, rho, miss_rate, device)
        starts = ends = []
    elif engine == "none":
        starts = ends = []
    elif engine != "numpy":
        raise ValueError(f"engine {engine!r}")
    for s0, e0 in zip(starts, ends):
        for c0 in range(s0, e0, chunk):
            c1 = min(e0, c0 + chunk)
            e = rng.standard_normal((c1 - c0, 2 * n_ref), dtype=np.float32)
            if c0 == s0:                     # stationary start of the block: u0 ~ N(0, 1)
                u = np.empty_like(e)
                u[0] = e[0]
                if c1 - c0 > 1:
                    u[1:] = lfilter([a], [1.0, -rho], e[1:], axis=0, zi=(rho * e[0])[None, :])[0]
            else:
                u = lfilter([a], [1.0, -rho], e, axis=0, zi=(rho * last)[None, :])[0].astype(np.float32)
            last = u[-1].copy()
            hap = u < thr[c0:c1, None]
            dos = (hap[:, :n_ref].astype(np.int8) + hap[:, n_ref:].astype(np.int8))
            if miss_rate > 0:
                dos[rng.random(dos.shape) < miss_rate] = -1
            rows[c0:c1] = pack_dosages(dos)
    z = rng.standard_normal(m)
    large = np.zeros(m, dtype=bool)
    if large_every:
        for b in np.unique(blk):
            if rng.random() < 1.0 / large_every:
                idx = np.flatnonzero(blk == b)
                j = idx[rng.integers(len(idx))]
                large[j] = True
                z[j] = large_z * (1 if rng.random() < 0.5 else -1)
    return SynthPanel(n_ref, blocks, chrom, ps, blk, af, bed, z, large, n_obs, h2)


def _gpu_rows(rows, starts, ends, thr, n_ref, seed, rho, miss_rate, device):
    import ctypes as C
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdbslmm_synth.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built (make -C dbslmm_amd/csrc)")
    L = C.CDLL(path)
    L.dbslmm_synth_bed.argtypes = [C.c_int, C.c_int32, C.c_void_p, C.c_void_p, C.c_int32,
                                   C.c_uint64, C.c_float, C.c_float, C.c_void_p]
    L.dbslmm_synth_last_error.restype = C.c_char_p
    ptr = np.ascontiguousarray(np.concatenate([starts, ends[-1:]]).astype(np.int64))
    thr = np.ascontiguousarray(thr, dtype=np.float32)
    rc = L.dbslmm_synth_bed(device, len(starts), ptr.ctypes.data, thr.ctypes.data, n_ref, seed,
                            rho, miss_rate, rows.ctypes.data)
    if rc != 0:
        raise RuntimeError("dbslmm_synth_bed: " + L.dbslmm_synth_last_error().decode())


def make_problem(panel: SynthPanel, lmm_only: bool = False, tau: float = 0.8):
    """BlockProblem (CSR over the panel's blocks) with nsnp = M, sigma_s = h2 / M."""
    from . import BlockProblem
    nb = len(panel.blocks)
    small = ~panel.large if not lmm_only else np.ones(panel.m, dtype=bool)
    si = np.flatnonzero(small)
    s_ptr = np.zeros(nb + 1, dtype=np.int64)
    np.add.at(s_ptr, panel.block[si] + 1, 1)
    s_ptr = np.cumsum(s_ptr)
    kw = {}
    if not lmm_only:
        li = np.flatnonzero(panel.large)
        l_ptr = np.zeros(nb + 1, dtype=np.int64)
        np.add.at(l_ptr, panel.block[li] + 1, 1)
        kw = dict(l_ptr=np.cumsum(l_ptr), l_pos=li.astype(np.int32), z_l=panel.z[li])
    return BlockProblem(bed=panel.bed, n_ref=panel.n_ref, n_obs=panel.n_obs,
                        sigma_s=panel.h2 / panel.m, s_ptr=s_ptr, s_pos=si.astype(np.int32),
                        z_s=panel.z[si], tau=tau, **kw)


def write_plink(panel: SynthPanel, outdir: str, prefix: str = "ref") -> dict:
    """Write ref.{bed,bim,fam}, summ_s.txt, summ_l.txt (GEMMA 11 columns, no header), blocks."""
    os.makedirs(outdir, exist_ok=True)
    base = os.path.join(outdir, prefix)
    panel.bed.tofile(base + ".bed")
    snp = [f"rs{c}_{p}" for c, p in zip(panel.chrom, panel.ps)]
    with open(base + ".bim", "w") as f:
        for c, s, p in zip(panel.chrom, snp, panel.ps):
            f.write(f"{c}\t{s}\t0\t{p}\tA\tG\n")
    with open(base + ".fam", "w") as f:
        for i in range(panel.n_ref):
            f.write(f"id{i} id{i} 0 0 0 -9\n")
    se = 1.0 / math.sqrt(panel.n_obs)

    def summ(path, idx):
        with open(path, "w") as f:
            for j in idx:
                beta = panel.z[j] * se
                f.write(f"{panel.chrom[j]}\t{snp[j]}\t{panel.ps[j]}\t0\t{panel.n_obs}\tA\tG\t"
                        f"{panel.af[j]:.6f}\t{beta:.6e}\t{se:.6e}\t0.5\n")
    summ(os.path.join(outdir, "summ_s.txt"), np.flatnonzero(~panel.large))
    summ(os.path.join(outdir, "summ_l.txt"), np.flatnonzero(panel.large))
    with open(os.path.join(outdir, "blocks.bed"), "w") as f:
        for c, s, e in panel.blocks:
            f.write(f"chr{c}\t{s}\t{e}\n")
    return dict(ref=base, s=os.path.join(outdir, "summ_s.txt"), l=os.path.join(outdir, "summ_l.txt"),
                b=os.path.join(outdir, "blocks.bed"), nsnp=panel.m, n=panel.n_obs)
