"""dbslmm_amd -- MI355X-native per-LD-block effect-size solver of DBSLMM.

Python front-end over the C-ABI library ``libdbslmm_hip.so`` (include/dbslmm_hip.h).  The
entry points mirror the reference operator interface (fboehm/DBSLMM, scr/dbslmmfit.hpp):

* ``DBSLMMFIT.est(...)``  -- DBSLMMFIT::est, both overloads (dbslmmfit.hpp:38-66): large +
  small effects, or LMM-only when no large SNPs are given.
* ``Plan``                -- the same problem kept resident in HBM for repeated solves.
* ``bed_maf``             -- the MAF pass of IO::readBim (dtpr.cpp:93-102).
* ``read_snp_std``        -- IO::readSNPIm + SNPPROC::nomalizeVec for a list of rows.

All compute runs on the GPU through the HIP library; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import (WORKLOAD_LEN, BLOCK_EMPTY, BLOCK_MONOMORPHIC, BLOCK_NOT_CONVERGED, BLOCK_NOT_PD,
                   BLOCK_OK, KERNEL_NAMES, SOLVER_AUTO, SOLVER_FACTOR, SOLVER_PCG, DbslmmError)

__all__ = ["Context", "Plan", "DBSLMMFIT", "BlockProblem", "bed_maf", "read_snp_std", "valid_blocks",
           "DbslmmError", "BLOCK_OK", "BLOCK_EMPTY", "BLOCK_NOT_PD", "BLOCK_MONOMORPHIC",
           "BLOCK_NOT_CONVERGED", "KERNEL_NAMES", "SOLVER_AUTO", "SOLVER_FACTOR", "SOLVER_PCG"]


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Context:
    """One HIP device (dbslmm_ctx_create), or several (a list of ordinals, repeats allowed:
    dbslmm_ctx_create_multi -- every plan's LD blocks are sharded over the devices)."""

    def __init__(self, device=0):
        self.lib = _lib.load()
        h = C.c_void_p()
        if isinstance(device, (list, tuple)):
            ids = np.ascontiguousarray(device, dtype=np.int32)
            rc = self.lib.dbslmm_ctx_create_multi(len(ids), _ptr(ids), C.byref(h))
        else:
            rc = self.lib.dbslmm_ctx_create(int(device), C.byref(h))
        if rc != 0:
            raise DbslmmError(f"dbslmm_ctx_create(device={device}) failed rc={rc}")
        self.h = h
        self.device = device

    @property
    def num_devices(self) -> int:
        return int(self.lib.dbslmm_ctx_num_devices(self.h))

    def cache_bed(self, bed):
        """Keep a device copy of this .bed image (dbslmm_ctx_cache_bed); bed_maf / plan_create on
        the same array then skip their upload (a plan reads the cached image in place).  The
        array is matched by address and length only: do not modify it while it is cached (call
        cache_bed again after a change).  None releases it."""
        if bed is None:
            self._cached_bed = None
            self.check(self.lib.dbslmm_ctx_cache_bed(self.h, None, 0), "ctx_cache_bed")
            return
        b = np.ascontiguousarray(bed, dtype=np.uint8)
        self.check(self.lib.dbslmm_ctx_cache_bed(self.h, _ptr(b), b.size), "ctx_cache_bed")
        self._cached_bed = b       # the host range must stay alive and unchanged

    def check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.dbslmm_last_error(self.h).decode(errors="replace")
            raise DbslmmError(f"{what} failed rc={rc}: {msg}")

    def close(self):
        if self.h:
            self.lib.dbslmm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class BlockProblem:
    """Flat form of DBSLMMFIT::est's arguments (see include/dbslmm_hip.h dbslmm_problem)."""
    bed: np.ndarray            # uint8 .bed image incl. magic
    n_ref: int
    n_obs: int
    sigma_s: float
    s_ptr: np.ndarray          # int64 [num_block+1]
    s_pos: np.ndarray          # int32 bed rows
    z_s: np.ndarray            # float64
    l_ptr: np.ndarray | None = None
    l_pos: np.ndarray | None = None
    z_l: np.ndarray | None = None
    tau: float = 0.8
    # dbslmm_options (path-selection thresholds; missing keys = the library defaults):
    # tiled_min, gram_big_min, gram_huge_min, h2f_mode (0 auto / 1 merged), cheb_tol, lead_min,
    # ..., solver (0 auto / 1 factorisation / 2 PCG), pcg_tol, pcg_maxit
    opts: dict = field(default_factory=dict)

    def __post_init__(self):
        self.bed = np.ascontiguousarray(self.bed, dtype=np.uint8)
        self.s_ptr = np.ascontiguousarray(self.s_ptr, dtype=np.int64)
        self.s_pos = np.ascontiguousarray(self.s_pos, dtype=np.int32)
        self.z_s = np.ascontiguousarray(self.z_s, dtype=np.float64)
        if self.l_ptr is not None:
            self.l_ptr = np.ascontiguousarray(self.l_ptr, dtype=np.int64)
            self.l_pos = np.ascontiguousarray(self.l_pos, dtype=np.int32)
            self.z_l = np.ascontiguousarray(self.z_l, dtype=np.float64)
        nb = len(self.s_ptr) - 1
        if self.l_ptr is not None and len(self.l_ptr) != nb + 1:
            raise ValueError("s_ptr and l_ptr must have the same number of blocks")

    @property
    def num_block(self) -> int:
        return len(self.s_ptr) - 1

    @property
    def n_s(self) -> int:
        return int(self.s_ptr[-1])

    @property
    def n_l(self) -> int:
        return 0 if self.l_ptr is None else int(self.l_ptr[-1])

    def c_struct(self) -> _lib.Problem:
        unknown = set(self.opts) - {f[0] for f in _lib.Options._fields_}
        if unknown:
            raise ValueError(f"unknown dbslmm_options fields: {sorted(unknown)}")
        self._opts = _lib.Options(**self.opts)     # kept alive with the problem
        return _lib.Problem(
            _ptr(self.bed), self.bed.size, self.n_ref, self.n_obs, self.sigma_s, self.tau,
            self.num_block, _ptr(self.s_ptr), _ptr(self.s_pos), _ptr(self.z_s),
            _ptr(self.l_ptr), _ptr(self.l_pos), _ptr(self.z_l), C.pointer(self._opts))


class Plan:
    """A BlockProblem resident in HBM (dbslmm_plan_*)."""

    def __init__(self, ctx: Context, prob: BlockProblem):
        self.ctx, self.prob = ctx, prob
        self._cs = prob.c_struct()          # keep the struct (and arrays) alive
        h = C.c_void_p()
        ctx.check(ctx.lib.dbslmm_plan_create(ctx.h, C.byref(self._cs), C.byref(h)), "plan_create")
        self.h = h

    @classmethod
    def units(cls, ctx: Context, prob: BlockProblem, unit_device, device_index: int):
        """dbslmm_plan_create_units: the (block, h2f copy) units of `prob` that a shard plan
        (dist.shard_units -> unit_device [num_block, n_copies]) gives device `device_index`, on
        this single-device context.  run_multi(sigmas) with len(sigmas) == n_copies writes only
        those units' entries of the full-size outputs."""
        self = cls.__new__(cls)
        self.ctx, self.prob = ctx, prob
        ud = np.ascontiguousarray(unit_device, dtype=np.int32)
        if ud.ndim != 2 or ud.shape[0] != prob.num_block:
            raise ValueError("unit_device: [num_block, n_copies]")
        self._cs = prob.c_struct()
        self._ud = ud
        h = C.c_void_p()
        ctx.check(ctx.lib.dbslmm_plan_create_units(ctx.h, C.byref(self._cs), ud.shape[1], _ptr(ud),
                                                   int(device_index), C.byref(h)), "plan_create_units")
        self.h = h
        return self

    def run(self):
        self.ctx.check(self.ctx.lib.dbslmm_plan_run(self.h), "plan_run")

    def sync(self):
        self.ctx.check(self.ctx.lib.dbslmm_plan_sync(self.h), "plan_sync")

    def set_sigma(self, sigma_s: float):
        self.ctx.check(self.ctx.lib.dbslmm_plan_set_sigma(self.h, float(sigma_s)), "plan_set_sigma")

    def run_multi(self, sigmas, out=None):
        """h2f tuning: one unpack + Gram, one solve per sigma_s -> [(beta_s, beta_l, status)].
        out: optional (beta_s, beta_l, status) arrays of shapes (n, n_s), (n, n_l), (n, num_block)
        to write into (a caller that solves repeatedly reuses its buffers)."""
        p = self.prob
        sig = np.ascontiguousarray(sigmas, dtype=np.float64)
        n = len(sig)
        if out is not None:
            bs, bl, st = out
            if (bs.shape != (n, p.n_s) or bl.shape != (n, p.n_l) or st.shape != (n, p.num_block)
                    or bs.dtype != np.float64 or bl.dtype != np.float64 or st.dtype != np.int32
                    or not all(a.flags.c_contiguous for a in out)):
                raise ValueError("out: C-contiguous float64 (n, n_s), (n, n_l) and int32 (n, num_block)")
        else:
            bs = np.zeros((n, p.n_s))
            bl = np.zeros((n, p.n_l))
            st = np.zeros((n, p.num_block), dtype=np.int32)
        self.ctx.check(self.ctx.lib.dbslmm_plan_run_multi(self.h, _ptr(sig), n, _ptr(bs), _ptr(bl),
                                                          _ptr(st)), "plan_run_multi")
        return [(bs[i], bl[i], st[i]) for i in range(n)]

    def enable_timing(self, on: bool = True):
        self.ctx.check(self.ctx.lib.dbslmm_plan_enable_timing(self.h, int(on)), "plan_enable_timing")

    def kernel_ms(self):
        out = np.zeros(len(KERNEL_NAMES))
        n = np.zeros(1, dtype=np.int32)
        self.ctx.check(self.ctx.lib.dbslmm_plan_kernel_ms(self.h, _ptr(out), _ptr(n)), "plan_kernel_ms")
        return out, int(n[0])

    def workload(self) -> dict:
        w = np.zeros(WORKLOAD_LEN)
        self.ctx.check(self.ctx.lib.dbslmm_plan_workload(self.h, _ptr(w)), "plan_workload")
        keys = ("snps", "unpack_read_bytes", "unpack_write_bytes", "gram_ops_alg",
                "gram_ops_exec", "chol_flops_large", "blocks", "gram_tiles", "chol_flops_small",
                "blocks_large", "chol_flops_tiled", "blocks_tiled", "tiled_launches", "trsv_bytes",
                "cheb_iters", "cheb_base", "h2f_pass_bytes", "pcg_route", "pcg_iters", "pcg_chip_bytes",
                "pcg_partial_bytes", "pcg_block_bytes")
        return dict(zip(keys, w.tolist()))

    def block_iters(self) -> np.ndarray:
        """PCG iterations of each block in the latest run (dbslmm_plan_block_iters; 0: empty block
        or the factorisation route)."""
        out = np.zeros(max(1, self.prob.num_block), dtype=np.int32)
        self.ctx.check(self.ctx.lib.dbslmm_plan_block_iters(self.h, _ptr(out)), "plan_block_iters")
        return out[:self.prob.num_block]

    def shard_info(self) -> np.ndarray:
        """Device index (in the context's device order) solving each block; -1 = empty block."""
        out = np.zeros(self.prob.num_block, dtype=np.int32)
        self.ctx.check(self.ctx.lib.dbslmm_plan_shard_info(self.h, _ptr(out)), "plan_shard_info")
        return out

    def block_matrix(self, block: int, copy: int = 0) -> np.ndarray:
        """Diagnostics (dbslmm_plan_block_matrix): block `block`'s ld x ld working matrix of
        factorisation copy `copy` after the last run -- Sigma after a debug_stop = 1 run, the
        factor (strict lower L, row m = L^-1 z) after a full run of a tiled block."""
        ld = C.c_int32()
        self.ctx.check(self.ctx.lib.dbslmm_plan_block_matrix(self.h, int(block), int(copy), None,
                                                             C.byref(ld)), "plan_block_matrix")
        out = np.empty((ld.value, ld.value))
        self.ctx.check(self.ctx.lib.dbslmm_plan_block_matrix(self.h, int(block), int(copy), _ptr(out),
                                                             None), "plan_block_matrix")
        return out

    def download(self):
        p = self.prob
        bs = np.zeros(p.n_s)
        bl = np.zeros(p.n_l)
        st = np.zeros(p.num_block, dtype=np.int32)
        self.ctx.check(self.ctx.lib.dbslmm_plan_download(self.h, _ptr(bs), _ptr(bl), _ptr(st)),
                       "plan_download")
        return bs, bl, st

    def variance(self, test_bed: np.ndarray, indicator, s_pos, l_pos=None) -> np.ndarray:
        """Test-set variance diags (the variance.txt matrix of DBSLMMFIT::est,
        scr/dbslmmfit.cpp:116,242) of the last run: n_test x num_block.  s_pos / l_pos = each
        small / large SNP's row in the test .bed (calcBlock's test_info_*_block[i].pos)."""
        tb = np.ascontiguousarray(test_bed, dtype=np.uint8)
        ind = np.ascontiguousarray(indicator, dtype=np.int32)
        sp = np.ascontiguousarray(s_pos, dtype=np.int32)
        lp = None if l_pos is None else np.ascontiguousarray(l_pos, dtype=np.int32)
        if sp.size != self.prob.n_s or (self.prob.n_l and (lp is None or lp.size != self.prob.n_l)):
            raise ValueError("test s_pos / l_pos must align with the plan's small / large SNPs")
        n_test = int((ind != 0).sum())
        out = np.zeros(n_test * self.prob.num_block)
        nt = np.zeros(1, dtype=np.int32)
        tp = _lib.TestPanel(_ptr(tb), tb.size, ind.size, _ptr(ind), _ptr(sp), _ptr(lp))
        self.ctx.check(self.ctx.lib.dbslmm_plan_variance(self.h, C.byref(tp), _ptr(out), _ptr(nt)),
                       "plan_variance")
        return out.reshape(self.prob.num_block, n_test).T

    def close(self):
        if self.h:
            self.ctx.lib.dbslmm_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DBSLMMFIT:
    """Mirror of the reference's DBSLMMFIT::est (scr/dbslmmfit.hpp:35-66) on one GPU, or on
    several (device = a list of ordinals: the LD blocks sharded over them)."""

    def __init__(self, device=0):
        self.ctx = Context(device)

    def est(self, prob: BlockProblem):
        """Return (beta_s, beta_l, block_status).  LMM-only when prob.l_ptr is None."""
        bs = np.zeros(prob.n_s)
        bl = np.zeros(prob.n_l)
        st = np.zeros(prob.num_block, dtype=np.int32)
        cs = prob.c_struct()
        self.ctx.check(self.ctx.lib.dbslmm_est(self.ctx.h, C.byref(cs), _ptr(bs), _ptr(bl), _ptr(st)),
                       "dbslmm_est")
        return bs, bl, st


def bed_maf(ctx: Context, bed: np.ndarray, n_ref: int, n_snp: int) -> np.ndarray:
    bed = np.ascontiguousarray(bed, dtype=np.uint8)
    maf = np.zeros(n_snp)
    ctx.check(ctx.lib.dbslmm_bed_maf(ctx.h, _ptr(bed), bed.size, n_ref, n_snp, _ptr(maf)), "bed_maf")
    return maf


def read_snp_std(ctx: Context, bed: np.ndarray, n_ref: int, rows) -> tuple[np.ndarray, np.ndarray]:
    """Standardised genotype columns (n_ref x len(rows), Fortran order) and MAFs."""
    bed = np.ascontiguousarray(bed, dtype=np.uint8)
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    out = np.zeros(n_ref * len(rows))
    maf = np.zeros(len(rows))
    ctx.check(ctx.lib.dbslmm_read_snp_std(ctx.h, _ptr(bed), bed.size, n_ref, _ptr(rows), len(rows),
                                          _ptr(out), _ptr(maf)), "read_snp_std")
    return out.reshape(len(rows), n_ref).T, maf


def valid_blocks(ctx: Context, bed: np.ndarray, n_ref: int, ptr, pos, z1, z2):
    """External-validation terms of the `valid` tool (scr/validate.cpp:221-257) on the GPU:
    per block nume = z1.z2 and deno = z1^T (X^T X / n_ref) z1."""
    bed = np.ascontiguousarray(bed, dtype=np.uint8)
    ptr = np.ascontiguousarray(ptr, dtype=np.int64)
    pos = np.ascontiguousarray(pos, dtype=np.int32)
    z1 = np.ascontiguousarray(z1, dtype=np.float64)
    z2 = np.ascontiguousarray(z2, dtype=np.float64)
    nb = len(ptr) - 1
    nume = np.zeros(nb)
    deno = np.zeros(nb)
    ctx.check(ctx.lib.dbslmm_valid_blocks(ctx.h, _ptr(bed), bed.size, n_ref, nb, _ptr(ptr), _ptr(pos),
                                          _ptr(z1), _ptr(z2), _ptr(nume), _ptr(deno)), "valid_blocks")
    return nume, deno
