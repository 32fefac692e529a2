"""ctypes binding of libdbslmm_hip.so (the C-ABI declared in include/dbslmm_hip.h).

The product path has no CPU fallback: if the in-tree HIP library is missing or no GPU is
present, every compute call raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libdbslmm_hip.so")

# symbols include/dbslmm_hip.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "dbslmm_abi_version", "dbslmm_ctx_create", "dbslmm_ctx_destroy", "dbslmm_last_error",
    "dbslmm_est", "dbslmm_plan_create", "dbslmm_plan_run", "dbslmm_plan_sync",
    "dbslmm_plan_download", "dbslmm_plan_set_sigma", "dbslmm_plan_destroy", "dbslmm_plan_run_multi",
    "dbslmm_plan_enable_timing", "dbslmm_plan_kernel_ms", "dbslmm_plan_workload",
    "dbslmm_bed_maf", "dbslmm_read_snp_std", "dbslmm_valid_blocks", "dbslmm_plan_variance",
    "dbslmm_ctx_create_multi", "dbslmm_ctx_num_devices", "dbslmm_plan_shard_info",
    "dbslmm_ctx_cache_bed", "dbslmm_ctx_cache_bed_fd", "dbslmm_plan_block_matrix",
    "dbslmm_shard_plan", "dbslmm_plan_create_units", "dbslmm_shard_plan_problem",
    "dbslmm_plan_block_iters",
)

ABI_VERSION = 15
K_UNPACK, K_GRAM, K_CHOL_LARGE, K_CHOL_SMALL, K_CHOL_TILED, K_TRSV, K_PCG, K_PCG_BLOCK = 0, 1, 2, 3, 4, 5, 6, 7
KERNEL_NAMES = ("dbslmm_unpack_stats", "dbslmm_gram", "dbslmm_chol_large", "dbslmm_chol_small",
                "dbslmm_tchol", "dbslmm_trsv", "dbslmm_pcg", "dbslmm_pcg_block")
WORKLOAD_LEN = 22
BLOCK_OK, BLOCK_EMPTY, BLOCK_NOT_PD, BLOCK_MONOMORPHIC, BLOCK_NOT_CONVERGED = 0, 1, 2, 3, 4
SOLVER_AUTO, SOLVER_FACTOR, SOLVER_PCG = 0, 1, 2


class Options(C.Structure):
    """dbslmm_options: path-selection thresholds (0 = default)."""
    _fields_ = [
        ("tiled_min", C.c_int32), ("gram_big_min", C.c_int32), ("gram_huge_min", C.c_int32),
        ("h2f_mode", C.c_int32), ("cheb_tol", C.c_double), ("lead_min", C.c_int32),
        ("large_cheb", C.c_int32), ("cheb_fused", C.c_int32), ("debug_delay_us", C.c_int32),
        ("debug_stop", C.c_int32), ("sub_split", C.c_int32), ("sub_grid_lead", C.c_int32),
        ("sub_grid_rest", C.c_int32), ("shard_copies", C.c_int32), ("h2f_iter", C.c_int32),
        ("solver", C.c_int32), ("pcg_tol", C.c_double), ("pcg_maxit", C.c_int32),
        ("pcg_whole", C.c_int32),
    ]


class Problem(C.Structure):
    _fields_ = [
        ("bed", C.c_void_p), ("bed_len", C.c_int64), ("n_ref", C.c_int32), ("n_obs", C.c_int32),
        ("sigma_s", C.c_double), ("tau", C.c_double), ("num_block", C.c_int32),
        ("s_ptr", C.c_void_p), ("s_pos", C.c_void_p), ("z_s", C.c_void_p),
        ("l_ptr", C.c_void_p), ("l_pos", C.c_void_p), ("z_l", C.c_void_p),
        ("opts", C.POINTER(Options)),
    ]


class TestPanel(C.Structure):
    _fields_ = [
        ("bed", C.c_void_p), ("bed_len", C.c_int64), ("n_total", C.c_int32),
        ("indicator", C.c_void_p), ("s_pos", C.c_void_p), ("l_pos", C.c_void_p),
    ]


_lib = None


class DbslmmError(RuntimeError):
    pass


def load(path: str | None = None):
    """Load the in-tree HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("DBSLMM_LIB_PATH") or LIB_PATH
    if not os.path.exists(p):
        raise DbslmmError(f"{p} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (or `make -C dbslmm_amd/csrc`)")
    L = C.CDLL(p)
    V, P = C.c_void_p, C.POINTER
    L.dbslmm_abi_version.restype = C.c_int
    L.dbslmm_ctx_create.argtypes = [C.c_int, P(V)]
    L.dbslmm_ctx_create_multi.argtypes = [C.c_int32, V, P(V)]
    L.dbslmm_ctx_num_devices.argtypes = [V]
    L.dbslmm_plan_shard_info.argtypes = [V, V]
    L.dbslmm_ctx_destroy.argtypes = [V]
    L.dbslmm_ctx_destroy.restype = None
    L.dbslmm_last_error.argtypes = [V]
    L.dbslmm_last_error.restype = C.c_char_p
    L.dbslmm_est.argtypes = [V, P(Problem), V, V, V]
    L.dbslmm_plan_create.argtypes = [V, P(Problem), P(V)]
    L.dbslmm_plan_run.argtypes = [V]
    L.dbslmm_plan_sync.argtypes = [V]
    L.dbslmm_plan_download.argtypes = [V, V, V, V]
    L.dbslmm_plan_set_sigma.argtypes = [V, C.c_double]
    L.dbslmm_plan_run_multi.argtypes = [V, V, C.c_int32, V, V, V]
    L.dbslmm_plan_destroy.argtypes = [V]
    L.dbslmm_plan_destroy.restype = None
    L.dbslmm_plan_enable_timing.argtypes = [V, C.c_int]
    L.dbslmm_plan_kernel_ms.argtypes = [V, V, V]
    L.dbslmm_plan_workload.argtypes = [V, V]
    L.dbslmm_bed_maf.argtypes = [V, V, C.c_int64, C.c_int32, C.c_int64, V]
    L.dbslmm_read_snp_std.argtypes = [V, V, C.c_int64, C.c_int32, V, C.c_int32, V, V]
    L.dbslmm_valid_blocks.argtypes = [V, V, C.c_int64, C.c_int32, C.c_int32, V, V, V, V, V, V]
    L.dbslmm_plan_variance.argtypes = [V, P(TestPanel), V, V]
    L.dbslmm_ctx_cache_bed.argtypes = [V, V, C.c_int64]
    L.dbslmm_ctx_cache_bed_fd.argtypes = [V, C.c_int, C.c_int64, V]
    L.dbslmm_shard_plan.argtypes = [C.c_int32, V, C.c_int32, C.c_int32, C.c_int32, V, V]
    L.dbslmm_plan_create_units.argtypes = [V, P(Problem), C.c_int32, V, C.c_int32, P(V)]
    L.dbslmm_shard_plan_problem.argtypes = [P(Problem), V, C.c_int32, C.c_int32, V, V]
    L.dbslmm_plan_block_iters.argtypes = [V, V]
    if hasattr(L, "dbslmm_plan_block_matrix"):   # (tools/race_probe.py loads older builds for A/B)
        L.dbslmm_plan_block_matrix.argtypes = [V, C.c_int32, C.c_int32, V, V]
    if L.dbslmm_abi_version() != ABI_VERSION:
        raise DbslmmError("ABI version mismatch")
    _lib = L
    return L
