"""ctypes front-end of the C oracle (TEST INFRASTRUCTURE ONLY -- see dbslmm_oracle.c header).

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product.
"""
from __future__ import annotations

import ctypes as C
import glob
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build() -> None:
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def numpy_openblas_path() -> str | None:
    """The OpenBLAS shipped inside NumPy (ILP64, scipy_-prefixed symbols), if present."""
    import numpy
    d = os.path.join(os.path.dirname(os.path.dirname(numpy.__file__)), "numpy.libs")
    c = sorted(glob.glob(os.path.join(d, "libscipy_openblas64_*.so")))
    return c[0] if c else None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.oracle_use_blas.argtypes = [C.c_char_p]
        L.oracle_read_snp_im.argtypes = [P, C.c_int64, P, C.c_int64, P, C.c_int64, P]
        L.oracle_normalize.argtypes = [P, C.c_int64]
        L.oracle_bed_maf.argtypes = [P, C.c_int32, C.c_int64, P, C.c_int]
        L.oracle_blas_threads.argtypes = [C.c_int]
        L.oracle_read_block_std.argtypes = [P, C.c_int32, P, C.c_int64, P, C.c_int]
        L.oracle_est_block.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, P, C.c_int, P,
                                       C.c_int, P, P, P, P, C.c_int, P]
        L.oracle_est.argtypes = [P, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int, P, P, P,
                                 P, P, P, P, P, C.c_int, C.c_int, P]
        _lib = L
    return _lib


def use_blas(enable: bool = True) -> bool:
    """Route the oracle's Gram/gemv through NumPy's OpenBLAS (single-threaded)."""
    if not enable:
        return False
    p = numpy_openblas_path()
    return bool(p) and lib().oracle_use_blas(p.encode()) == 0


def blas_threads(n: int) -> bool:
    """Threads of the shared OpenBLAS (oracle and NumPy) for the calls that follow."""
    return lib().oracle_blas_threads(int(n)) == 0


def read_block_std(bed: np.ndarray, n_ref: int, rows, threads: int = 8) -> np.ndarray:
    """Standardised n_ref x m block matrix (calcBlock's readSNPIm + nomalizeVec loop)."""
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    out = np.zeros((n_ref, len(rows)), dtype=np.float64, order="F")
    lib().oracle_read_block_std(_p(np.ascontiguousarray(bed, dtype=np.uint8)), n_ref, _p(rows),
                                len(rows), _p(out), threads)
    return out


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def read_snp_im(bed: np.ndarray, pos: int, indicator: np.ndarray):
    ind = np.ascontiguousarray(indicator, dtype=np.int32)
    n_sel = int((ind != 0).sum())
    g = np.zeros(n_sel)
    maf = np.zeros(1)
    lib().oracle_read_snp_im(_p(bed), pos, _p(ind), len(ind), _p(g), n_sel, _p(maf))
    return g, float(maf[0])


def normalize(x: np.ndarray) -> np.ndarray:
    y = np.ascontiguousarray(x, dtype=np.float64).copy()
    lib().oracle_normalize(_p(y), y.size)
    return y


def bed_maf(bed: np.ndarray, n_ref: int, n_snp: int, threads: int = 1) -> np.ndarray:
    maf = np.zeros(n_snp)
    lib().oracle_bed_maf(_p(bed), n_ref, n_snp, _p(maf), threads)
    return maf


def est_block(n_ref, n_obs, sigma_s, Xs, z_s, Xl=None, z_l=None, tau=0.8, method="pcg"):
    Xs = np.asfortranarray(Xs, dtype=np.float64)
    ms = Xs.shape[1]
    ml = 0 if Xl is None else Xl.shape[1]
    Xl = np.asfortranarray(Xl if Xl is not None else np.zeros((n_ref, 0)), dtype=np.float64)
    z_s = np.ascontiguousarray(z_s, dtype=np.float64)
    z_l = np.ascontiguousarray(z_l if z_l is not None else np.zeros(0), dtype=np.float64)
    bs = np.zeros(ms)
    bl = np.zeros(ml)
    it = np.zeros(1, dtype=np.int32)
    rc = lib().oracle_est_block(n_ref, n_obs, sigma_s, tau, _p(Xs), ms, _p(Xl), ml, _p(z_s),
                                _p(z_l), _p(bs), _p(bl), 0 if method == "pcg" else 1, _p(it))
    if rc:
        raise RuntimeError(f"oracle_est_block failed rc={rc}")
    return bs, bl, int(it[0])


def est(bed, n_ref, n_obs, sigma_s, s_ptr, s_rows, z_s, l_ptr=None, l_rows=None, z_l=None,
        tau=0.8, method="pcg", threads=1):
    """Whole-problem est over CSR block arrays (see dbslmm_oracle.c:oracle_est)."""
    bed = np.ascontiguousarray(bed, dtype=np.uint8)
    s_ptr = np.ascontiguousarray(s_ptr, dtype=np.int64)
    s_rows = np.ascontiguousarray(s_rows, dtype=np.int32)
    z_s = np.ascontiguousarray(z_s, dtype=np.float64)
    nb = len(s_ptr) - 1
    bs = np.zeros(len(s_rows))
    if l_ptr is not None:
        l_ptr = np.ascontiguousarray(l_ptr, dtype=np.int64)
        l_rows = np.ascontiguousarray(l_rows, dtype=np.int32)
        z_l = np.ascontiguousarray(z_l, dtype=np.float64)
        bl = np.zeros(len(l_rows))
    else:
        bl = None
    status = np.zeros(nb, dtype=np.int32)
    rc = lib().oracle_est(_p(bed), n_ref, n_obs, sigma_s, tau, nb, _p(s_ptr), _p(s_rows), _p(z_s),
                          _p(l_ptr), _p(l_rows), _p(z_l), _p(bs), _p(bl), threads,
                          0 if method == "pcg" else 1, _p(status))
    return bs, (bl if bl is not None else np.zeros(0)), status, rc
