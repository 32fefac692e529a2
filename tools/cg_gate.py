"""Gate for the CG route (round 6): iteration counts of plain CG on A = Sigma_ss + d I.

A synthetic LD block of m SNPs x n_ref individuals is drawn from the bench generator's model
(dbslmm_amd/synth.py: AR(1) latent haplotypes, rho 0.9, p ~ U(0.05, 0.5)); Sigma = tau/n_ref X^T X +
(1 - tau) I with N-1 standardised columns (scr/dbslmmfit.cpp:705-709), A = Sigma + d I (:712) with
d = 1/(sigma_s n) of each BASELINE config (sigma_s = h2 h2f / M, n = 100 000).  CG runs from x = 0
until |r| <= tol * lambda_min_bound * |x|, lambda_min_bound = d + 1 - tau -- a bound on the relative
2-norm error of x that holds for any data.  Prints iterations and the true relative error vs a
Cholesky solve.  CPU, NumPy only; usage: python tools/cg_gate.py [m ...]
"""
from __future__ import annotations

import math
import sys

import numpy as np
from scipy.signal import lfilter
from scipy.special import ndtri


def block(m, n_ref, seed=1, rho=0.9):
    rng = np.random.default_rng(seed)
    af = rng.uniform(0.05, 0.5, size=m)
    thr = ndtri(af)
    a = math.sqrt(1 - rho * rho)
    e = rng.standard_normal((m, 2 * n_ref))
    u = np.empty_like(e)
    u[0] = e[0]
    u[1:] = lfilter([a], [1.0, -rho], e[1:], axis=0, zi=(rho * e[0])[None, :])[0]
    hap = u < thr[:, None]
    g = (hap[:, :n_ref].astype(np.float64) + hap[:, n_ref:])      # m x n
    return g


def sigma(g, tau=0.8):
    m, n = g.shape
    x = g - g.mean(axis=1, keepdims=True)
    x /= x.std(axis=1, ddof=1, keepdims=True)
    return tau / n * (x @ x.T) + (1 - tau) * np.eye(m)


def cg(A, b, tol, lam_min, maxit=1000):
    x = np.zeros_like(b)
    r = b.copy()
    p = r.copy()
    g = r @ r
    for k in range(1, maxit + 1):
        q = A @ p
        al = g / (p @ q)
        x += al * p
        r -= al * q
        gn = r @ r
        if math.sqrt(gn) <= tol * lam_min * np.linalg.norm(x):
            return x, k
        p = r + (gn / g) * p
        g = gn
    return x, maxit


def main():
    sizes = [int(s) for s in sys.argv[1:]] or [600, 2000, 5000]
    n_ref = 10000
    tau = 0.8
    rng = np.random.default_rng(7)
    for m in sizes:
        S = sigma(block(m, n_ref, seed=m), tau)
        ev = np.linalg.eigvalsh(S) if m <= 5000 else None
        for name, M, h2 in (("c2 50k", 5e4, 0.5), ("c3 500k", 5e5, 0.5), ("c4 1M h2f0.8", 1e6, 0.4),
                            ("c4 1M h2f1.2", 1e6, 0.6)):
            d = 1.0 / (h2 / M * 1e5)
            A = S + d * np.eye(m)
            z = rng.standard_normal(m)
            xd = np.linalg.solve(A, z)
            for tol in (1e-10, 1e-12):
                x, k = cg(A, z, tol, d + 1 - tau)
                err = np.abs(x - xd).max() / np.abs(xd).max()
                kap = (ev[-1] + d) / (ev[0] + d) if ev is not None else float("nan")
                print(f"m={m:5d} {name:14s} d={d:7.3f} kappa={kap:7.2f} tol={tol:.0e} "
                      f"iters={k:4d} err_inf_rel={err:.2e}", flush=True)
        if ev is not None:
            print(f"m={m}: lambda(Sigma) in [{ev[0]:.3f}, {ev[-1]:.3f}]", flush=True)


if __name__ == "__main__":
    main()
