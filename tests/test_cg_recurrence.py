"""The h2f CG recurrence of trsv.hip's dbslmm_cg_update, restated in NumPy (CPU): Chronopoulos-Gear
CG on M_c = M_b + delta P_s preconditioned by the base factor, both inner products from r and
z = M_b^{-1} r, q = M_c p carried without a product with M_b.  Checks, on LD-shaped blocks with and
without large SNPs: the iterate reaches the direct solve of M_c x = z; the kernel's stopping test
(|r| <= tol lambda_min(M_c) |x|, lambda_min >= d_c + 1 - tau, or 1 - tau with large SNPs) only
passes once the relative error is below tol; CG stops no later than the a priori Chebyshev count
(plan.hip cheb_plan) for h2f 0.8 / 1.2 around the base 1.0."""
import math

import numpy as np
import pytest
import scipy.linalg as sl

TAU, TOL = 0.8, 1e-9


def _sigma(m, n, rho, seed):
    rng = np.random.default_rng(seed)
    u = np.empty((m, n))
    u[0] = rng.standard_normal(n)
    for i in range(1, m):   # AR(1) latent along the SNPs, thresholded to dosages
        u[i] = rho * u[i - 1] + math.sqrt(1 - rho * rho) * rng.standard_normal(n)
    x = (u > 0.3).astype(float) + (rng.random((m, n)) < 0.2)
    x = (x - x.mean(1, keepdims=True)) / x.std(1, ddof=1, keepdims=True)
    return TAU * (x @ x.T) / n + (1 - TAU) * np.eye(m)


def _cheb_count(ext):
    lo, hi = min(1, 1 + ext) * (1 - 1e-6), max(1, 1 + ext) * (1 + 1e-6)
    q = (math.sqrt(hi / lo) - 1) / (math.sqrt(hi / lo) + 1)
    return max(1, math.ceil(math.log(TOL / abs(ext)) / math.log(q)))


def _cg(Mb_fac, ms, m, dl, xb, fl, K):
    """dbslmm_cg_update's arithmetic, one copy; returns (x, iterations, errors per iteration)."""
    ps = np.zeros(m)
    ps[:ms] = 1.0
    x, r = xb.copy(), -dl * ps * xb
    p, q = np.zeros(m), np.zeros(m)
    gp = ap = 0.0
    for k in range(K):
        z = sl.cho_solve(Mb_fac, r)                       # the forward + backward passes
        gam, zeta = r @ z, (ps * z) @ z
        eta = gam + dl * zeta
        if k == 0:
            be, den = 0.0, eta
        else:
            be = gam / gp if gp > 0 else 0.0
            den = eta - (be * gam / ap if ap != 0 else 0.0)
        al = gam / den if den > 0 and gam > 0 else 0.0
        gp, ap = gam, al
        p = z + be * p
        q = r + dl * ps * z + be * q
        x = x + al * p
        r = r - al * q
        if np.linalg.norm(r) <= TOL * fl * np.linalg.norm(x):
            return x, k + 1
    return x, K


@pytest.mark.parametrize("m,large", [(300, 0), (300, 1), (500, 2)])
def test_cg_recurrence_reaches_the_direct_solve(m, large):
    n, n_obs, sigma = 400, 100_000, 0.5 / 1_000_000
    S = _sigma(m, n, 0.9, seed=m + large)
    ms = m - large
    z = np.random.default_rng(7).standard_normal(m)
    d = {h: 1 / (sigma * h * n_obs) for h in (0.8, 1.0, 1.2)}
    db = d[1.0]
    Mb = S.copy()
    Mb[np.arange(ms), np.arange(ms)] += db
    fac = sl.cho_factor(Mb, lower=True)
    xb = sl.cho_solve(fac, z)
    for h in (0.8, 1.2):
        dl = d[h] - db
        Mc = S.copy()
        Mc[np.arange(ms), np.arange(ms)] += d[h]
        exact = np.linalg.solve(Mc, z)
        K = _cheb_count(dl / (db + 1 - TAU))
        fl = (d[h] + 1 - TAU) if large == 0 else 1 - TAU
        # lambda_min(M_c) is at least the bound the kernel stops on
        assert np.linalg.eigvalsh(Mc)[0] >= fl * (1 - 1e-12)
        x, its = _cg(fac, ms, m, dl, xb, fl, K)
        err = np.linalg.norm(x - exact) / np.linalg.norm(exact)
        assert err <= TOL, (h, its, err)
        assert its <= K
        if large == 0:
            assert its < K, (h, its, K)     # the adaptive stop beats the a priori count
