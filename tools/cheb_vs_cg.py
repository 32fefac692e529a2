"""h2f tuning: iterations to cheb_tol for the plan's Chebyshev iteration vs a base-factor
preconditioned CG, per block, on blocks shaped like config 4's (numpy, CPU).

The h2f copies of a block solve M_c x = z with M_c = M_b + delta_c P_s (P_s: the small SNPs'
coordinates), M_b the base copy's matrix, factored once (plan.hip cheb_plan / trsv.hip).  Both
iterations start from the base solution x_b and apply M_b^{-1} once per iteration (one forward and
one backward substitution on the base factor); neither needs a product with M_b (the Chebyshev
recurrence carries s = M_b d, CG carries M_b p the same way).  CG needs two dot products per
iteration and block; the Chebyshev coefficients are a priori (interval [1, 1 + delta / (d_b + 1 -
tau)], plan.hip:1555-1592).  Also reported: the spectrum of M_b^{-1} M_c (its extreme
eigenvalues) and the Chebyshev count on that measured interval.

    python tools/cheb_vs_cg.py [m ...]        (default 9667 2579 544; n_ref 10000)
Block model: dbslmm_amd/synth.py (AR(1) rho 0.9 haplotypes, af ~ U(0.05, 0.5)); Sigma_ss of
estBlock (ref_numpy.block_sigmas_tau); sigma_s = h2 / M with M = 1e6, n_obs = 1e5, h2f 0.8 / 1 / 1.2;
optional one large SNP (bordered block, 'l' suffix: 9667l)."""
import math
import sys
import time

import numpy as np
import scipy.linalg as sl
from scipy.signal import lfilter
from scipy.special import ndtri

TAU, NOBS, M_TOTAL, H2, NREF, TOL = 0.8, 100_000, 1_000_000, 0.5, 10_000, 1e-9
H2F = (0.8, 1.0, 1.2)


def block_matrix(m, n, seed, rho=0.9):
    rng = np.random.default_rng(seed)
    thr = ndtri(rng.uniform(0.05, 0.5, size=m)).astype(np.float32)
    e = rng.standard_normal((m, 2 * n), dtype=np.float32)
    a = np.float32(math.sqrt(1 - rho * rho))
    u = np.empty_like(e)
    u[0] = e[0]
    u[1:] = lfilter([a], [1.0, -rho], e[1:], axis=0, zi=(rho * e[0])[None, :])[0]
    del e
    hap = u < thr[:, None]
    del u
    x = (hap[:, :n].astype(np.float64) + hap[:, n:].astype(np.float64)).T     # n x m
    del hap
    x -= x.mean(0)
    sd = x.std(0, ddof=1)
    sd[sd == 0] = 1.0
    x /= sd
    S = x.T @ x
    S *= TAU / n
    S[np.diag_indices(m)] += 1 - TAU
    return S


def cheb_coefs(lo, hi, K):
    th, de = 0.5 * (hi + lo), 0.5 * (hi - lo)
    sg, out = th / de, []
    for k in range(K):
        if k == 0:
            rho, al, be = 1 / sg, 0.0, 1 / th
        else:
            rn = 1 / (2 * sg - rho)
            al, be, rho = rn * rho, 2 * rn / de, rn
        out.append((al, be))
    return out


def cheb_k(lo, hi, e0):
    kap = hi / lo
    q = (math.sqrt(kap) - 1) / (math.sqrt(kap) + 1)
    return max(1, math.ceil(math.log(TOL / e0) / math.log(q)))


def run(spec):
    bordered = spec.endswith("l")
    m = int(spec.rstrip("l"))
    t0 = time.time()
    S = block_matrix(m, NREF, seed=m)
    ms = m - 1 if bordered else m          # the last coordinate plays the large SNP
    ps = np.zeros(m)
    ps[:ms] = 1.0
    z = np.random.default_rng(m + 1).standard_normal(m)
    sig = H2 / M_TOTAL
    d = {h: 1 / (sig * h * NOBS) for h in H2F}
    db = d[1.0]
    Mb = S.copy()
    Mb[np.arange(ms), np.arange(ms)] += db
    cf = sl.cho_factor(Mb, lower=True)
    prec = lambda r: sl.cho_solve(cf, r)
    xb = prec(z)
    print(f"m = {m}{' (1 large SNP)' if bordered else ''}: built in {time.time() - t0:.0f} s")
    # spectrum of M_b^{-1} P_s (generalised: P_s v = mu M_b v) -> M_b^{-1} M_c = I + delta mu
    Li = sl.solve_triangular(cf[0], np.eye(m), lower=True)
    B = (Li * ps) @ Li.T
    mu = sl.eigvalsh(B)
    del Li, B
    floor_ = db + 1 - TAU
    for h in (0.8, 1.2):
        dl = d[h] - db
        Mc = Mb.copy()
        Mc[np.arange(ms), np.arange(ms)] += dl
        x = sl.cho_solve(sl.cho_factor(Mc, lower=True), z)
        nx = np.linalg.norm(x)
        err = lambda y: np.linalg.norm(y - x) / nx
        ext = dl / floor_
        lo, hi = min(1, 1 + ext) * (1 - 1e-6), max(1, 1 + ext) * (1 + 1e-6)
        K = cheb_k(lo, hi, abs(ext))
        ev = 1 + dl * mu
        lo_m, hi_m = ev.min(), ev.max()
        mu_pos = mu[mu > 1e-12]
        lo_p, hi_p = (1 + dl * mu_pos).min(), (1 + dl * mu_pos).max()
        # Chebyshev as trsv.hip (a priori interval)
        def cheb(lo, hi, K):
            xk, r, dd, s, errs = xb.copy(), -dl * ps * xb, np.zeros(m), np.zeros(m), []
            for al, be in cheb_coefs(lo, hi, K):
                zz = prec(r)
                dd = al * dd + be * zz
                s = al * s + be * r
                xk = xk + dd
                r = r - s - dl * ps * dd
                errs.append(err(xk))
            return errs
        ec = cheb(lo, hi, K)
        # PCG on M_c with preconditioner M_b, from x_b; q = M_c p = (M_b p) + dl P_s p
        xk, r = xb.copy(), -dl * ps * xb
        zz = prec(r)
        p, mp = zz.copy(), r.copy()         # M_b p = r (p = M_b^{-1} r)
        rz, eg, cr = r @ zz, [], []
        fl = (d[h] + 1 - TAU) if ms == m else 1 - TAU     # lambda_min(M_c) >= fl
        for k in range(12):
            q = mp + dl * ps * p
            al = rz / (p @ q)
            xk = xk + al * p
            r = r - al * q
            zz = prec(r)
            rz2 = r @ zz
            be = rz2 / rz
            p = zz + be * p
            mp = r + be * mp
            rz = rz2
            eg.append(err(xk))
            cr.append(np.linalg.norm(r) / (fl * np.linalg.norm(xk)))   # >= the relative error
        kcg = next((i + 1 for i, e in enumerate(eg) if e <= TOL), None)
        kc_meas = cheb_k(lo_p * (1 - 1e-6), hi_p * (1 + 1e-6), abs(ext)) if lo_p > 0 else None
        em = cheb(lo_p * (1 - 1e-6), hi_p * (1 + 1e-6), kc_meas)
        print(f"  h2f {h}: delta {dl:+.3f}, a priori interval [{lo:.4f}, {hi:.4f}] -> K = {K}; "
              f"spectrum [{lo_m:.4f}, {hi_m:.4f}] ({(mu <= 1e-12).sum()} at 1; others [{lo_p:.4f}, {hi_p:.4f}])")
        print("    Chebyshev (a priori) error per iteration: " + " ".join(f"{e:.1e}" for e in ec))
        print(f"    Chebyshev on the measured interval: K = {kc_meas}: " + " ".join(f"{e:.1e}" for e in em))
        print(f"    PCG (M_b-preconditioned) error per iteration: " + " ".join(f"{e:.1e}" for e in eg[:8])
              + f"  -> cheb_tol at {kcg}")
        kst = next((i + 1 for i, e in enumerate(cr) if e <= TOL), None)
        print(f"    stopping bound |r| / (lambda_min(M_c) |x|) per iteration: " + " ".join(f"{e:.1e}" for e in cr[:8])
              + f"  -> stops at {kst}")
    sys.stdout.flush()


if __name__ == "__main__":
    for spec in (sys.argv[1:] or ["544", "2579", "9667"]):
        run(spec)
