"""NumPy check of the PCG route's multi-shift recurrence (round 6): the h2f copies of a block
without large SNPs solve (Sigma + d_c I) x_c = z -- one matrix, scalar shifts -- so ONE Krylov
sequence serves every copy (Jegerlehner, hep-lat/9612014; residuals of the shifted systems stay
collinear with the seed's).  The seed is the smallest shift (the slowest copy), iterated in the
Chronopoulos-Gear form the GPU kernels use (one product w = A r and one reduction per iteration):
    gamma = r.r, delta = w.r, beta = gamma / gamma_prev, alpha = gamma / (delta - beta gamma / alpha_prev)
    p = r + beta p, s = w + beta s, x += alpha p, r -= alpha s
and each shift e = d_c - d_seed >= 0 follows from the seed's scalars (c = alpha_k beta_{k-1} / alpha_{k-1}):
    zeta_{k+1} = zeta_k zeta_{k-1} / ((1 + c + alpha_k e) zeta_{k-1} - c zeta_k)
    alpha^e_k = alpha_k zeta_{k+1} / zeta_k,   beta^e_{k-1} = (zeta_k / zeta_{k-1})^2 beta_{k-1}
    p^e = zeta_k r + beta^e_{k-1} p^e,   x^e += alpha^e_k p^e,   |r^e_k| = |zeta_k| |r_k|.
Stops copy c when |r^e| <= tol (d_c + 1 - tau) |x^e|.  Prints iterations and errors vs direct
solves.  Usage: python tools/multishift_check.py [m]"""
import math
import sys

import numpy as np

from cg_gate import block, sigma


def multishift(A, z, shifts, tol, lam):
    n = len(shifts)
    x = [np.zeros_like(z) for _ in range(n)]
    p = [np.zeros_like(z) for _ in range(n)]
    r = z.copy()
    s = np.zeros_like(z)
    zeta = [1.0] * n
    zeta_m = [1.0] * n
    conv = [0] * n
    gp = ap = None
    for k in range(1000):
        w = A @ r
        gam, dlt, rr = r @ r, w @ r, r @ r
        for c in range(n):
            if not conv[c] and math.sqrt(rr) * abs(zeta[c]) <= tol * lam[c] * np.linalg.norm(x[c]) or rr == 0:
                conv[c] = conv[c] or k
        if all(conv):
            return x, k
        if k == 0:
            be, al, cc = 0.0, gam / dlt, 0.0
        else:
            be = gam / gp
            al = gam / (dlt - be * gam / ap)
            cc = al * be / ap
        for c in range(n):
            if conv[c]:
                continue
            e = shifts[c]
            zn = zeta[c] * zeta_m[c] / ((1.0 + cc + al * e) * zeta_m[c] - cc * zeta[c])
            alc = al * zn / zeta[c]
            bec = (zeta[c] / zeta_m[c]) ** 2 * be
            p[c] = zeta[c] * r + bec * p[c]
            x[c] = x[c] + alc * p[c]
            zeta_m[c], zeta[c] = zeta[c], zn
        s = w + be * s
        r = r - al * s
        gp, ap = gam, al
    return x, 1000


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    S = sigma(block(m, 10000, seed=m))
    z = np.random.default_rng(1).standard_normal(m)
    for M, facs in ((1e6, (0.8, 1.0, 1.2)), (5e5, (0.8, 1.0, 1.2)), (5e4, (0.5, 1.0, 2.0))):
        d = [1.0 / (0.5 * f / M * 1e5) for f in facs]
        dseed = min(d)
        A = S + dseed * np.eye(m)
        x, k = multishift(A, z, [di - dseed for di in d], 1e-12, [di + 0.2 for di in d])
        errs = []
        for di, xi in zip(d, x):
            xd = np.linalg.solve(S + di * np.eye(m), z)
            errs.append(np.abs(xi - xd).max() / np.abs(xd).max())
        print(f"M={M:.0e} d={[round(v, 2) for v in d]} iterations {k} errors {['%.1e' % e for e in errs]}")


if __name__ == "__main__":
    main()
