"""NumPy restatement of the DBSLMM per-block effect-size path (TEST INFRASTRUCTURE ONLY).

This module is part of the oracle: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it, and only as the checker.  The product path
(``dbslmm_amd``) never imports anything under ``oracle/``.

It restates, as plainly as possible, what the reference computes (all citations are paths in
fboehm/DBSLMM, ``scr/``):

* ``read_snp_im``    -- ``IO::readSNPIm``           dtpr.cpp:285-364
* ``normalize``      -- ``SNPPROC::nomalizeVec``    dtpr.cpp:375-380  (N-1 sd, Armadillo default)
* ``pcg_v``/``pcg_m``-- ``DBSLMMFIT::PCGv/PCGm``     dbslmmfit.cpp:629-678
* ``est_block_ls``   -- ``estBlock`` (large+small)  dbslmmfit.cpp:680-738
* ``est_block_s``    -- ``estBlock`` (small-only)   dbslmmfit.cpp:740-770
* ``read_summ`` / ``read_bim`` / ``read_block`` / ``match_ref`` / ``add_block``
                     -- dtpr.cpp:47-68, 83-123, 178-220, 383-408, 455-481
* ``est``            -- ``DBSLMMFIT::est`` x2       dbslmmfit.cpp:56-244, 247-363 (beta only)
* ``format_eff``     -- output writer               dbslmm.cpp:353-364, 391-395

Parity pinning: with tau=1.0 (the pre-fork code) this restatement reproduces the 20-row
example output printed in ``Rmd/Manual.Rmd:126-145`` exactly (see tests/test_oracle.py).
tau=0.8 (the current code, dbslmmfit.cpp:697,751) is pinned only by this restatement.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

# ----------------------------------------------------------------------------- genotype reader

def bytes_per_snp(n_total: int) -> int:
    """dtpr.cpp:295-300: n_bit = ceil(n/4)."""
    return n_total // 4 + (1 if n_total % 4 else 0)


def decode_codes(row: np.ndarray, n_total: int) -> np.ndarray:
    """Unpack one packed SNP-major row into 2-bit codes, low bit pair first (dtpr.cpp:329-350).

    code = b[2j] | b[2j+1] << 1 ;  0 -> 2.0, 2 -> 1.0, 3 -> 0.0, 1 -> missing.
    """
    r = np.asarray(row, dtype=np.uint8)
    codes = np.stack([(r >> (2 * j)) & 3 for j in range(4)], axis=1).reshape(-1)
    return codes[:n_total]


_CODE2DOSE = np.array([2.0, np.nan, 1.0, 0.0])


def read_snp_im(bed: bytes | np.ndarray, pos: int, indicator: np.ndarray):
    """IO::readSNPIm (dtpr.cpp:285-364).

    ``indicator`` has one 0/1 entry per individual in the .fam (ni_total = len(indicator)).
    Returns (geno[float64, n_selected], maf).  Missing calls are mean-imputed with the mean of
    the non-missing selected calls; maf = min(af, 1-af) with af = 0.5*sum(geno)/n.
    """
    buf = np.frombuffer(bed, dtype=np.uint8) if not isinstance(bed, np.ndarray) else bed
    n_total = len(indicator)
    nb = bytes_per_snp(n_total)
    start = 3 + pos * nb                      # dtpr.cpp:302  (magic not checked)
    codes = decode_codes(buf[start:start + nb], n_total)
    sel = np.asarray(indicator) != 0
    g = _CODE2DOSE[codes[sel]]
    miss = np.isnan(g)
    mean = g[~miss].sum() / float(g.size - miss.sum())   # dtpr.cpp:358 (NaN if all missing)
    g[miss] = mean
    af = 0.5 * _arma_accumulate(g) / g.size               # dtpr.cpp:361 (sum(geno): Armadillo order)
    return g, min(af, 1.0 - af)


def _arma_accumulate(x: np.ndarray) -> float:
    """Armadillo arrayops::accumulate: two sequential accumulators over even/odd elements.

    np.cumsum is a strictly sequential left-to-right sum, so this reproduces the reference's
    rounding (needed: the Manual KAT is only reproduced at 6 digits with this order).
    """
    if x.size == 0:
        return 0.0
    a1 = np.cumsum(x[0::2])[-1]
    a2 = np.cumsum(x[1::2])[-1] if x.size > 1 else 0.0
    return float(a1 + a2)


def arma_mean(x: np.ndarray) -> float:
    """op_mean::direct_mean."""
    return _arma_accumulate(x) / x.size


def arma_var(x: np.ndarray) -> float:
    """op_var::direct_var with norm_type 0 (N-1), pairwise accumulation order."""
    n = x.size
    m = arma_mean(x)
    t = m - x
    k = n // 2
    pair_sq = t[0:2 * k:2] * t[0:2 * k:2] + t[1:2 * k:2] * t[1:2 * k:2]
    pair_s = t[0:2 * k:2] + t[1:2 * k:2]
    acc2 = np.cumsum(pair_sq)[-1] if k else 0.0
    acc3 = np.cumsum(pair_s)[-1] if k else 0.0
    if n % 2:
        acc2 += t[-1] * t[-1]
        acc3 += t[-1]
    return float((acc2 - acc3 * acc3 / n) / (n - 1))


def normalize(x: np.ndarray) -> np.ndarray:
    """SNPPROC::nomalizeVec (dtpr.cpp:375-380): x -= mean(x); x /= stddev(x) with N-1."""
    x = x - arma_mean(x)
    with np.errstate(divide="ignore", invalid="ignore"):
        return x / np.sqrt(arma_var(x))


def read_block_matrix(bed, rows, n_ref: int) -> np.ndarray:
    """calcBlock's column loop (dbslmmfit.cpp:419-430): standardised n_ref x m matrix."""
    idv = np.ones(n_ref, dtype=np.int32)        # dbslmm.cpp:328-329 (all ones)
    X = np.zeros((n_ref, len(rows)))
    for c, p in enumerate(rows):
        g, _ = read_snp_im(bed, int(p), idv)
        X[:, c] = normalize(g)
    return X


# ----------------------------------------------------------------------------- solvers

def pcg_v(A: np.ndarray, b: np.ndarray, maxiter: int = 1000, tol: float = 1e-7):
    """DBSLMMFIT::PCGv (dbslmmfit.cpp:629-668): Jacobi PCG, stop on ABSOLUTE ||r||2 <= tol."""
    dA = np.diag(A).copy()
    dA[dA == 0] = 1e-4
    Minv = 1.0 / dA
    x = np.zeros_like(b)
    r = b.copy()
    z = Minv * r
    p = z.copy()
    it = 0
    sumr2 = np.linalg.norm(r)
    while sumr2 > tol and it < maxiter:
        it += 1
        Ap = A @ p
        a = np.dot(r, z) / np.dot(p, Ap)
        x = x + a * p
        r1 = r - a * Ap
        z1 = Minv * r1
        bet = np.dot(z1, r1) / np.dot(z, r)
        p = z1 + bet * p
        z = z1
        r = r1
        sumr2 = np.linalg.norm(r)
    return x, it


def pcg_m(A, B, maxiter=1000, tol=1e-7):
    """DBSLMMFIT::PCGm (dbslmmfit.cpp:670-678): PCGv per column."""
    X = np.zeros((A.shape[0], B.shape[1]))
    for i in range(B.shape[1]):
        X[:, i], _ = pcg_v(A, B[:, i], maxiter, tol)
    return X


def _solve(A, B, method):
    if method == "pcg":
        return pcg_m(A, B) if B.ndim == 2 else pcg_v(A, B)[0]
    if method == "chol":      # direct, SPD: one Cholesky (used by the full-size parity tests)
        from scipy.linalg import cho_factor, cho_solve
        return cho_solve(cho_factor(A, lower=True, check_finite=False), B, check_finite=False)
    return np.linalg.solve(A, B)


def _solver(A, method):
    """x = A^-1 B for repeated right-hand sides of one matrix (factor once when direct)."""
    if method == "chol":
        from scipy.linalg import cho_factor, cho_solve
        cf = cho_factor(A, lower=True, check_finite=False)
        return lambda B: cho_solve(cf, B, check_finite=False)
    return lambda B: _solve(A, B, method)


def block_sigmas_tau(Xs, Xl, n_ref, tau=0.8):
    """Sigma_ss, Sigma_ls, Sigma_ll of estBlock (dbslmmfit.cpp:697-709); Xl may be None."""
    Sss = (Xs.T @ Xs) * (tau / n_ref) + np.eye(Xs.shape[1]) * (1.0 - tau)   # :705-709
    if Xl is None:
        return Sss, None, None
    Sls = (Xl.T @ Xs) * (tau / n_ref)                                  # :698-699
    Sll = (Xl.T @ Xl) * (tau / n_ref) + np.eye(Xl.shape[1]) * (1.0 - tau)   # :700-704
    return Sss, Sls, Sll


def est_block_ls_sigma(Sss, Sls, Sll, n_obs, sigma_s, z_s, z_l, method="pcg"):
    """estBlock (large + small) from its Sigma blocks (dbslmmfit.cpp:711-729)."""
    d = 1.0 / (sigma_s * n_obs)
    A = Sss + np.eye(Sss.shape[0]) * d                                 # :712
    solve_a = _solver(A, method)
    P = solve_a(Sls.T)                                                 # :713
    S = Sll - Sls @ P                                                  # :714-715
    q = solve_a(z_s)                                                   # :716
    rhs = z_l - Sls @ q                                                # :717-718
    beta_l = _solve(S, rhs, method) / math.sqrt(n_obs)                 # :719-720
    # :723-729 verbatim order of operations
    qs = q * math.sqrt(n_obs)
    Pb = n_obs * (P @ beta_l)
    w = qs - Pb
    beta_s = math.sqrt(n_obs) * z_s - n_obs * (Sls.T @ beta_l) - Sss @ w
    beta_s = beta_s * sigma_s
    return beta_s, beta_l


def est_block_s_sigma(Sss, n_obs, sigma_s, z_s, method="pcg"):
    """estBlock (small only) from Sigma_ss (dbslmmfit.cpp:758-764)."""
    d = 1.0 / (sigma_s * n_obs)
    A = Sss + np.eye(Sss.shape[0]) * d                                 # :759
    q = _solve(A, z_s, method)                                         # :760
    return math.sqrt(n_obs) * sigma_s * (z_s - Sss @ q)                # :761-764


def est_block_ls(n_ref, n_obs, sigma_s, Xs, Xl, z_s, z_l, tau=0.8, method="pcg"):
    """estBlock, large + small (dbslmmfit.cpp:680-738). Returns (beta_s, beta_l, Sss, Ssl, Sll)."""
    Sss, Sls, Sll = block_sigmas_tau(Xs, Xl, n_ref, tau)
    beta_s, beta_l = est_block_ls_sigma(Sss, Sls, Sll, n_obs, sigma_s, z_s, z_l, method)
    return beta_s, beta_l, Sss, Sls.T, Sll


def est_block_s(n_ref, n_obs, sigma_s, Xs, z_s, tau=0.8, method="pcg"):
    """estBlock, small only (dbslmmfit.cpp:740-770). Returns (beta_s, Sss)."""
    Sss, _, _ = block_sigmas_tau(Xs, None, n_ref, tau)
    return est_block_s_sigma(Sss, n_obs, sigma_s, z_s, method), Sss


# ----------------------------------------------------------------------------- host parsing

def get_row(path: str) -> int:
    """IO::getRow (dtpr.cpp:71-80)."""
    with open(path, "rb") as f:
        return sum(1 for _ in f)


def read_block(path: str):
    """IO::readBlock (dtpr.cpp:47-68): list of (chr, start, end)."""
    out = []
    with open(path) as f:
        for line in f:
            t = line.rstrip("\n").split("\t")
            out.append((t[0], int(t[1]), int(t[2])))
    return out


def read_bim(ref: str, n_ref: int, constr: bool):
    """IO::readBim (dtpr.cpp:83-123): dict snp -> (pos, a1, a2, maf). MAF pass if constr."""
    n_snp = get_row(ref + ".bim")
    maf = np.zeros(n_snp)
    if constr:
        bed = open(ref + ".bed", "rb").read()
        idv = np.ones(n_ref, dtype=np.int32)
        for i in range(n_snp):
            _, maf[i] = read_snp_im(bed, i, idv)
    bim = {}
    with open(ref + ".bim") as f:
        for count, line in enumerate(f):
            t = line.rstrip("\n").split("\t")
            if t[1] not in bim:          # std::map::insert keeps the first
                bim[t[1]] = (count, t[4], t[5], maf[count])
    return bim


@dataclass
class Summ:
    chr: int
    snp: str
    ps: int
    a1: str
    a2: str
    maf: float
    z: float


def _atof(s: str) -> float:
    """C atof prefix semantics (enough for GEMMA numeric fields)."""
    s = s.strip()
    try:
        return float(s)
    except ValueError:
        import re
        m = re.match(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", s)
        return float(m.group(0)) if m else 0.0


def read_summ(path: str):
    """IO::readSumm (dtpr.cpp:178-220): z = beta/se if se starts with a digit and > 1e-20."""
    out = []
    with open(path) as f:
        for line in f:
            t = line.rstrip("\n").split("\t")
            z = 0.0
            if t[9][:1].isdigit():
                se = _atof(t[9])
                if se - 0.0 > 1e-20:
                    z = _atof(t[8]) / se
            af = _atof(t[7])
            out.append(Summ(int(_atof(t[0])), t[1], int(_atof(t[2])), t[5], t[6],
                            min(af, 1.0 - af), z))
    return out


def match_ref(summ, bim, maf_max):
    """SNPPROC::matchRef (dtpr.cpp:383-408). Returns (inter list of dict, good flags)."""
    inter, good = [], []
    for s in summ:
        b = bim.get(s.snp)
        if b is None:
            # reference indexes bim[] (inserting an empty ALLELE) before the find(); an
            # absent SNP fails a1/a2 equality unless the summary alleles are empty strings.
            good.append(False)
            continue
        ok = b[1] == s.a1 and b[2] == s.a2 and abs(b[3] - s.maf) < maf_max
        good.append(ok)
        if ok:
            inter.append(dict(snp=s.snp, ps=s.ps, pos=b[0], a1=s.a1, maf=s.maf, z=s.z))
    return inter, good


def add_block(inter, blocks):
    """SNPPROC::addBlock (dtpr.cpp:455-481): [start, end) intervals, sequential scan.

    Returns the list of assigned SNPs (with 'block'); SNPs that the sequential scan never
    assigns are dropped ('documented divergences').
    """
    count = 0
    out = []
    for i, (_, start, end) in enumerate(blocks):
        for j in range(count, len(inter)):
            if start <= inter[j]["ps"] < end:
                e = dict(inter[j])
                e["block"] = i
                out.append(e)
                count += 1
            else:
                break
    return out


# ----------------------------------------------------------------------------- est

@dataclass
class EstResult:
    beta_s: np.ndarray
    beta_l: np.ndarray
    info_s: list = field(default_factory=list)
    info_l: list = field(default_factory=list)


def est(bed, n_ref, n_obs, sigma_s, num_block, info_s, info_l=None, tau=0.8, method="pcg"):
    """DBSLMMFIT::est (both overloads, beta part): per block, in block order."""
    info_l = info_l or []
    bs = np.zeros(len(info_s))
    bl = np.zeros(len(info_l))
    ps = 0
    pl = 0
    for b in range(num_block):
        s_idx = []
        while ps < len(info_s) and info_s[ps]["block"] == b:
            s_idx.append(ps)
            ps += 1
        l_idx = []
        while pl < len(info_l) and info_l[pl]["block"] == b:
            l_idx.append(pl)
            pl += 1
        if not s_idx and not l_idx:
            continue
        Xs = read_block_matrix(bed, [info_s[i]["pos"] for i in s_idx], n_ref)
        z_s = np.array([info_s[i]["z"] for i in s_idx])
        if l_idx:
            Xl = read_block_matrix(bed, [info_l[i]["pos"] for i in l_idx], n_ref)
            z_l = np.array([info_l[i]["z"] for i in l_idx])
            b_s, b_l, *_ = est_block_ls(n_ref, n_obs, sigma_s, Xs, Xl, z_s, z_l, tau, method)
            bl[l_idx] = b_l
        else:
            b_s, _ = est_block_s(n_ref, n_obs, sigma_s, Xs, z_s, tau, method)
        bs[s_idx] = b_s
    return EstResult(bs, bl, info_s, info_l)


def format_g(x: float) -> str:
    """C++ default ostream formatting of a double (precision 6, %g)."""
    return "%g" % x


def format_eff(res: EstResult) -> list[str]:
    """dbslmm.cpp:353-364: large rows then small rows, 'snp a1 beta beta_noscl flag'."""
    lines = []
    for info, beta, flag in ((res.info_l, res.beta_l, 1), (res.info_s, res.beta_s, 0)):
        for e, b in zip(info, beta):
            with np.errstate(divide="ignore", invalid="ignore"):
                noscl = b / math.sqrt(2 * e["maf"] * (1 - e["maf"])) if e["maf"] not in (0.0, 1.0) \
                    else (math.copysign(math.inf, b) if b != 0 else math.nan)
            if math.isinf(noscl):
                continue
            lines.append(f"{e['snp']} {e['a1']} {format_g(b)} {format_g(noscl)} {flag}")
    return lines


# ------------------------------------------------------------------------ `valid`
def read_bim_b(ref: str, n_ref: int, constr: bool):
    """IO::readBim, ALLELEB overload (dtpr.cpp:125-166): dict snp -> (pos, ps, a1, a2, maf);
    MAF pass over the .bed when constr; std::map::insert keeps the first of duplicate ids."""
    n_snp = get_row(ref + ".bim")
    maf = np.zeros(n_snp)
    if constr:
        bed = open(ref + ".bed", "rb").read()
        idv = np.ones(n_ref, dtype=np.int32)
        for i in range(n_snp):
            _, maf[i] = read_snp_im(bed, i, idv)
    bim = {}
    with open(ref + ".bim") as f:
        for count, line in enumerate(f):
            t = line.rstrip("\n").split("\t")
            if t[1] not in bim:
                bim[t[1]] = (count, int(_atof(t[3])), t[4], t[5], maf[count])
    return bim


def read_dbslmm(path: str):
    """IO::readDBSLMM (dtpr.cpp:223-245): space separated; (snp, a1, z = 3rd column = beta)."""
    out = []
    with open(path) as f:
        for line in f:
            t = line.rstrip("\n").split(" ")
            out.append((t[0], t[1], _atof(t[2])))
    return out


def read_ext(path: str):
    """IO::readExt (dtpr.cpp:248-268): space separated snp a1 maf z; map keyed by snp, first kept."""
    out = {}
    with open(path) as f:
        for line in f:
            t = line.rstrip("\n").split(" ")
            if t[0] not in out:
                out[t[0]] = (t[0], t[1], _atof(t[2]), _atof(t[3]))
    return out


def match_summ(dbslmm, ext):
    """SNPPROC::matchSumm (dtpr.cpp:411-433): DBSLMM rows in order that the external file has;
    z2 sign-flipped when the A1 alleles differ.  -> [(snp, a1, maf_ext, z1, z2)]"""
    out = []
    for snp, a1, z in dbslmm:
        if snp in ext:
            e = ext[snp]
            out.append((e[0], a1, e[2], z, e[3] if e[1] == a1 else -e[3]))
    return out


def match_all(summc, bim, maf_max):
    """SNPPROC::matchAll (dtpr.cpp:436-455): A1 equal to the bim A1 and |maf_ref - maf_ext| <
    mafMax; sorted by bp (std::sort).  -> [(snp, z1, z2, pos, ps)]"""
    out = []
    for snp, a1, maf, z1, z2 in summc:
        if snp in bim:
            pos, ps, ba1, _, bmaf = bim[snp]
            if ba1 == a1 and abs(bmaf - maf) < maf_max:
                out.append((snp, z1, z2, pos, ps))
    out.sort(key=lambda x: x[4])
    return out


def valid_blocks(bed, n_ref: int, summp, blocks):
    """VALID::BatchRun per-block loop (validate.cpp:221-257): sequential block scan (stalls like
    addBlock), standardised reference genotypes, SIGMA = X^T X / n_ref, nume = z1.z2,
    deno = z1^T SIGMA z1.  -> (nume[num_block], deno[num_block], per-block row lists)"""
    nb = len(blocks)
    nume, deno = np.zeros(nb), np.zeros(nb)
    rows = []
    count = 0
    for b, (_, start, end) in enumerate(blocks):
        idx = []
        for j in range(count, len(summp)):
            if start <= summp[j][4] < end:
                idx.append(j)
                count += 1
            else:
                break
        rows.append(idx)
        if not idx:
            continue
        z1 = np.array([summp[j][1] for j in idx])
        z2 = np.array([summp[j][2] for j in idx])
        X = read_block_matrix(bed, [summp[j][3] for j in idx], n_ref)
        sigma = X.T @ X / n_ref
        nume[b] = z1 @ z2
        deno[b] = z1 @ sigma @ z1
    return nume, deno, rows


def valid(d_path, s_path, ref, maf_max, block_path):
    """The `valid` tool end to end (validate.cpp:130-262) -> lines of <r2>.txt."""
    n_ref = get_row(ref + ".fam")
    summc = match_summ(read_dbslmm(d_path), read_ext(s_path))
    bim = read_bim_b(ref, n_ref, abs(maf_max - 1.0) >= 1e-10)
    summp = match_all(summc, bim, maf_max)
    blocks = read_block(block_path)
    bed = open(ref + ".bed", "rb").read()
    nume, deno, _ = valid_blocks(bed, n_ref, summp, blocks)
    return [f"{format_g(a)} {format_g(b)}" for a, b in zip(nume, deno)], nume, deno


# ------------------------------------------------------------ test-set variance
def read_test_bim(path: str):
    """readTestBim (calc_asymptotic_variance.cpp:143-153): the 4th tab field (bp) of each line."""
    with open(path) as f:
        return [line.rstrip("\n").split("\t")[3] for line in f]


def make_pos_for_test_bim(base_nums, inter):
    """makePosObjectForTestBim (calc_asymptotic_variance.cpp:160-180): each SNP's row in the test
    .bim = the FIRST line with the same bp (O(M^2) scan in the reference; same result)."""
    first = {}
    for i, s in enumerate(base_nums):
        first.setdefault(int(s), i)
    out = []
    for p in inter:
        if p["ps"] in first:
            e = dict(p)
            e["pos"] = first[p["ps"]]
            out.append(e)
    return out


def read_indicator(path: str) -> np.ndarray:
    """read_indices_file (subset_to_test_and_training.cpp:132-150): first space field per line."""
    with open(path) as f:
        return np.array([int(line.rstrip("\n").split(" ")[0]) for line in f], dtype=np.int32)


def read_test_block_matrix(bed, rows, indicator: np.ndarray) -> np.ndarray:
    """calcBlock's test columns (dbslmmfit.cpp:427-429): readSNPIm over the indicator-1
    individuals of the test panel, nomalizeVec -> n_test x m."""
    n_test = int(indicator.sum())
    X = np.zeros((n_test, len(rows)))
    for c, p in enumerate(rows):
        g, _ = read_snp_im(bed, int(p), indicator)
        X[:, c] = normalize(g)
    return X


def nt_diag_ls(sigma_ll, sigma_sl, sigma_ss, sigma2_s, n, Xl_test, Xs_test):
    """calc_nt_by_nt_matrix, large+small (calc_asymptotic_variance.cpp:22-43, with calc_A_inverse
    :66-74, calc_var_betal :86-96, calc_var_betas :109-123) -> diag of the n_test x n_test matrix."""
    ms = sigma_ss.shape[0]
    ainv = np.linalg.inv(np.eye(ms) / (n * sigma2_s) + sigma_ss)
    big = sigma_ll - sigma_sl.T @ ainv @ sigma_sl
    var_bl = np.linalg.inv(big) / n
    mat1 = sigma_ss - sigma_ss @ ainv @ sigma_ss
    mat2 = sigma_sl - sigma_ss @ ainv @ sigma_sl
    var_bs = n * sigma2_s * sigma2_s * (mat1 + mat2 * n @ var_bl @ mat2.T)
    res = Xl_test @ var_bl @ Xl_test.T + Xs_test @ var_bs @ Xs_test.T
    return np.diag(res).copy()


def nt_diag_s(sigma_ss, sigma2_s, n, Xs_test):
    """calc_nt_by_nt_matrix, small only (calc_asymptotic_variance.cpp:47-57, :127-137)."""
    ms = sigma_ss.shape[0]
    ainv = np.linalg.inv(np.eye(ms) / (n * sigma2_s) + sigma_ss)
    var_bs = n * sigma2_s * sigma2_s * (sigma_ss - sigma_ss @ ainv @ sigma_ss)
    return np.diag(Xs_test @ var_bs @ Xs_test.T).copy()


def block_sigmas(Xs, Xl, n_ref, tau=0.8):
    """Sigma_ss, Sigma_sl, Sigma_ll of estBlock (dbslmmfit.cpp:698-709), diagonal restored."""
    ss = tau * Xs.T @ Xs / n_ref + (1 - tau) * np.eye(Xs.shape[1])
    if Xl is None or Xl.shape[1] == 0:
        return ss, None, None
    sl = tau * Xs.T @ Xl / n_ref
    ll = tau * Xl.T @ Xl / n_ref + (1 - tau) * np.eye(Xl.shape[1])
    return ss, sl, ll


def variance_diags(bed, n_ref, n_obs, sigma_s, num_block, info_s, info_l, test_bed, indicator,
                   test_info_s, test_info_l, tau=0.8):
    """The diags matrix of DBSLMMFIT::est (dbslmmfit.cpp:116, 191-214, 242): n_test x num_block,
    column b = calcBlock's variance diag (zeros for a block without SNPs)."""
    n_test = int(indicator.sum())
    diags = np.zeros((n_test, num_block))
    for b in range(num_block):
        rs = [x["pos"] for x in info_s if x["block"] == b]
        rl = [x["pos"] for x in (info_l or []) if x["block"] == b]
        ts = [x["pos"] for x in test_info_s if x["block"] == b]
        tl = [x["pos"] for x in (test_info_l or []) if x["block"] == b]
        if not rs:
            continue
        Xs = read_block_matrix(bed, rs, n_ref)
        Xs_t = read_test_block_matrix(test_bed, ts[:len(rs)], indicator)
        if rl:
            Xl = read_block_matrix(bed, rl, n_ref)
            Xl_t = read_test_block_matrix(test_bed, tl[:len(rl)], indicator)
            ss, sl, ll = block_sigmas(Xs, Xl, n_ref, tau)
            diags[:, b] = nt_diag_ls(ll, sl, ss, sigma_s, n_obs, Xl_t, Xs_t)
        else:
            ss, _, _ = block_sigmas(Xs, None, n_ref, tau)
            diags[:, b] = nt_diag_s(ss, sigma_s, n_obs, Xs_t)
    return diags
