"""Oracle: batched fp64 restatement of OptiMOBO's acquisition functions.

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

Each function takes per-candidate posterior moments (μ_k, σ²_k; arrays of shape (N,))
instead of a model list, because the reference calls ``model.predict`` on one row and then
does pure arithmetic on the returned (μ, σ²).  The arithmetic below follows the reference
line by line, including its four quirks:
  1. ``change`` uses objective 0's variance for every objective (util_functions.py:233);
  2. ``EHVI`` passes the flattened sample covariance as "sigma" (σA = c00, σB = c01;
     util_functions.py:163-167, 114-115);
  3. ``EHVI_2D_aux`` omits the last stripe (``range(1, n+1)``, util_functions.py:120);
  4. ``EHVI_3D`` is the Monte-Carlo mean of max(0, Π(r − s) − HV(PF)) and pygmo raises when
     a sample leaves the reference box (util_functions.py:197-214).
The "textbook" EHVI-2D mode (per-objective σ and the last stripe) is the exact EHVI.
"""
import numpy as np
from scipy import special

from . import scalarisations as scal_mod

INV_SQRT_2PI = 1.0 / np.sqrt(2.0 * np.pi)


def norm_cdf(t):
    """scipy.stats.norm.cdf(t) == scipy.special.ndtr(t)."""
    return special.ndtr(t)


def norm_pdf(t):
    """scipy.stats.norm.pdf(t) == exp(-t²/2) / sqrt(2π)."""
    return np.exp(-np.square(t) / 2.0) * INV_SQRT_2PI


def psi_cal(a, b, m, s):
    """util_functions.py:130-133: ψ(a,b,m,s) = s·φ((b−m)/s) + (a−m)·Φ((b−m)/s)."""
    t = (b - m) / s
    return s * norm_pdf(t) + (a - m) * norm_cdf(t)


def cache_stats(cache):
    """Per-solve constants of np.cov(cache[:,0], cache[:,1]) (ddof=1): (s00, s01).

    Inside ``EHVI`` (util_functions.py:163) the covariance of the translated samples is
    σ²₀·Cov(cache) because ``change`` scales every column by sqrt(σ²₀).
    """
    c = np.cov(cache[:, 0], cache[:, 1])
    return float(c[0, 0]), float(c[0, 1])


def change(mu, var0, cache):
    """util_functions.py:217-237 batched: S[n, j, i] = cache[j, i]·sqrt(σ²₀[n]) + μ_i[n].

    mu: (k, N); var0: (N,) — objective 0's variance, used for every objective (quirk 1).
    Returns (N, M, k).
    """
    mu = np.asarray(mu, np.float64)
    sd = np.sqrt(np.asarray(var0, np.float64))
    return cache[None, :, :] * sd[:, None, None] + mu.T[:, None, :]


def sample_cov2(S):
    """np.cov(S[:,0], S[:,1]) per candidate (util_functions.py:163): (c00, c01)."""
    M = S.shape[1]
    X = S - S.mean(axis=1, keepdims=True)
    c00 = np.einsum("nj,nj->n", X[:, :, 0], X[:, :, 0]) / (M - 1)
    c01 = np.einsum("nj,nj->n", X[:, :, 0], X[:, :, 1]) / (M - 1)
    return c00, c01


def stripes_2d(pf, r):
    """util_functions.py:93-112: S = [(r0,−∞), PF sorted by f2 ascending, (−∞, r1)]."""
    pf = np.asarray(pf, np.float64).reshape(-1, 2)
    idx = np.argsort(pf[:, 1])
    S = np.concatenate(([[r[0], -np.inf]], pf[idx, :], [[-np.inf, r[1]]]), axis=0)
    return S[:, 0].copy(), S[:, 1].copy()


def ehvi2d_aux(pf, r, mu0, mu1, sA, sB, last_stripe=False):
    """util_functions.py:81-128 (EHVI_2D_aux), vectorised over candidates.

    mu0, mu1, sA, sB: (N,).  ``last_stripe`` adds the i = P+1 term the reference omits
    (quirk 3): ψ(y1[P], y1[P], μ0, σA)·ψ(r1, r1, μ1, σB).
    """
    y1, y2 = stripes_2d(pf, r)
    n = len(y1) - 2
    sum1 = np.zeros_like(np.asarray(mu0, np.float64))
    sum2 = np.zeros_like(sum1)
    for i in range(1, n + 1):
        t = (y1[i] - mu0) / sA
        p2 = psi_cal(y2[i], y2[i], mu1, sB)
        sum1 = sum1 + (y1[i - 1] - y1[i]) * norm_cdf(t) * p2
        sum2 = sum2 + (psi_cal(y1[i - 1], y1[i - 1], mu0, sA) - psi_cal(y1[i - 1], y1[i], mu0, sA)) * p2
    out = sum1 + sum2
    if last_stripe:
        out = out + psi_cal(y1[n], y1[n], mu0, sA) * psi_cal(r[1], r[1], mu1, sB)
    return out


def ehvi2d(mu, var, pf, r, cache, mode="reference"):
    """util_functions.py:136-167 (EHVI) batched over candidates.

    mu, var: (2, N).  mode "reference": samples via ``change`` → np.cov → σA=c00, σB=c01,
    last stripe omitted.  mode "textbook": σA = sqrt(σ²₀), σB = sqrt(σ²₁), all stripes.
    """
    mu = np.asarray(mu, np.float64)
    var = np.asarray(var, np.float64)
    if mode == "reference":
        S = change(mu, var[0], cache)
        c00, c01 = sample_cov2(S)
        return ehvi2d_aux(pf, r, mu[0], mu[1], c00, c01, last_stripe=False)
    if mode == "textbook":
        return ehvi2d_aux(pf, r, mu[0], mu[1], np.sqrt(var[0]), np.sqrt(var[1]), last_stripe=True)
    raise ValueError(mode)


def ehvi3d_reference(mu, var, hv_pf, r, cache):
    """util_functions.py:170-214 (EHVI_3D) batched.

    hv_pf = HV(PF, r) (``Sminus``, recomputed per call by the reference, constant per solve).
    Returns (value (N,), raises (N,) bool): pygmo's hypervolume raises ValueError when a
    sample is not inside the reference box (any s_j > r_j, or s == r).
    """
    mu = np.asarray(mu, np.float64)
    var = np.asarray(var, np.float64)
    S = change(mu, var[0], cache)                       # (N, M, k)
    r = np.asarray(r, np.float64)
    vol = np.prod(r[None, None, :] - S, axis=2)         # Π_j (r_j − s_j)
    h = vol - hv_pf
    value = np.where(h > 0, h, 0.0).sum(axis=1) / S.shape[1]
    outside = np.any(S > r[None, None, :], axis=2) | np.all(S == r[None, None, :], axis=2)
    raises = np.any(outside, axis=1) | np.any(np.isnan(S), axis=(1, 2))
    return value, raises


def hvpoi(mu, var, cells):
    """emo.py:192-228 (EMO.hypervolume_based_PoI) with emo.py:176-189 (vol5), batched.

    cells: (C, 2, k) with cells[c][0] = upper, cells[c][1] = lower.
    """
    mu = np.asarray(mu, np.float64)        # (k, N)
    var = np.asarray(var, np.float64)
    std = np.sqrt(var + 1e-5)
    cells = np.asarray(cells, np.float64)
    up = cells[:, 0, :].T[:, :, None]      # (k, C, 1)
    lo = cells[:, 1, :].T[:, :, None]
    m = mu[:, None, :]
    s = std[:, None, :]
    ppp = norm_cdf((up - m) / s) - norm_cdf((lo - m) / s)   # (k, C, N)
    poi = np.prod(ppp, axis=0).sum(axis=0)
    valid = np.all(up > m, axis=0)                          # (C, N)
    vol = np.prod(up - np.maximum(lo, m), axis=0)
    improvement = np.where(valid, vol, 0.0).sum(axis=0)
    return poi * improvement


def expected_decomposition(mu, var, cache, scalarisation, weights, agg_min):
    """util_functions.py:285-327 batched.

    S = change(...) (N, M, k); g = scal(S, w) (N, M); value = mean_j max(0, min − g_j)
    (the (M, M) broadcast at :324 has constant columns, so its mean equals this).
    ``scalarisation`` is an oracle.scalarisations object (same names/params as the reference).
    """
    mu = np.asarray(mu, np.float64)
    var = np.asarray(var, np.float64)
    S = change(mu, var[0], cache)
    g = scalarisation.batched(S, np.asarray(weights, np.float64))
    return np.mean(np.maximum(0.0, agg_min - g), axis=1)


def ei(mu, var, best, var_eps=0.0):
    """Expected improvement.

    var_eps = 0    : MonoSurrogateOptimiser._expected_improvement (optimisers.py:325-344)
    var_eps = 1e-6 : ParEGO / KEEP _expected_improvement (parego.py:126-145, keep.py:118-137)
    γ = (best − μ)/(σ + 1e-10); EI = σ(γΦ(γ) + φ(γ)).
    """
    mu = np.asarray(mu, np.float64).reshape(-1)
    sigma = np.sqrt(np.asarray(var, np.float64).reshape(-1) + var_eps)
    gamma = (best - mu) / (sigma + 1e-10)
    return sigma * (gamma * norm_cdf(gamma) + norm_pdf(gamma))


def pareto_ei(mu, var, best, var_eps=1e-6):
    """KEEP.pareto_expected_improvement (keep.py:142-151) with its EI (keep.py:118-137), batched.

    mu, var: (2, N) — row 0 the scalarised model, row 1 the Pareto-membership model.
    value = μ1 · EI(μ0, σ = sqrt(σ²0 + 1e-6)).
    """
    mu = np.asarray(mu, np.float64)
    var = np.asarray(var, np.float64)
    return mu[1] * ei(mu[0], var[0], best, var_eps)


def constrained_ei(mu, var, best, var_eps=0.0, pof_eps=1e-5):
    """ParEGO_C2.consraint_ei (cparego.py:486-496), batched.

    mu, var: (1 + m, N) — row 0 the aggregate model (EI with σ = sqrt(σ²), cparego.py:450-469),
    rows 1..m the constraint models; PoF_c = Φ((0 − μc) / sqrt(σ²c + 1e-5)) (cparego.py:471-484).
    """
    mu = np.asarray(mu, np.float64)
    var = np.asarray(var, np.float64)
    pof = np.ones(mu.shape[1])
    for c in range(1, mu.shape[0]):
        pof = pof * norm_cdf((0 - mu[c]) / np.sqrt(var[c] + pof_eps))
    return ei(mu[0], var[0], best, var_eps) * pof


def argmax(values, offset=0):
    """Arg-max with the build's rule: lowest index among maxima; NaN and −inf never win.

    Returns (best_value, best_index + offset) or (-inf, -1) when nothing qualifies.
    Replaces scipy ``differential_evolution(lambda x: −acq(x))`` (optimisers.py:87,118).
    """
    v = np.asarray(values, np.float64)
    ok = ~np.isnan(v) & (v > -np.inf)
    if not ok.any():
        return -np.inf, -1
    w = np.where(ok, v, -np.inf)
    i = int(np.argmax(w))
    return float(w[i]), i + offset


__all__ = ["norm_cdf", "norm_pdf", "psi_cal", "cache_stats", "change", "sample_cov2", "stripes_2d",
           "ehvi2d_aux", "ehvi2d", "ehvi3d_reference", "hvpoi", "expected_decomposition", "ei", "pareto_ei",
           "constrained_ei", "argmax", "scal_mod"]


def ehvi_exact_boxes(mu, var, lo, hi):
    """Exact EHVI for independent Gaussian objectives over a disjoint box decomposition of the
    non-dominated region (oracle.pareto.nondominated_boxes): Σ_b Π_j G(lo_bj, hi_bj; μ_j, σ_j),
    G(l, u) = E[(u − max(Y, l))⁺] = (u − l)Φ(α) + (u − μ)(Φ(β) − Φ(α)) + σ(φ(β) − φ(α)),
    α = (l − μ)/σ, β = (u − μ)/σ (l = −∞ → Φ(α) = φ(α) = 0).  "textbook" EHVI-3D mode.
    """
    mu = np.asarray(mu, np.float64)          # (k, N)
    sd = np.sqrt(np.asarray(var, np.float64))
    total = np.zeros(mu.shape[1])
    for b in range(len(lo)):
        prod = np.ones(mu.shape[1])
        for j in range(mu.shape[0]):
            l, u = lo[b, j], hi[b, j]
            be = (u - mu[j]) / sd[j]
            if np.isfinite(l):
                al = (l - mu[j]) / sd[j]
                Pa, pa = norm_cdf(al), norm_pdf(al)
                first = (u - l) * Pa
            else:
                Pa = pa = 0.0
                first = 0.0
            prod = prod * (first + (u - mu[j]) * (norm_cdf(be) - Pa) + sd[j] * (norm_pdf(be) - pa))
        total += prod
    return total
