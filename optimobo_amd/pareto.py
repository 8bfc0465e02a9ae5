"""Per-iteration host geometry for the acquisition kernels (pymoo/pygmo-free).

These run once per BO iteration on at most a few thousand objective vectors (SURVEY.md §8f
row 3), so they are host numpy; the per-candidate work they feed runs on the GPU.

* ``calc_pf``   — first non-dominated front, as util_functions.py:64-77 gets it from
                  pygmo.fast_non_dominated_sorting (row order kept, duplicates kept).
* ``stripes_2d``— the PF sorted by f2 ascending, the order EHVI_2D_aux walks
                  (util_functions.py:98-101); this is what omb_ehvi2d takes.
* ``decompose_into_cells`` — emo.py:55-152's 2-D cell list in closed form, reference-exact
                  including the lower-bound quirk (lower f2 of cells j ≥ 1 = max(I0, I1)).
* ``hypervolume`` — exact dominated volume (pymoo HV at optimisers.py:216-220; pygmo at
                  util_functions.py:198-199): sweep in 2-D, z-slab sweep in 3-D, WFG beyond.
* ``cached_samples`` / ``cache_stats`` — optimisers.py:121-141 and the np.cov constants EHVI
                  needs (util_functions.py:163).
"""
import numpy as np
from scipy.stats import norm, qmc


def nondominated_mask(Y, block=2048):
    """mask[i] = no row of Y Pareto-dominates row i (minimisation)."""
    Y = np.asarray(Y, np.float64)
    n = len(Y)
    mask = np.ones(n, bool)
    for s in range(0, n, block):
        B = Y[s:s + block]                                         # candidates to test
        le = np.all(Y[:, None, :] <= B[None, :, :], axis=2)       # Y[a] <= B[b]
        lt = np.any(Y[:, None, :] < B[None, :, :], axis=2)
        mask[s:s + block] = ~np.any(le & lt, axis=0)
    return mask


def calc_pf(Y):
    Y = np.asarray(Y, np.float64)
    if len(Y) < 2:
        return Y
    return Y[nondominated_mask(Y)]


def stripes_2d(pf):
    pf = np.asarray(pf, np.float64).reshape(-1, 2)
    return np.ascontiguousarray(pf[np.argsort(pf[:, 1], kind="stable")])


def decompose_into_cells(pf, ideal_point, max_point):
    pf = np.asarray(pf, np.float64).reshape(-1, 2)
    ideal = np.asarray(ideal_point, np.float64)
    mx = np.asarray(max_point, np.float64)
    p = pf[np.argsort(pf[:, 0], kind="stable")]
    P = len(p)
    up = np.empty((P + 1, 2))
    lo = np.empty((P + 1, 2))
    up[0] = (p[0, 0], max(p[0, 1], mx[1]))
    lo[0] = ideal
    up[1:P, 0] = p[1:, 0]
    up[1:P, 1] = p[:-1, 1]
    up[P] = (max(p[-1, 0], mx[0]), p[-1, 1])
    lo[1:, 0] = np.maximum(p[:, 0], ideal[0])
    lo[1:, 1] = max(ideal[0], ideal[1])
    return np.ascontiguousarray(np.stack([up, lo], axis=1))


def hypervolume(points, ref):
    P = np.asarray(points, np.float64)
    r = np.asarray(ref, np.float64)
    if P.size == 0:
        return 0.0
    P = P[np.all(P < r, axis=1)]
    if len(P) == 0:
        return 0.0
    P = calc_pf(P)
    k = P.shape[1]
    if k == 1:
        return float(r[0] - P[:, 0].min())
    if k == 2:
        P = P[np.argsort(P[:, 0], kind="stable")]
        f2 = np.minimum.accumulate(P[:, 1])
        prev = np.concatenate(([r[1]], f2[:-1]))
        return float(np.sum((r[0] - P[:, 0]) * np.clip(prev - f2, 0.0, None)))
    # sweep the last objective: each slab between consecutive levels is a (k-1)-D volume
    order = np.argsort(P[:, -1], kind="stable")
    P = P[order]
    levels = np.append(P[:, -1], r[-1])
    total = 0.0
    for i in range(len(P)):
        h = levels[i + 1] - levels[i]
        if h > 0:
            total += hypervolume(P[: i + 1, :-1], r[:-1]) * h
    return float(total)


def box_decomposition(pf, ref):
    """Disjoint boxes covering the part of (−∞, ref] the front does not dominate (k = 2, 3).

    Input of omb_ehvi_boxes (the exact "textbook" EHVI): HVI(y) = Σ_b Π_j (hi_bj − max(y_j, lo_bj))⁺.
    Returns (coords (k, C) f64 — per objective the sorted grid [−∞, front values…, ref_j] padded
    with ref_j —, ncoord (k,) int32, boxes (B, 2k) uint16 = [lo_idx_0, hi_idx_0, lo_idx_1, …]).
    3-D: one slab per distinct f3 level; inside a slab the 2-D staircase of the points below it.
    """
    pf = np.asarray(pf, np.float64)
    ref = np.asarray(ref, np.float64)
    k = ref.size
    if k not in (2, 3):
        raise NotImplementedError("box_decomposition: 2 or 3 objectives")
    pts = pf[np.all(pf < ref, axis=1)] if pf.size else np.zeros((0, k))
    pts = calc_pf(pts) if len(pts) > 1 else pts
    grids = [np.concatenate(([-np.inf], np.unique(pts[:, j]), [ref[j]])) for j in range(k)]

    def staircase(P2):
        """(x_lo, x_hi, y_hi) of the 2-D non-dominated stripes below ref[:2]."""
        if len(P2) == 0:
            return [(-np.inf, ref[0], ref[1])]
        F = calc_pf(P2)
        F = F[np.argsort(F[:, 0], kind="stable")]
        xb = np.concatenate(([-np.inf], F[:, 0], [ref[0]]))
        yt = np.concatenate(([ref[1]], F[:, 1]))
        return [(xb[i], xb[i + 1], yt[i]) for i in range(len(F) + 1) if xb[i + 1] > xb[i]]

    rows = []
    if k == 2:
        for xl, xh, yh in staircase(pts):
            rows.append((xl, xh, -np.inf, yh))
    else:
        z_levels = grids[2]                      # −∞, distinct f3 values, ref_3
        for a in range(len(z_levels) - 1):
            below = pts[pts[:, 2] <= z_levels[a], :2]
            for xl, xh, yh in staircase(below):
                rows.append((xl, xh, -np.inf, yh, z_levels[a], z_levels[a + 1]))
    vals = np.asarray(rows, np.float64).reshape(-1, 2 * k)
    idx = np.empty(vals.shape, np.int64)
    for j in range(k):
        for s in (0, 1):
            idx[:, 2 * j + s] = np.searchsorted(grids[j], vals[:, 2 * j + s])
    C = max(len(g) for g in grids)
    coords = np.stack([np.concatenate((g, np.full(C - len(g), g[-1]))) for g in grids])
    if C > 65535:
        raise ValueError("box_decomposition: front too large for 16-bit grid indices")
    return (np.ascontiguousarray(coords), np.array([len(g) for g in grids], np.int32),
            np.ascontiguousarray(idx.astype(np.uint16)))


def cached_samples(k, sample_exponent, seed=None):
    s = qmc.Sobol(d=k, scramble=True, seed=seed).random_base2(m=sample_exponent)
    return np.ascontiguousarray(np.column_stack([norm.ppf(s[:, i]) for i in range(k)]))


def cache_stats(cache):
    c = np.cov(cache[:, 0], cache[:, 1])
    return float(c[0, 0]), float(c[0, 1])
