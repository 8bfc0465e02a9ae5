"""Oracle: Pareto filter, 2-D cell decomposition and exact hypervolume (fp64 numpy).

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

* ``calc_pf`` restates util_functions.py:64-77: the first front of
  ``pygmo.fast_non_dominated_sorting`` (pygmo>=2.0, absent here): the rows no other row
  Pareto-dominates, in ascending row order, duplicates kept; fewer than 2 rows → identity.
* ``decompose_into_cells`` restates the 2-D WFG-style decomposition of emo.py:55-152
  (≡ util_functions.py:414-517) in closed form; pinned against the
  reference implementation's own output (tests/golden/cells.npz).
* ``hypervolume`` is the exact dominated volume that ``pygmo.hypervolume(PF).compute(r)``
  (util_functions.py:198-206) and pymoo's ``HV`` (optimisers.py:216-220) return.  k = 2, 3: sweeps;
  k ≥ 4 (EHVI_3D runs for every n_obj != 2, optimisers.py:245-248): one point is the product
  Π_j (r_j − p_j) taken left to right (pagmo's single-point volume), a few points inclusion–exclusion
  over their subsets, more points slices along objective 0 — an algorithm independent of the build's
  last-objective sweep (optimobo_amd/pareto.py).
"""
import numpy as np


def dominates_matrix(Y):
    Y = np.asarray(Y, np.float64)
    le = np.all(Y[:, None, :] <= Y[None, :, :], axis=2)
    lt = np.any(Y[:, None, :] < Y[None, :, :], axis=2)
    return le & lt          # D[a, b]: a dominates b


def calc_pf(Y):
    Y = np.asarray(Y, np.float64)
    if len(Y) < 2:
        return Y
    D = dominates_matrix(Y)
    first = ~np.any(D, axis=0)
    return Y[first]


def decompose_into_cells(pf, ideal_point, max_point):
    """Closed form of emo.py:55-152 for 2 objectives → (P+1, 2, 2) [upper, lower].

    PF sorted by f1 ascending (emo.py:126; Python's stable ``sorted``), p_1..p_P:
      cell 0    : upper = (p1.f1, max(p1.f2, R1)),  lower = (I0, I1)            (emo.py:142-148)
      cell j    : upper = (p_{j+1}.f1, p_j.f2),      lower = (max(p_j.f1, I0), max(I0, I1))   (1 ≤ j < P)
      cell P    : upper = (max(pP.f1, R0), pP.f2),    lower = (max(pP.f1, I0), max(I0, I1))
    Quirk 5 (reference-exact): the lower bound of cells j ≥ 1 is
    ``np.maximum(np.rot90(incl)[-1], hv[-1])`` (emo.py:102) with incl = [p, ideal], so its
    f2 coordinate is max(I0, I1) — ideal's f1 leaks into f2; it equals I1 only when I0 ≤ I1.
    """
    pf = np.asarray(pf, np.float64).reshape(-1, 2)
    I = np.asarray(ideal_point, np.float64)
    R = np.asarray(max_point, np.float64)
    order = np.argsort(pf[:, 0], kind="stable")
    p = pf[order]
    P = len(p)
    cells = np.empty((P + 1, 2, 2))
    cells[0, 0] = (p[0, 0], max(p[0, 1], R[1]))
    cells[0, 1] = (I[0], I[1])
    lo2 = max(I[0], I[1])
    for j in range(1, P):
        cells[j, 0] = (p[j, 0], p[j - 1, 1])
        cells[j, 1] = (max(p[j - 1, 0], I[0]), lo2)
    cells[P, 0] = (max(p[P - 1, 0], R[0]), p[P - 1, 1])
    cells[P, 1] = (max(p[P - 1, 0], I[0]), lo2)
    return cells


def hypervolume(pts, r):
    """Exact hypervolume of the region dominated by ``pts`` and bounded by ``r`` (k = 2 or 3)."""
    pts = np.asarray(pts, np.float64)
    r = np.asarray(r, np.float64)
    if len(pts) == 0:
        return 0.0
    pts = pts[np.all(pts < r, axis=1)]
    if len(pts) == 0:
        return 0.0
    k = pts.shape[1]
    if k == 2:
        return _hv2d(pts, r)
    if k == 3:
        zs = np.unique(pts[:, 2])
        total = 0.0
        for i, z in enumerate(zs):
            z_next = zs[i + 1] if i + 1 < len(zs) else r[2]
            total += _hv2d(pts[pts[:, 2] <= z][:, :2], r[:2]) * (z_next - z)
        return total
    return _hv_kd(pts, r)


def _box(p, r):
    v = 1.0
    for j in range(len(r)):
        v *= r[j] - p[j]
    return v


def _hv_kd(pts, r):
    """Exact HV for k ≥ 4 of points strictly inside the box."""
    if len(pts) == 1:
        return _box(pts[0], r)
    if len(pts) <= 10:
        total = 0.0
        n = len(pts)
        for mask in range(1, 1 << n):
            idx = [i for i in range(n) if mask >> i & 1]
            corner = np.max(pts[idx], axis=0)            # the intersection of the boxes [p_i, r]
            total += (1.0 if len(idx) % 2 else -1.0) * _box(corner, r)
        return total
    # slice along objective 0: between consecutive levels, the (k-1)-D HV of the points at or below
    xs = np.unique(pts[:, 0])
    total = 0.0
    for i, x in enumerate(xs):
        x_next = xs[i + 1] if i + 1 < len(xs) else r[0]
        sub = pts[pts[:, 0] <= x][:, 1:]
        total += (x_next - x) * (hypervolume(sub, r[1:]) if sub.shape[1] >= 2 else r[1] - sub[:, 0].min())
    return total


def _hv2d(pts, r):
    p = pts[np.lexsort((pts[:, 1], pts[:, 0]))]
    total = 0.0
    best_f2 = r[1]
    for x, y in p:
        if y < best_f2:
            total += (r[0] - x) * (best_f2 - y)
            best_f2 = y
    return total


def nondominated_boxes(pf, r):
    """Disjoint boxes [lo, hi) covering the region below ``r`` that ``pf`` does NOT dominate
    (k = 2 or 3), so that HVI(y) = Σ_b Π_j (hi_j − max(y_j, lo_j))⁺ exactly.

    Not a reference function: it is the textbook decomposition behind the exact EHVI that
    "textbook" mode computes in place of the Monte-Carlo EHVI_3D (util_functions.py:170-214).
    2-D: the staircase stripes of EHVI_2D_aux (util_functions.py:93-125) as boxes.
    3-D: slabs between consecutive f3 levels, each the 2-D staircase of the points below it.
    Lower bounds may be −inf.  Returns (lo (B, k), hi (B, k)).
    """
    pf = np.asarray(pf, np.float64)
    r = np.asarray(r, np.float64)
    pf = calc_pf(pf[np.all(pf < r, axis=1)]) if len(pf) else pf.reshape(0, len(r))
    k = len(r)

    def stairs(P2, r2):
        # x-sorted 2-D front → boxes [lo, hi) in (x, y)
        out_lo, out_hi = [], []
        if len(P2) == 0:
            return [(-np.inf, -np.inf)], [(r2[0], r2[1])]
        Q = calc_pf(P2)
        Q = Q[np.lexsort((Q[:, 1], Q[:, 0]))]
        xs = [-np.inf] + list(Q[:, 0]) + [r2[0]]
        ys = [r2[1]] + list(Q[:, 1])
        for i in range(len(Q) + 1):
            if xs[i + 1] > xs[i]:
                out_lo.append((xs[i], -np.inf))
                out_hi.append((xs[i + 1], ys[i]))
        return out_lo, out_hi

    if k == 2:
        lo, hi = stairs(pf, r)
        return np.array(lo), np.array(hi)
    if k != 3:
        raise NotImplementedError("nondominated_boxes: k must be 2 or 3")
    levels = np.unique(pf[:, 2]) if len(pf) else np.array([])
    zs = np.concatenate(([-np.inf], levels, [r[2]]))
    LO, HI = [], []
    for a in range(len(zs) - 1):
        below = pf[pf[:, 2] <= zs[a]][:, :2] if a > 0 else np.zeros((0, 2))
        lo2, hi2 = stairs(below, r[:2])
        for (l0, l1), (h0, h1) in zip(lo2, hi2):
            LO.append((l0, l1, zs[a]))
            HI.append((h0, h1, zs[a + 1]))
    return np.array(LO), np.array(HI)
