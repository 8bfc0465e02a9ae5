"""Property-based checks (hypothesis) of the host-side geometry and the oracle's acquisitions
(layer 5: random Pareto fronts, EHVI against an independent exact form,
closed-form cells against the area identity, the arg-max rule).

These run on CPU.  Each property is an identity that holds for every input, so it pins the
product's host code (optimobo_amd.pareto) and the oracle against each other on inputs no
fixture covers: ties and duplicate front points, single-point fronts, points outside the
reference box.  Tolerances are written per assertion (fp64 sums of O(P) terms: 1e-12).
``derandomize=True`` keeps the draws reproducible; the example database is off so the tree
stays clean.
"""
import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from oracle import acquisition as oacq  # noqa: E402
from oracle import pareto as opar  # noqa: E402
from oracle import turbo as oturbo  # noqa: E402
from optimobo_amd import pareto as hpar  # noqa: E402

SETTINGS = dict(max_examples=80, deadline=None, derandomize=True, database=None)

# coordinates drawn from a coarse grid (forces ties / duplicates) or continuously
_coord = st.one_of(st.sampled_from([0.1, 0.25, 0.4, 0.5, 0.6, 0.75, 0.9]),
                   st.floats(0.01, 1.1, allow_nan=False, allow_infinity=False))


def _points(k, min_size=1, max_size=24):
    return st.lists(st.tuples(*([_coord] * k)), min_size=min_size, max_size=max_size).map(
        lambda v: np.array(v, np.float64).reshape(-1, k))


def _same_rows(a, b):
    a = a[np.lexsort(a.T[::-1])]
    b = b[np.lexsort(b.T[::-1])]
    return a.shape == b.shape and np.array_equal(a, b)


def _hvi_from_boxes(y, lo, hi):
    return float(np.prod(np.clip(hi - np.maximum(y[None, :], lo), 0.0, None), axis=1).sum())


# ----------------------------------------------------------------------------- Pareto front
@settings(**SETTINGS)
@given(st.integers(2, 3).flatmap(lambda k: _points(k, 1, 40)))
def test_calc_pf_is_the_nondominated_set(Y):
    pf = hpar.calc_pf(Y)
    assert _same_rows(pf, opar.calc_pf(Y))
    # mutually non-dominated ...
    for i in range(len(pf)):
        others = np.delete(pf, i, axis=0)
        assert not np.any(np.all(others <= pf[i], axis=1) & np.any(others < pf[i], axis=1))
    # ... and every input point is weakly dominated by a front point
    for y in Y:
        assert np.any(np.all(pf <= y, axis=1))


@settings(**SETTINGS)
@given(st.integers(2, 3).flatmap(lambda k: _points(k, 0, 30)))
def test_hypervolume_host_matches_oracle(Y):
    k = Y.shape[1]
    r = np.full(k, 1.0)
    assert abs(hpar.hypervolume(Y, r) - opar.hypervolume(Y, r)) <= 1e-12
    # monotone: adding a point never lowers the dominated volume
    if len(Y) > 1:
        assert opar.hypervolume(Y[:-1], r) <= opar.hypervolume(Y, r) + 1e-15


# ----------------------------------------------------------------------------- box decomposition
@settings(**SETTINGS)
@given(st.integers(2, 3).flatmap(lambda k: st.tuples(_points(k, 1, 16), _points(k, 1, 6))))
def test_box_decomposition_gives_exact_hvi(args):
    """Σ_b Π_j (hi − max(y, lo))⁺ over the non-dominated boxes == HV(PF ∪ {y}) − HV(PF), for the
    product's uint16-indexed decomposition and the oracle's float one alike."""
    Y, probes = args
    k = Y.shape[1]
    r = np.full(k, 1.0)
    pf = opar.calc_pf(Y)
    coords, ncoord, boxes = hpar.box_decomposition(pf, r)
    assert np.all(ncoord <= coords.shape[1])
    lo = np.stack([coords[j][boxes[:, 2 * j]] for j in range(k)], axis=1)
    hi = np.stack([coords[j][boxes[:, 2 * j + 1]] for j in range(k)], axis=1)
    olo, ohi = opar.nondominated_boxes(pf, r)
    hv = opar.hypervolume(pf, r)
    for y in probes:
        want = opar.hypervolume(np.vstack([pf, y]), r) - hv
        assert abs(_hvi_from_boxes(y, lo, hi) - want) <= 1e-12
        assert abs(_hvi_from_boxes(y, olo, ohi) - want) <= 1e-12


@settings(**SETTINGS)
@given(_points(2, 1, 20), st.floats(-0.3, 0.05), st.floats(1.0, 1.6))
def test_cells_closed_form(Y, ideal, top):
    """Host decompose_into_cells == oracle closed form; with I0 == I1 the cells and the
    dominated region tile [ideal, max]² (the identity emo.py's decomposition relies on) when the
    front lies inside that box, as it does in the reference (max = the front's nadir + margin)."""
    inside = Y[np.all((Y < top) & (Y > ideal), axis=1)]
    hyp.assume(len(inside) > 0)
    pf = opar.calc_pf(inside)
    I = np.array([ideal, ideal])
    R = np.array([top, top])
    cells = hpar.decompose_into_cells(pf, I, R)
    np.testing.assert_array_equal(cells, opar.decompose_into_cells(pf, I, R))
    area = np.prod(cells[:, 0, :] - cells[:, 1, :], axis=1).sum()
    assert abs(area + opar.hypervolume(pf, R) - (top - ideal) ** 2) <= 1e-12


# ----------------------------------------------------------------------------- acquisitions
_moments = st.tuples(st.floats(-0.2, 1.3), st.floats(-0.2, 1.3),
                     st.floats(-6, 0), st.floats(-6, 0))


@settings(**SETTINGS)
@given(_points(2, 1, 20), st.lists(_moments, min_size=1, max_size=8))
def test_ehvi2d_textbook_equals_box_form(Y, moments):
    """Two independent exact EHVI forms agree: the stripe sum of EHVI_2D_aux with every stripe
    (util_functions.py:93-125, "textbook") and the product of 1-D partial expectations over the
    non-dominated boxes.  The stripe form assumes the front lies below r, which the reference
    guarantees (r = nadir + margin, optimisers.py); the box form is ≥ 0."""
    r = np.array([1.0, 1.0])
    inside = Y[np.all(Y < r, axis=1)]
    hyp.assume(len(inside) > 0)
    pf = opar.calc_pf(inside)
    m = np.array(moments, np.float64)
    mu, var = m[:, :2].T.copy(), (10.0 ** m[:, 2:]).T.copy()
    a = oacq.ehvi2d(mu, var, pf, r, None, mode="textbook")
    lo, hi = opar.nondominated_boxes(pf, r)
    b = oacq.ehvi_exact_boxes(mu, var, lo, hi)
    np.testing.assert_allclose(a, b, rtol=1e-9, atol=1e-13)
    assert np.all(b >= -1e-15)


@settings(**SETTINGS)
@given(st.integers(2, 3).flatmap(lambda k: st.tuples(_points(k, 1, 12), _points(k, 1, 4))))
def test_exact_ehvi_tends_to_hvi_at_zero_variance(args):
    """σ → 0: EHVI(μ, σ²) → HVI(μ) (deterministic limit of the exact box form)."""
    Y, probes = args
    k = Y.shape[1]
    r = np.full(k, 1.0)
    pf = opar.calc_pf(Y)
    lo, hi = opar.nondominated_boxes(pf, r)
    mu = probes.T.copy()
    var = np.full_like(mu, 1e-24)
    got = oacq.ehvi_exact_boxes(mu, var, lo, hi)
    want = np.array([opar.hypervolume(np.vstack([pf, y]), r) for y in probes]) - opar.hypervolume(pf, r)
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-10)


# ----------------------------------------------------------------------------- selection rules
_val = st.one_of(st.sampled_from([np.nan, -np.inf, np.inf, 0.0, 1.0, 1.0, -2.5]),
                 st.floats(-10, 10, allow_nan=False))


@settings(**SETTINGS)
@given(st.lists(_val, min_size=0, max_size=40), st.integers(0, 1000))
def test_argmax_rule(vals, offset):
    """Lowest index among the maxima; NaN and −inf never win; (−inf, −1) when nothing does."""
    best, idx = None, -1
    for i, v in enumerate(vals):
        if np.isnan(v) or v == -np.inf:
            continue
        if best is None or v > best:
            best, idx = v, i
    got = oacq.argmax(np.array(vals, np.float64), offset=offset)
    if idx < 0:
        assert got == (-np.inf, -1)
    else:
        assert got == (best, idx + offset)


@settings(**SETTINGS)
@given(st.integers(1, 12), st.integers(1, 6), st.data())
def test_thompson_select_rule(N, B, data):
    """TuRBO's greedy selection (turbo.py:142-153): sample k's pick is the np.argmin (first NaN,
    else first minimum) over the column with earlier picks set to +inf.  Picks are distinct while
    B ≤ N and no value is +inf; a column that is all +inf re-picks index 0, as the reference."""
    vals = data.draw(st.lists(st.lists(_val, min_size=B, max_size=B), min_size=N, max_size=N))
    y = np.array(vals, np.float64)
    idx = oturbo.select(y)
    taken = []
    for k in range(B):
        col = y[:, k].copy()
        col[taken] = np.inf
        assert idx[k] == int(np.argmin(col))
        taken.append(int(idx[k]))
    if B <= N and not np.any(y == np.inf):
        assert len(set(idx.tolist())) == B
