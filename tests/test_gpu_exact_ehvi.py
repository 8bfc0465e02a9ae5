"""GPU: exact (textbook) EHVI over the box decomposition vs the oracle (k = 2, 3)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import acquisition as oacq  # noqa: E402
from oracle import pareto as opar  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    from optimobo_amd.device import AcqContext
    c = AcqContext(0)
    yield c
    c.close()


def dev(x):
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device="cuda:0")


@pytest.mark.parametrize("k,P,N", [(2, 1, 7), (2, 30, 3000), (3, 1, 5), (3, 12, 2000), (3, 60, 700)])
def test_exact_ehvi_vs_oracle(ctx, k, P, N):
    from optimobo_amd import pareto
    rng = np.random.default_rng(10 * k + P)
    pts = rng.uniform(0.05, 1, (P * 10, k))
    pts /= np.linalg.norm(pts, axis=1, keepdims=True)
    pf = opar.calc_pf(pts)[:P]
    r = np.full(k, 1.2)
    mu = rng.uniform(0.0, 1.3, (k, N))
    var = 10 ** rng.uniform(-5, -0.5, (k, N))
    coords, _, boxes = pareto.box_decomposition(pf, r)
    out = ctx.ehvi_boxes(dev(mu), dev(var), coords, boxes).cpu().numpy()
    lo, hi = opar.nondominated_boxes(pf, r)
    ref = oacq.ehvi_exact_boxes(mu, var, lo, hi)
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-13)
    if k == 2:
        np.testing.assert_allclose(out, oacq.ehvi2d(mu, var, pf, r, None, mode="textbook"), rtol=1e-9, atol=1e-13)


def test_exact_ehvi_large_box_list_from_global(ctx):
    """Box lists too large for LDS are read from global memory."""
    from optimobo_amd import pareto
    rng = np.random.default_rng(5)
    pts = rng.uniform(0.05, 1, (3000, 3))
    pts /= np.linalg.norm(pts, axis=1, keepdims=True)
    pf = opar.calc_pf(pts)[:250]
    r = np.full(3, 1.2)
    coords, _, boxes = pareto.box_decomposition(pf, r)
    assert boxes.nbytes > 40000
    mu = rng.uniform(0.0, 1.3, (3, 300))
    var = 10 ** rng.uniform(-4, -1, (3, 300))
    out = ctx.ehvi_boxes(dev(mu), dev(var), coords, boxes).cpu().numpy()
    lo, hi = opar.nondominated_boxes(pf, r)
    np.testing.assert_allclose(out, oacq.ehvi_exact_boxes(mu, var, lo, hi), rtol=1e-9, atol=1e-13)
