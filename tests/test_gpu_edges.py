"""GPU edge cases through the C-ABI: error codes, empty/tiny batches, maximum geometry sizes,
NaN propagation, degenerate training sets."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import acquisition as oacq  # noqa: E402
from oracle import gp as ogp  # noqa: E402


@pytest.fixture()
def ctx():
    from optimobo_amd.device import AcqContext
    c = AcqContext(0)
    yield c
    c.close()


def dev(x):
    return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device="cuda:0")


def _gp(ctx, obj, X, y, ls, var=1.0):
    from optimobo_amd.gp import GPState
    ctx.set_gp_state(obj, GPState(X, y, ls, var))


def test_counter_ring_timeout_is_reported(ctx):
    """A posterior counter-ring wait that runs out marks the fault word and the next call returns
    OMB_EHIP (once).  omb_debug_set(SPIN_LIMIT, 0) lets every wait poll only once, which forces
    the path in practice (a wave reaching a counter before the other 7 waves signal it)."""
    from optimobo_amd import _lib
    rng = np.random.default_rng(8)
    n, d, N = 300, 4, 1 << 15          # 128 < n ≤ 1024: the counter-synchronised ring
    X = rng.uniform(0, 1, (n, d))
    Y = np.column_stack([np.sin(3 * X).sum(1), np.cos(2 * X).prod(1)])
    ls = np.array([0.4, 0.8, 1.1, 0.6])
    for o in range(2):
        _gp(ctx, o, X, Y[:, o], ls, float(np.var(Y[:, o])))
    Xc = dev(rng.uniform(0, 1, (N, d)))
    ctx.posterior(Xc, n_obj=2)
    ctx.synchronize()                                   # default bound: no fault
    ctx.debug_set("spin_limit", 0)
    with pytest.raises(_lib.OMBError) as e:
        for _ in range(3):
            ctx.posterior(Xc, n_obj=2)
            ctx.synchronize()
    assert e.value.code == _lib.OMB_EHIP and "counter-ring" in str(e.value)
    ctx.synchronize()                                   # reported once; the word is clear again
    ctx.debug_set("spin_limit", 1 << 22)
    mu, var = ctx.posterior(Xc[:500], n_obj=2)
    ctx.synchronize()
    for o in range(2):
        m, v = ogp.ExactGP(X, Y[:, o], ls, float(np.var(Y[:, o]))).predict(Xc[:500].cpu().numpy())
        np.testing.assert_allclose(mu[o].cpu().numpy(), m[:, 0], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(var[o].cpu().numpy(), v[:, 0], rtol=1e-6, atol=1e-9)
    with pytest.raises(_lib.OMBError) as e:
        ctx.debug_set("spin_limit", -1)
    assert e.value.code == _lib.OMB_EINVAL


def test_error_codes(ctx):
    from optimobo_amd import _lib
    with pytest.raises(_lib.OMBError) as e:
        ctx.posterior(dev(np.zeros((4, 2))), n_obj=1)
    assert e.value.code == _lib.OMB_ESTATE
    rng = np.random.default_rng(0)
    _gp(ctx, 0, rng.uniform(0, 1, (10, 2)), rng.uniform(0, 1, 10), [0.5, 0.5])
    _gp(ctx, 1, rng.uniform(0, 1, (10, 3)), rng.uniform(0, 1, 10), [0.5, 0.5, 0.5])
    with pytest.raises(_lib.OMBError) as e:
        ctx.posterior(dev(np.zeros((4, 2))), n_obj=2)
    assert e.value.code == _lib.OMB_EINVAL
    import ctypes
    rc = ctx.lib.omb_set_gp(ctx._h, 2, 0, _lib.MAX_TRAIN_DENSE + 1, 2, ctypes.c_void_p(8), _lib.darr([1, 1]), 1.0,
                            ctypes.c_void_p(8), ctypes.c_void_p(8))      # rejected before any access
    assert rc == _lib.OMB_EUNSUP
    with pytest.raises(_lib.OMBError) as e:
        ctx.set_gp(2, np.zeros((4, _lib.MAX_DIM + 1)), np.ones(_lib.MAX_DIM + 1), 1.0, np.zeros(4), np.eye(4))
    assert e.value.code == _lib.OMB_EUNSUP
    with pytest.raises(_lib.OMBError):
        ctx.set_gp(2, np.zeros((4, 2)), [1.0, -1.0], 1.0, np.zeros(4), np.eye(4))   # ℓ ≤ 0


def test_empty_and_single_candidate(ctx):
    rng = np.random.default_rng(1)
    X = rng.uniform(0, 1, (30, 3))
    y = X.sum(1)
    _gp(ctx, 0, X, y, [0.4, 0.6, 0.9], 2.0)
    mu, var = ctx.posterior(dev(np.zeros((0, 3))), n_obj=1)
    assert mu.shape == (1, 0)
    x1 = rng.uniform(0, 1, (1, 3))
    mu, var = ctx.posterior(dev(x1), n_obj=1)
    m, v = ogp.ExactGP(X, y, [0.4, 0.6, 0.9], 2.0).predict(x1)
    assert mu.item() == pytest.approx(m.item(), rel=1e-9, abs=1e-12)
    assert var.item() == pytest.approx(v.item(), rel=1e-7, abs=1e-12)
    assert ctx.argmax(dev(np.zeros(0))) == (-np.inf, -1)


def test_max_geometry_sizes(ctx):
    from optimobo_amd import _lib
    rng = np.random.default_rng(2)
    x = np.sort(rng.uniform(0, 1, 4095))
    pf = np.column_stack([x, 1 - np.sqrt(x)])
    pf_sorted = pf[np.argsort(pf[:, 1])]
    mu = rng.uniform(0, 1, (2, 64))
    var = 10 ** rng.uniform(-4, -1, (2, 64))
    r = np.array([1.1, 1.1])
    out = ctx.ehvi2d(dev(mu), dev(var), pf_sorted, r, 1.0, 0.1, mode="textbook").cpu().numpy()
    ref = oacq.ehvi2d(mu, var, pf, r, None, mode="textbook")
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-13)
    with pytest.raises(_lib.OMBError) as e:
        ctx.ehvi2d(dev(mu), dev(var), np.vstack([pf_sorted, [[2.0, 2.0]]]), r, 1.0, 0.1)
    assert e.value.code == _lib.OMB_EUNSUP
    cache = rng.standard_normal((4096, 2))
    out = ctx.expdec(dev(mu), dev(var), cache, 1, [], [0.5, 0.5], [0, 0], [1, 1], 0.3).cpu().numpy()
    from oracle import scalarisations as osc
    ref = oacq.expected_decomposition(mu, var, cache, osc.Tchebicheff([0, 0], [1, 1]), np.array([0.5, 0.5]), 0.3)
    np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-13)
    with pytest.raises(_lib.OMBError):
        ctx.expdec(dev(mu), dev(var), rng.standard_normal((4097, 2)), 1, [], [0.5, 0.5], [0, 0], [1, 1], 0.3)


def test_nan_moments_never_win(ctx):
    mu = np.array([[0.2, np.nan, 0.4], [0.3, 0.1, np.nan]])
    var = np.full((2, 3), 0.01)
    pf = np.array([[0.5, 0.5]])
    out = ctx.ehvi2d(dev(mu), dev(var), pf, [1.0, 1.0], 1.0, 0.1, mode="textbook").cpu().numpy()
    assert np.isfinite(out[0]) and np.isnan(out[1]) and np.isnan(out[2])
    assert ctx.argmax(dev(out)) == (out[0], 0)


def test_duplicate_training_points(ctx):
    """Repeated rows make K singular; GPy's 1e-8 jitter (and jitchol) keeps the fit finite."""
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 1, (40, 2))
    X[20:] = X[:20]
    y = np.sin(3 * X[:, 0]) + X[:, 1]
    _gp(ctx, 0, X, y, [0.3, 0.3], 1.0)
    Xc = rng.uniform(0, 1, (500, 2))
    mu, var = ctx.posterior(dev(Xc), n_obj=1)
    m, v = ogp.ExactGP(X, y, [0.3, 0.3], 1.0).predict(Xc)
    np.testing.assert_allclose(mu[0].cpu().numpy(), m[:, 0], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(var[0].cpu().numpy(), v[:, 0], rtol=1e-6, atol=1e-9)


# ----------------------------------------------------------------------------- n_train > 1024
@pytest.mark.parametrize("n,d,N", [(1025, 2, 700), (1500, 6, 3000), (2600, 30, 513)])
def test_dense_posterior_path_vs_oracle(ctx, n, d, N):
    """n_train above the fused kernel's 1024: K block → GEMM V = L⁻¹K* → column reduction."""
    from oracle import gp as ogp
    from optimobo_amd.gp import GPState
    rng = np.random.default_rng(n)
    X = rng.uniform(0, 1, (n, d))
    y = np.sin(3 * X).sum(1)
    ls = rng.uniform(0.5, 2.0, d)
    var = float(np.var(y))
    ctx.set_gp_state(0, GPState(X, y, ls, var))
    Xc = rng.uniform(0, 1, (N, d))
    Xc[:3] = X[:3]
    mu, v = ctx.posterior(dev(Xc), n_obj=1)
    mo, vo = ogp.ExactGP(X, y, ls, var).predict(Xc)
    np.testing.assert_allclose(mu[0].cpu().numpy(), mo[:, 0], rtol=1e-6, atol=1e-7 * np.sqrt(var))
    np.testing.assert_allclose(v[0].cpu().numpy(), vo[:, 0], rtol=1e-6, atol=1e-9 * var)


def test_dense_paths_read_lower_triangle_of_linv_only(ctx):
    """V = L⁻¹K* (launch_gemm_ltri_nn, dense posterior and full covariance) reads only the lower
    triangle of L⁻¹, as the fused kernel's packed L⁻¹ does: junk above the diagonal changes nothing."""
    from optimobo_amd.gp import GPState
    rng = np.random.default_rng(41)
    n, d, N = 1100, 3, 777
    X = rng.uniform(0, 1, (n, d))
    y = np.sin(3 * X).sum(1)
    st = GPState(X, y, np.full(d, 0.7), float(np.var(y)))
    Xc = dev(rng.uniform(0, 1, (N, d)))
    ctx.set_gp_state(0, st)
    mu, var = ctx.posterior(Xc, n_obj=1)
    mc, cov = ctx.posterior_cov(0, Xc[:300])
    assert np.all(np.triu(st.Linv, 1) == 0)
    st.Linv = st.Linv + np.triu(rng.uniform(-1e3, 1e3, (n, n)), 1)
    ctx.set_gp_state(0, st)
    mu2, var2 = ctx.posterior(Xc, n_obj=1)
    mc2, cov2 = ctx.posterior_cov(0, Xc[:300])
    assert torch.equal(mu, mu2) and torch.equal(var, var2)
    assert torch.equal(mc, mc2) and torch.equal(cov, cov2)


def test_dense_path_in_fused_chain(ctx):
    """The fused chain (plan → eval_argmax) runs the dense path too; same values as per-kernel calls."""
    from optimobo_amd import pareto
    from optimobo_amd.gp import GPState
    rng = np.random.default_rng(77)
    n, d, N = 1100, 4, 5000
    X = rng.uniform(0, 1, (n, d))
    Y = np.column_stack([X[:, 0], 1 - np.sqrt(X[:, 0]) + X[:, 1:].sum(1)])
    ls = np.full(d, 0.8)
    for o in range(2):
        ctx.set_gp_state(o, GPState(X, Y[:, o], ls, float(np.var(Y[:, o]))))
    pf = pareto.stripes_2d(pareto.calc_pf(Y))
    r = Y.max(0) + 0.1
    ctx.plan_ehvi2d(pf, r, 1.0, 0.0, mode="textbook")
    Xc = dev(rng.uniform(0, 1, (N, d)))
    fused = ctx.eval(Xc).cpu().numpy()
    mu, var = ctx.posterior(Xc, n_obj=2)
    sep = ctx.ehvi2d(mu, var, dev(pf), r, 1.0, 0.0, mode="textbook").cpu().numpy()
    assert np.array_equal(fused, sep)
