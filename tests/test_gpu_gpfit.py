"""GPU: the GP fit on the device (omb_gp_lml_grad, omb_gp_fit_state) — GPy's exact-inference log
marginal likelihood and its gradient against scikit-learn (an independent implementation,
pinned in tests/test_oracle.py) and against the host numpy fit; the device-factorised state
against the oracle posterior.

Tolerances: log marginal likelihood 1e-7 relative (+1e-6 absolute); gradient 1e-5 relative to
its largest entry; posterior as tests/test_gpu_parity.py (1e-6 relative, floors 1e-7·σ_f on μ
and 1e-9·σ_f² on σ²).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import gp as ogp  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    from optimobo_amd.device import AcqContext
    c = AcqContext(0)
    yield c
    c.close()


def data(n, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(0, 1, (n, d))
    y = np.sin(3 * X).sum(1) + 0.3 * X[:, 0] ** 2
    ls = rng.uniform(0.3, 2.0, d)
    return X, y, ls, max(float(np.var(y)), 0.5)


def sklearn_lml_grad(X, y, ls, var, nu=2.5):
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, ConstantKernel, Matern
    base = Matern(length_scale=ls, nu=nu) if nu else RBF(length_scale=ls)
    gpr = GaussianProcessRegressor(kernel=ConstantKernel(var) * base, alpha=1e-8, optimizer=None).fit(X, y)
    lml, g = gpr.log_marginal_likelihood(gpr.kernel_.theta, eval_gradient=True)
    return lml, g


@pytest.mark.parametrize("n,d", [(1, 1), (20, 2), (96, 8), (97, 2), (100, 6), (64, 9), (129, 3), (300, 6),
                                 (257, 30), (700, 4), (150, 50),
                                 (12, 100), (150, 100), (70, 256)])   # n_var > 64: wide K and gradient kernels
def test_lml_grad_vs_sklearn(ctx, n, d):
    X, y, ls, var = data(n, d, n + d)
    lml, g, jit = ctx.gp_lml_grad(X, y, ls, var)
    lml_s, g_s = sklearn_lml_grad(X, y, ls, var)
    assert jit == 0.0
    assert lml == pytest.approx(lml_s, rel=1e-7, abs=1e-6)
    np.testing.assert_allclose(g, g_s, rtol=1e-5, atol=1e-5 * np.max(np.abs(g_s)))


def test_rbf_lml_grad_vs_sklearn(ctx):
    X, y, ls, var = data(80, 3, 5)
    lml, g, _ = ctx.gp_lml_grad(X, y, ls, var, kernel="rbf")
    lml_s, g_s = sklearn_lml_grad(X, y, ls, var, nu=None)
    assert lml == pytest.approx(lml_s, rel=1e-7, abs=1e-6)
    np.testing.assert_allclose(g, g_s, rtol=1e-5, atol=1e-5 * np.max(np.abs(g_s)))


def test_lml_grad_matches_host_fit(ctx):
    """The device evaluation is the host numpy one (optimobo_amd.gp, log parametrisation)."""
    from optimobo_amd.gp import GPRegression, Matern52
    X, y, ls, var = data(150, 5, 9)
    m = GPRegression(X, y[:, None], Matern52(5, variance=var, lengthscale=ls, ARD=True), device_fit=False)
    m.Gaussian_noise.variance.fix(0)
    theta = m._get_free()
    f_h, g_h = m._neg_lml_and_grad(theta)
    md = GPRegression(X, y[:, None], Matern52(5, variance=var, lengthscale=ls, ARD=True), device_fit=True)
    md.Gaussian_noise.variance.fix(0)
    f_d, g_d = md._neg_lml_and_grad_device(theta)
    assert f_d == pytest.approx(f_h, rel=1e-7, abs=1e-6)
    np.testing.assert_allclose(g_d, g_h, rtol=1e-5, atol=1e-5 * np.max(np.abs(g_h)))


@pytest.mark.parametrize("n,d", [(400, 6), (200, 100)])
def test_fit_state_posterior_matches_oracle(ctx, n, d):
    X, y, ls, var = data(n, d, 13)
    if d > 8:
        ls = ls * np.sqrt(d)                 # a correlated surface at n_var = 100
    jit = ctx.gp_fit_state(0, X, y, ls, var)
    assert jit == 0.0
    Xc = np.random.default_rng(14).uniform(0, 1, (3000, d))
    Xc[:5] = X[:5]
    mu, v = ctx.posterior(torch.as_tensor(Xc, device="cuda:0"), n_obj=1)
    mo, vo = ogp.ExactGP(X, y, ls, var).predict(Xc)
    np.testing.assert_allclose(mu[0].cpu().numpy(), mo[:, 0], rtol=1e-6, atol=1e-7 * np.sqrt(var))
    np.testing.assert_allclose(v[0].cpu().numpy(), vo[:, 0], rtol=1e-6, atol=1e-9 * var)


def test_device_optimize_reaches_host_optimum():
    from optimobo_amd.gp import GPRegression, Matern52
    X, y, ls, var = data(60, 3, 17)
    out = []
    for dev_fit in (False, True):
        m = GPRegression(X, y[:, None], Matern52(3, ARD=True), device_fit=dev_fit)
        m.Gaussian_noise.variance.fix(0)
        m.optimize(max_f_eval=300)
        out.append(m._neg_lml_and_grad(m._get_free())[0])
    assert out[1] <= out[0] + 1e-4 * abs(out[0])


def test_gp_fit_errors(ctx):
    from optimobo_amd import _lib
    X, y, ls, var = data(10, 2, 1)
    with pytest.raises(_lib.OMBError) as e:
        ctx.gp_lml_grad(X, y, [0.5, -1.0], var)
    assert e.value.code == _lib.OMB_EINVAL
    import ctypes
    rc = ctx.lib.omb_gp_fit_state(ctx._h, 0, 0, _lib.MAX_TRAIN_DENSE + 1, 2, ctypes.c_void_p(8), ctypes.c_void_p(8),
                                  _lib.darr([1, 1]), 1.0, 0.0, None)      # rejected before any access
    assert rc == _lib.OMB_EUNSUP


@pytest.mark.parametrize("n", [40, 96, 97])
def test_lml_grad_small_and_blocked_paths_agree_with_jitter(ctx, n):
    """Exact duplicate inputs with σ_f² = 1e10 (the 1e-8 jitter is below half an ulp of the diagonal)
    make K + 1e-8·I singular in fp64: both the one-workgroup path (n ≤ 128) and the blocked path must
    take GPy jitchol's jitter retries, and match the host evaluation at the jitter they report."""
    rng = np.random.default_rng(n)
    base = rng.uniform(0, 1, (6, 2))
    X = base[np.arange(n) % 6]
    y = np.sin(3 * X).sum(1)
    ls, var = np.array([0.5, 0.8]), 1e10
    lml, g, jit = ctx.gp_lml_grad(X, y, ls, var)
    assert jit > 0.0
    # host numpy at the same diagonal shift
    K = ogp.matern52_K(X, X, ls, var) + (1e-8 + jit) * np.eye(n)
    L = np.linalg.cholesky(K)
    a = np.linalg.solve(K, y)
    lml_h = -0.5 * y @ a - np.log(np.diag(L)).sum() - 0.5 * n * np.log(2 * np.pi)
    assert lml == pytest.approx(lml_h, rel=1e-6, abs=1e-4)
    assert np.all(np.isfinite(g))


def test_lml_grad_small_path_deterministic(ctx):
    X, y, ls, var = data(100, 4, 3)
    r1 = ctx.gp_lml_grad(X, y, ls, var)
    r2 = ctx.gp_lml_grad(X, y, ls, var)
    assert r1[0] == r2[0] and np.array_equal(r1[1], r2[1])


@pytest.mark.parametrize("n", [20, 60, 96, 119])
def test_concurrent_fits_match_sequential(n):
    """gp.fit_concurrently (the drivers' per-objective fits in lockstep, each round of evaluations one
    batched C call) gives bitwise the hyperparameters and predictions of fitting the same models one
    after another (n ≤ 96: one launch per round; n = 119: the blocked path, problem after problem)."""
    from optimobo_amd.gp import GPRegression, Matern52, fit_concurrently
    rng = np.random.default_rng(n)
    X = rng.uniform(-2, 2, (n, 2))
    Y = np.column_stack([100 * (X ** 2).sum(1), ((X[:, 0] - 1) ** 2 + X[:, 1] ** 2), np.sin(3 * X).sum(1)])

    def models():
        out = []
        for i in range(Y.shape[1]):
            m = GPRegression(X, Y[:, i:i + 1], Matern52(2, ARD=True))
            m.Gaussian_noise.variance.fix(0)
            out.append(m)
        return out

    seq = models()
    for m in seq:
        m.optimize(max_f_eval=1000)
    con = models()
    fit_concurrently(con, max_f_eval=1000)
    Xc = rng.uniform(-2, 2, (257, 2))
    for a, b in zip(seq, con):
        assert float(a.kern.variance) == float(b.kern.variance)
        assert np.array_equal(a.kern.lengthscale.values, b.kern.lengthscale.values)
        ma, va = a.predict(Xc)
        mb, vb = b.predict(Xc)
        assert np.array_equal(ma, mb) and np.array_equal(va, vb)


@pytest.mark.parametrize("n,d", [(20, 2), (60, 3), (96, 8), (119, 2), (40, 12)])
def test_lml_grad_batch_matches_single(ctx, n, d):
    """omb_gp_lml_grad_batch: every problem bitwise equal to its own omb_gp_lml_grad (one launch with a
    workgroup per problem for n ≤ 96, n_var ≤ 8; the blocked path one problem after another)."""
    rng = np.random.default_rng(n + d)
    X = torch.as_tensor(rng.uniform(0, 1, (n, d)), device="cuda:0")
    k = 3
    ys = [torch.as_tensor(rng.normal(size=n), device="cuda:0") for _ in range(k)]
    ls = rng.uniform(0.3, 2.0, (k, d))
    var = rng.uniform(0.5, 2.0, k)
    lml, grad, jit, status = ctx.gp_lml_grad_batch(X, ys, ls, var)
    assert (status == 0).all()
    for p in range(k):
        l1, g1, j1 = ctx.gp_lml_grad(X, ys[p], ls[p], float(var[p]))
        assert lml[p] == l1 and np.array_equal(grad[p], g1) and jit[p] == j1
