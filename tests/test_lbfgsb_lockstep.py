"""CPU: the reverse-communication L-BFGS-B driver behind gp.fit_concurrently (optimobo_amd.gp._LbfgsbRun)
takes bitwise the path of scipy.optimize.minimize(method="L-BFGS-B") — same iterates, evaluation count,
iteration count and optimum — on smooth and badly scaled functions, including points scipy re-uses."""
import numpy as np
import pytest
from scipy import optimize

from optimobo_amd.gp import _LbfgsbRun


def _quartic(x):
    return float(np.sum((x - 1.5) ** 4) + np.sum(np.cos(x))), 4 * (x - 1.5) ** 3 - np.sin(x)


def _rosen(x):
    return float(optimize.rosen(x)), optimize.rosen_der(x)


def _scaled(x):
    w = 10.0 ** np.arange(len(x))
    return float(np.sum(w * x ** 2) + np.exp(x[0])), 2 * w * x + np.array([np.exp(x[0])] + [0.0] * (len(x) - 1))


@pytest.mark.parametrize("fun", [_quartic, _rosen, _scaled])
@pytest.mark.parametrize("x0", [np.array([0.3, -1.0, 2.0]), np.array([5.0, 5.0]), np.array([-1.2, 1.0, 0.4, 2.5])])
@pytest.mark.parametrize("maxfun", [1000, 7])
def test_lockstep_lbfgsb_equals_scipy(fun, x0, maxfun):
    ref = optimize.minimize(fun, x0, jac=True, method="L-BFGS-B", options={"maxfun": maxfun, "maxiter": 1000})
    f0, g0 = fun(x0)
    r = _LbfgsbRun(x0, f0, g0, maxfun, 1000)
    while True:
        x = r.advance()
        if x is None:
            break
        f, g = fun(x)
        r.supply(x, f, g)
    assert np.array_equal(ref.x, r.x)
    assert ref.nfev == r.nfev and ref.nit == r.nit and ref.fun == r.f


@pytest.fixture
def fresh_lockstep_check(monkeypatch):
    from optimobo_amd import gp
    monkeypatch.setattr(gp, "_LOCKSTEP_OK", None)
    return gp


def test_lockstep_disabled_without_routine(fresh_lockstep_check, monkeypatch):
    """Another scipy layout (no private setulb): the one-time check fails and fits run one after another."""
    gp = fresh_lockstep_check
    monkeypatch.setattr(gp, "_lbfgsb_routine", lambda: None)
    assert gp._lockstep_ok() is False


def test_lockstep_disabled_when_routine_differs(fresh_lockstep_check, monkeypatch):
    """A setulb whose iterates differ from scipy.optimize.minimize's (here: a perturbed gradient) fails the
    equivalence check, as would one with another signature."""
    gp = fresh_lockstep_check
    real = gp._lbfgsb_routine()

    def perturbed(m, x, low, up, nbd, f, g, *rest):
        return real(m, x, low, up, nbd, f, g * (1 + 1e-3), *rest)
    monkeypatch.setattr(gp, "_lbfgsb_routine", lambda: perturbed)
    assert gp._lockstep_ok() is False
    monkeypatch.setattr(gp, "_LOCKSTEP_OK", None)
    monkeypatch.setattr(gp, "_lbfgsb_routine", lambda: (lambda *a: (_ for _ in ()).throw(TypeError("signature"))))
    assert gp._lockstep_ok() is False


def test_sequential_fallback_fits_like_single_fits(fresh_lockstep_check, monkeypatch):
    """With the lockstep driver disabled, fit_concurrently gives each model exactly its single fit."""
    gp = fresh_lockstep_check
    monkeypatch.setattr(gp, "_LOCKSTEP_OK", False)
    rng = np.random.default_rng(4)
    X = rng.uniform(0, 1, (18, 2))
    Y = np.column_stack([np.sin(5 * X[:, 0]) + X[:, 1], (X ** 2).sum(1)])

    def models():
        return [gp.GPRegression(X, Y[:, i:i + 1], gp.Matern52(2, ARD=True), device_fit=False) for i in range(2)]
    ms, singles = models(), models()
    for m in ms + singles:
        m.Gaussian_noise.variance.fix(0)
    res = gp.fit_concurrently(ms, max_f_eval=200)
    for m, s, r in zip(ms, singles, res):
        rs = s.optimize(max_f_eval=200)
        assert np.array_equal(r.x, rs.x)
        assert np.array_equal(m.kern.lengthscale.values, s.kern.lengthscale.values)
