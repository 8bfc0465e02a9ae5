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
