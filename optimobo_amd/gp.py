"""Gaussian-process surrogate: host-side fit, device-side prediction.

Mirrors the part of GPy the reference uses (optimobo/algorithms/optimisers.py:223-231):

    model = GPRegression(X, y, Matern52(n_var, ARD=True))
    model.Gaussian_noise.variance.fix(0)
    model.optimize(messages=False, max_f_eval=1000)
    mu, var = model.predict(x[None, :])          # (1,1), (1,1)

The fit (kernel matrix, jittered Cholesky, α, L⁻¹, and the L-BFGS hyperparameter search) is
O(n³) once per BO iteration and runs on the host.  ``predict`` — the
hot path — runs on the GPU through the HIP posterior kernel (optimobo_amd.device); there is
no CPU prediction path.
"""
import numpy as np
from scipy import linalg, optimize

SQRT5 = np.sqrt(5.0)
JITTER = 1e-8     # GPy ExactGaussianInference adds σ_n² + 1e-8 to the diagonal


# ----------------------------------------------------------------------------- kernels
class _Param:
    """Minimal stand-in for a paramz parameter (``.fix()`` / ``.values``)."""

    def __init__(self, value):
        self.values = np.atleast_1d(np.asarray(value, np.float64)).copy()
        self.fixed = False

    def fix(self, value=None):
        if value is not None:
            self.values[:] = value
        self.fixed = True

    def unfix(self):
        self.fixed = False

    def __float__(self):
        return float(self.values[0])


class _Stationary:
    name = "stationary"
    kind = "matern52"

    def __init__(self, input_dim, variance=1.0, lengthscale=None, ARD=False):
        self.input_dim = int(input_dim)
        self.ARD = bool(ARD)
        n_ls = self.input_dim if ARD else 1
        ls = 1.0 if lengthscale is None else lengthscale
        self.variance = _Param(variance)
        self.lengthscale = _Param(np.broadcast_to(np.asarray(ls, np.float64), (n_ls,)))

    def ls_vector(self):
        return np.broadcast_to(self.lengthscale.values, (self.input_dim,)).astype(np.float64)

    def scaled_dist(self, X, X2=None):
        """GPy Stationary._scaled_dist: expanded-norm r on ℓ-scaled inputs, clipped at 0."""
        ls = self.ls_vector()
        a = X / ls
        asq = np.sum(np.square(a), 1)
        if X2 is None:
            r2 = -2.0 * (a @ a.T) + (asq[:, None] + asq[None, :])
            np.fill_diagonal(r2, 0.0)
        else:
            b = X2 / ls
            r2 = -2.0 * (a @ b.T) + (asq[:, None] + np.sum(np.square(b), 1)[None, :])
        return np.sqrt(np.clip(r2, 0.0, np.inf))

    def K(self, X, X2=None):
        return self.K_of_r(self.scaled_dist(X, X2))


class Matern52(_Stationary):
    """GPy.kern.Matern52: σ_f² (1 + √5 r + 5/3 r²) exp(−√5 r)."""
    name = "Mat52"
    kind = "matern52"

    def K_of_r(self, r):
        return float(self.variance) * (1.0 + SQRT5 * r + 5.0 / 3.0 * r ** 2) * np.exp(-SQRT5 * r)

    def dK_dr_over_r(self, r):
        # dK/dr / r = −5/3 σ_f² (1 + √5 r) exp(−√5 r)
        return -5.0 / 3.0 * float(self.variance) * (1.0 + SQRT5 * r) * np.exp(-SQRT5 * r)


class RBF(_Stationary):
    """GPy.kern.RBF: σ_f² exp(−r²/2)."""
    name = "rbf"
    kind = "rbf"

    def K_of_r(self, r):
        return float(self.variance) * np.exp(-0.5 * r ** 2)

    def dK_dr_over_r(self, r):
        return -float(self.variance) * np.exp(-0.5 * r ** 2)


# ----------------------------------------------------------------------------- fitted state
def jitchol(A, maxtries=5):
    """Cholesky with GPy's escalating jitter (GPy.util.linalg.jitchol)."""
    A = np.ascontiguousarray(A)
    L, info = linalg.lapack.dpotrf(A, lower=1)
    if info == 0:
        return np.tril(L)
    diagA = np.diag(A)
    if np.any(diagA <= 0.0):
        raise linalg.LinAlgError("not pd: non-positive diagonal elements")
    jitter = diagA.mean() * 1e-6
    for _ in range(maxtries):
        try:
            return linalg.cholesky(A + np.eye(A.shape[0]) * jitter, lower=True)
        except linalg.LinAlgError:
            jitter *= 10
    raise linalg.LinAlgError("not positive definite, even with jitter.")


class GPState:
    """Everything the device needs for one objective: X, ℓ, σ_f², α, L⁻¹."""

    def __init__(self, X, y, lengthscale, variance, kernel="matern52", noise=0.0):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.y = np.asarray(y, np.float64).reshape(-1, 1)
        n, d = self.X.shape
        self.lengthscale = np.broadcast_to(np.asarray(lengthscale, np.float64), (d,)).copy()
        self.variance = float(variance)
        self.kernel = kernel
        self.noise = float(noise)
        kern = (Matern52 if kernel == "matern52" else RBF)(d, self.variance, self.lengthscale, ARD=True)
        Ky = kern.K(self.X) + np.eye(n) * (self.noise + JITTER)
        self.L = jitchol(Ky)
        self.alpha, _ = linalg.lapack.dpotrs(self.L, self.y, lower=1)
        self.Linv = linalg.solve_triangular(self.L, np.eye(n), lower=True)

    @property
    def n(self):
        return self.X.shape[0]


# ----------------------------------------------------------------------------- GPRegression
class _Noise:
    def __init__(self):
        self.variance = _Param(1.0)


class GPRegression:
    """GPy.models.GPRegression subset: exact inference, fixed or fitted noise, device predict."""

    def __init__(self, X, Y, kernel=None, noise_var=1.0):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.Y = np.asarray(Y, np.float64).reshape(-1, 1)
        self.kern = kernel if kernel is not None else Matern52(self.X.shape[1], ARD=True)
        self.Gaussian_noise = _Noise()
        self.Gaussian_noise.variance.values[:] = noise_var
        self.likelihood = self.Gaussian_noise
        self._state = None
        self._ctx = None

    # -- fitted state
    def state(self):
        if self._state is None:
            self._state = GPState(self.X, self.Y, self.kern.ls_vector(), float(self.kern.variance), self.kern.kind,
                                  noise=float(self.Gaussian_noise.variance))
        return self._state

    def log_likelihood(self):
        return -self._neg_lml_and_grad(self._get_free())[0]

    # -- hyperparameter fit (GPy model.optimize: L-BFGS-B, max_f_eval)
    def _get_free(self):
        vals = [np.log(float(self.kern.variance))] + list(np.log(self.kern.lengthscale.values))
        if not self.Gaussian_noise.variance.fixed:
            vals.append(np.log(max(float(self.Gaussian_noise.variance), 1e-12)))
        return np.asarray(vals)

    def _set_free(self, theta):
        self.kern.variance.values[:] = np.exp(theta[0])
        nl = self.kern.lengthscale.values.size
        self.kern.lengthscale.values[:] = np.exp(theta[1:1 + nl])
        if not self.Gaussian_noise.variance.fixed:
            self.Gaussian_noise.variance.values[:] = np.exp(theta[1 + nl])
        self._state = None

    def _neg_lml_and_grad(self, theta):
        self._set_free(theta)
        n, d = self.X.shape
        kern = self.kern
        r = kern.scaled_dist(self.X)
        K = kern.K_of_r(r)
        noise = float(self.Gaussian_noise.variance)
        Ky = K + np.eye(n) * (noise + JITTER)
        try:
            L = jitchol(Ky)
        except linalg.LinAlgError:
            return 1e25, np.zeros_like(theta)
        alpha = linalg.cho_solve((L, True), self.Y)
        lml = -0.5 * float(self.Y.T @ alpha) - np.sum(np.log(np.diag(L))) - 0.5 * n * np.log(2 * np.pi)
        Kinv = linalg.cho_solve((L, True), np.eye(n))
        W = alpha @ alpha.T - Kinv                        # dLML/dK = 0.5 W
        g = [0.5 * np.sum(W * K)]                          # d/dlog σ_f²
        ls = kern.ls_vector()
        dKdr_r = kern.dK_dr_over_r(r)
        nl = kern.lengthscale.values.size
        for j in range(nl):
            if nl == 1:
                D2 = np.square(r)                          # Σ_j Δ_j²/ℓ²
            else:
                D2 = np.square(self.X[:, j:j + 1] - self.X[:, j:j + 1].T) / ls[j] ** 2
            # ∂K/∂log ℓ_j = −(dK/dr / r)·Δ_j²/ℓ_j²
            g.append(0.5 * np.sum(W * (-dKdr_r * D2)))
        if not self.Gaussian_noise.variance.fixed:
            g.append(0.5 * np.trace(W) * noise)
        return -lml, -np.asarray(g)

    def optimize(self, messages=False, max_f_eval=1000, max_iters=None):
        theta0 = self._get_free()
        bounds = [(np.log(1e-10), np.log(1e10))] * len(theta0)
        res = optimize.minimize(self._neg_lml_and_grad, theta0, jac=True, method="L-BFGS-B", bounds=bounds,
                                options={"maxfun": int(max_f_eval), "maxiter": int(max_iters or max_f_eval)})
        self._set_free(res.x)
        return res

    def optimize_restarts(self, num_restarts=10, robust=True, verbose=False, **kw):
        rng = np.random.default_rng(kw.pop("seed", None))
        best = None
        for i in range(num_restarts):
            if i > 0:
                self._set_free(self._get_free() + rng.normal(0, 1, len(self._get_free())))
            res = self.optimize(**kw)
            if best is None or res.fun < best[0]:
                best = (res.fun, res.x.copy())
        self._set_free(best[1])

    # -- device prediction (hot path)
    def _context(self):
        from .device import AcqContext
        if self._ctx is None:
            self._ctx = AcqContext(0)
        return self._ctx

    def predict(self, Xnew, full_cov=False):
        """μ (m,1), σ² (m,1) at Xnew on the GPU (GPy GPRegression.predict semantics)."""
        if full_cov:
            raise NotImplementedError("full_cov prediction is not on the acquisition hot path")
        import torch
        ctx = self._context()
        ctx.set_gp_state(0, self.state())
        Xnew = np.atleast_2d(np.asarray(Xnew, np.float64))
        mu, var = ctx.posterior(torch.as_tensor(Xnew, device=ctx.device), n_obj=1)
        noise = float(self.Gaussian_noise.variance)
        return mu[0].cpu().numpy()[:, None], var[0].cpu().numpy()[:, None] + noise


class kern:  # noqa: N801  — GPy.kern namespace look-alike
    Matern52 = Matern52
    RBF = RBF


class models:  # noqa: N801  — GPy.models namespace look-alike
    GPRegression = GPRegression
