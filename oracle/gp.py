"""Oracle: GPy Matern-5/2 ARD exact-inference GP posterior (fp64 numpy restatement).

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

The reference builds every surrogate as
``GPy.models.GPRegression(X, y, GPy.kern.Matern52(n_var, ARD=True))`` with the Gaussian
noise variance fixed to 0 (optimobo/algorithms/optimisers.py:226-231, emo.py:297-301,
parego.py:217-219) and calls ``model.predict(x[None, :])`` once per candidate
(optimobo/util_functions.py:155-158, 187-190, 307-310; emo.py:203-205;
optimisers.py:336; parego.py:137).

GPy (``gpy>=1.10.0``, requirements.txt:5) is not vendored and not installed.  The
formulas below restate GPy's published algorithm:
  * ``Stationary._unscaled_dist``: r² = ‖a‖² + ‖b‖² − 2a·b on ℓ-scaled inputs, clipped
    at 0 (diagonal forced to 0 for K(X, X)), r = sqrt(r²);
  * ``Matern52.K_of_r``: σ_f² (1 + √5 r + 5/3 r²) exp(−√5 r);
  * ``ExactGaussianInference.inference``: Ky = K + (σ_n² + 1e-8) I, L = jitchol(Ky),
    α = Ky⁻¹ y via dpotrs;
  * ``PosteriorExact._raw_predict``: μ = K*ᵀ α, σ² = Kdiag − Σ_rows (L⁻¹ K*)² with
    L⁻¹ K* from dtrtrs (triangular solve); ``GPRegression.predict`` adds σ_n² = 0 and
    no normalizer.
Pinned against scikit-learn's independent GaussianProcessRegressor in
tests/test_oracle.py (golden fixtures tests/golden/posterior_*.npz).
"""
import numpy as np
from scipy import linalg

SQRT5 = np.sqrt(5.0)


def scaled_dist(X, X2, lengthscale):
    """GPy Stationary._scaled_dist / _unscaled_dist (expanded-norm form, clip ≥ 0)."""
    a = np.asarray(X, dtype=np.float64) / lengthscale
    if X2 is None:
        asq = np.sum(np.square(a), 1)
        r2 = -2.0 * (a @ a.T) + (asq[:, None] + asq[None, :])
        np.fill_diagonal(r2, 0.0)
    else:
        b = np.asarray(X2, dtype=np.float64) / lengthscale
        asq = np.sum(np.square(a), 1)
        bsq = np.sum(np.square(b), 1)
        r2 = -2.0 * (a @ b.T) + (asq[:, None] + bsq[None, :])
    r2 = np.clip(r2, 0.0, np.inf)
    return np.sqrt(r2)


def matern52_K(X, X2, lengthscale, variance):
    """GPy Matern52.K_of_r applied to the scaled distance."""
    r = scaled_dist(X, X2, lengthscale)
    return variance * (1.0 + SQRT5 * r + 5.0 / 3.0 * r ** 2) * np.exp(-SQRT5 * r)


def rbf_K(X, X2, lengthscale, variance):
    """GPy RBF.K_of_r: σ_f² exp(−r²/2) (the north_star's "RBF" kernel id)."""
    r = scaled_dist(X, X2, lengthscale)
    return variance * np.exp(-0.5 * r ** 2)


KERNELS = {"matern52": matern52_K, "rbf": rbf_K}


def jitchol(A, maxtries=5):
    """GPy.util.linalg.jitchol: Cholesky with escalating diagonal jitter."""
    A = np.ascontiguousarray(A)
    L, info = linalg.lapack.dpotrf(A, lower=1)
    if info == 0:
        return np.tril(L)
    diagA = np.diag(A)
    if np.any(diagA <= 0.0):
        raise linalg.LinAlgError("not pd: non-positive diagonal elements")
    jitter = diagA.mean() * 1e-6
    num_tries = 1
    while num_tries <= maxtries and np.isfinite(jitter):
        try:
            return linalg.cholesky(A + np.eye(A.shape[0]) * jitter, lower=True)
        except linalg.LinAlgError:
            jitter *= 10
        finally:
            num_tries += 1
    raise linalg.LinAlgError("not positive definite, even with jitter.")


class ExactGP:
    """State of one fitted GPy GPRegression (noise fixed to 0) — the oracle side."""

    def __init__(self, X, y, lengthscale, variance, kernel="matern52", noise=0.0):
        self.X = np.asarray(X, dtype=np.float64)
        self.y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
        self.lengthscale = np.broadcast_to(np.asarray(lengthscale, np.float64), (self.X.shape[1],)).copy()
        self.variance = float(variance)
        self.kernel = kernel
        self.noise = float(noise)
        K = KERNELS[kernel](self.X, None, self.lengthscale, self.variance)
        Ky = K + np.eye(len(K)) * (self.noise + 1e-8)
        self.L = jitchol(Ky)
        self.alpha, _ = linalg.lapack.dpotrs(self.L, self.y, lower=1)

    def predict(self, Xnew):
        """μ (m,1), σ² (m,1) exactly as GPy PosteriorExact._raw_predict (+ σ_n² = 0)."""
        Xnew = np.atleast_2d(np.asarray(Xnew, dtype=np.float64))
        Kx = KERNELS[self.kernel](self.X, Xnew, self.lengthscale, self.variance)
        mu = Kx.T @ self.alpha
        tmp = linalg.solve_triangular(self.L, Kx, lower=True)
        var = (self.variance - np.square(tmp).sum(0))[:, None] + self.noise
        return mu, var

    def predict_full_cov(self, Xnew):
        """μ (m,), Σ (m, m) as GPy PosteriorExact._raw_predict(full_cov=True): Kxx − tdot(tmp.T),
        tmp = dtrtrs(L, Kx), plus σ_n² I (= 0) from GPRegression.predict (the call inside
        GP.posterior_samples that TuRBO makes, optimobo/algorithms/turbo.py:114)."""
        Xnew = np.atleast_2d(np.asarray(Xnew, dtype=np.float64))
        Kx = KERNELS[self.kernel](self.X, Xnew, self.lengthscale, self.variance)
        mu = (Kx.T @ self.alpha)[:, 0]
        tmp = linalg.solve_triangular(self.L, Kx, lower=True)
        Kxx = KERNELS[self.kernel](Xnew, None, self.lengthscale, self.variance)
        return mu, Kxx - tmp.T @ tmp + self.noise * np.eye(len(Xnew))


def sklearn_posterior(X, y, lengthscale, variance, Xnew):
    """Independent pin: scikit-learn GaussianProcessRegressor with the same kernel."""
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import ConstantKernel, Matern

    kern = ConstantKernel(variance, "fixed") * Matern(length_scale=np.asarray(lengthscale, np.float64),
                                                      length_scale_bounds="fixed", nu=2.5)
    gpr = GaussianProcessRegressor(kernel=kern, alpha=1e-8, optimizer=None, normalize_y=False)
    gpr.fit(X, np.asarray(y, np.float64).ravel())
    mu, cov_diag = _sk_mean_var(gpr, Xnew)
    return mu, cov_diag


def _sk_mean_var(gpr, Xnew):
    # sklearn only exposes std (sqrt-ed, clipped); recompute the variance from its own factors.
    K_trans = gpr.kernel_(Xnew, gpr.X_train_)
    mu = K_trans @ gpr.alpha_
    V = linalg.solve_triangular(gpr.L_, K_trans.T, lower=True, check_finite=False)
    var = gpr.kernel_.diag(Xnew) - np.einsum("ij,ji->i", V.T, V)
    return mu, var
