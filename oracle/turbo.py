"""Oracle: TuRBO's Thompson-sampling arithmetic (fp64 numpy restatement).

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py.

* ``select`` restates TuRBO_1.select_candidates (optimobo/algorithms/turbo.py:142-153) and
  TuRBO_M._select_candidates (turbo.py:365-383): for every sample k in order, the pick is
  ``np.argmin`` over that sample's values of all (trust region, candidate) pairs, flattened
  row-major as ``np.unravel_index`` reads them, and the picked candidate's values are then set
  to +inf for every sample.  Pinned against the reference functions themselves
  (tests/golden/turbo.npz, made by tests/golden/make_golden.py).
* ``chol_samples`` is the sampling rule of the device path, μ + chol(Σ + jI) z.  The reference
  samples with ``numpy.random.multivariate_normal`` (an SVD of Σ, inside GPy's
  posterior_samples_f); both draw from N(μ, Σ) up to the jitter, so per-draw values are not
  comparable and the device path is checked against this restatement on the same z.
"""
import numpy as np


def select(y_cand):
    """y_cand (T, N, B) | (N, 1, B) | (N, B) → flat candidate indices (B,) in row-major (T, N) order."""
    y = np.array(y_cand, dtype=np.float64, copy=True)
    B = y.shape[-1]
    flat = y.reshape(-1, B)
    idx = np.empty(B, np.int64)
    for k in range(B):
        i = int(np.argmin(flat[:, k]))
        idx[k] = i
        flat[i, :] = np.inf
    return idx


def chol_samples(mu, cov, Zt, jitter):
    """Y (B, N): row b = μ + L z_b, L = chol(Σ + jitter·I), z_b = Zt[b]."""
    L = np.linalg.cholesky(np.asarray(cov, np.float64) + jitter * np.eye(len(cov)))
    return np.asarray(mu, np.float64)[None, :] + np.asarray(Zt, np.float64) @ L.T
