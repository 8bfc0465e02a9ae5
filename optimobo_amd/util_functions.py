"""Drop-in ``optimobo.util_functions`` (util_functions.py:1-517) backed by the GPU.

Acquisition functions keep the reference signatures and return types for a single
candidate ``X`` of shape (n_var,), and also accept a batch (N, n_var), returning (N,).
``models`` are ``optimobo_amd.gp.GPRegression`` objects (or fitted ``GPState``s); the batch
goes through the HIP posterior and acquisition kernels.  The per-iteration geometry helpers
(calc_pf, decompose_into_cells, wfg) and the sample transform ``change`` are small host code.
"""
import numpy as np
from scipy import stats

from . import pareto
from .acquisition import engine_for


def _batch(X):
    X = np.asarray(X, np.float64)
    return (X[None, :], True) if X.ndim == 1 else (X, False)


# ----------------------------------------------------------------------------- host helpers
def generate_latin_hypercube_samples(num_samples, variable_ranges):
    """util_functions.py:46-61: one stratified sample per interval and dimension, shuffled."""
    num_vars = len(variable_ranges)
    samples = np.empty((num_samples, num_vars))
    for i, (lo, hi) in enumerate(variable_ranges):
        edges = np.linspace(lo, hi, num_samples + 1)
        u = (np.random.rand(num_samples) + np.arange(num_samples)) / num_samples
        samples[:, i] = np.random.permutation(edges[:-1] + (edges[1:] - edges[:-1]) * u)
    return samples


def calc_pf(Y):
    """util_functions.py:64-77 (first non-dominated front)."""
    return pareto.calc_pf(Y)


def change(predicitions, samples, dimensions):
    """util_functions.py:217-237: cached normal samples translated by the predictions.

    Bug-compatible: every column is scaled by objective 0's variance (quirk 1).
    """
    mus = [np.asarray(predicitions[i][0]).reshape(-1)[0] for i in range(dimensions)]
    sd = np.sqrt(np.asarray(predicitions[0][1]).reshape(-1)[0])
    return np.column_stack([samples[:, i] * sd + mus[i] for i in range(dimensions)])


def psi_cal(a, b, m, s):
    """util_functions.py:130-133."""
    t = np.asarray((b - m) / s).reshape(-1)
    return s * stats.norm.pdf(t[0]) + (a - m) * stats.norm.cdf(t[0])


def decompose_into_cells(data_points, ideal_point, max_point, n_obj=2):
    """util_functions.py:414-517 / emo.py:55-152 (2 objectives, reference-exact)."""
    if n_obj != 2:
        raise NotImplementedError("decompose_into_cells: only 2-objective problems (as the reference)")
    return pareto.decompose_into_cells(data_points, ideal_point, max_point)


def wfg(pl, ref_point):
    """Hypervolume of ``pl`` w.r.t. ``ref_point`` (util_functions.py:365-376)."""
    return pareto.hypervolume(pl, ref_point)


def inclhv(p, ref_point):
    """util_functions.py:403-410: volume of one point's box (2 objectives)."""
    return float(np.prod([abs(p[j] - ref_point[j]) for j in range(2)]))


# ----------------------------------------------------------------------------- acquisitions (GPU)
def EHVI_2D_aux(PF, r, mu, sigma):
    """util_functions.py:81-128 with σ given directly.

    Single evaluation (as the reference): mu (2,), sigma whose flattened first two entries are
    (σA, σB) — e.g. the flattened 2×2 covariance EHVI passes — returns (1,).
    Batch: mu (2, N), sigma (2, N) → (N,).
    """
    from .acquisition import AcquisitionEngine, _ENGINES
    eng = next(iter(_ENGINES.values()), None) or AcquisitionEngine()
    mu = np.asarray(mu, np.float64)
    sigma = np.asarray(sigma, np.float64)
    if mu.size == 2:
        out = eng.ehvi_2d_aux(PF, r, mu.reshape(2, 1), sigma.reshape(-1)[:2].reshape(2, 1)).cpu().numpy()
        return out[:1]
    return eng.ehvi_2d_aux(PF, r, mu.reshape(2, -1), sigma.reshape(2, -1)).cpu().numpy()


def EHVI(X, models, max_point, PF, cache, mode="reference"):
    """util_functions.py:136-167 — 2-objective EHVI; (1,) for one x, (N,) for a batch.

    mode "reference" reproduces the reference exactly (covariance-as-σ, last stripe omitted);
    "textbook" is the exact EHVI.
    """
    Xb, single = _batch(X)
    out = engine_for(models).ehvi(Xb, max_point, PF, cache, mode=mode).cpu().numpy()
    return out[:1] if single else out


def EHVI_3D(X, models, max_point, PF, cache, mode="reference"):
    """util_functions.py:170-214.  One x: float, ValueError where pygmo raises.

    Any number of objectives k = len(models) ≥ 3, as the reference (which calls it for every n_obj != 2,
    optimisers.py:245-248): the per-sample volume is pygmo's k-D single-point hypervolume.
    mode "reference": the reference's Monte-Carlo form; batch → (values (N,), raised (N,) bool),
    NaN where the reference would raise.  mode "textbook" (k = 3): the exact EHVI over a box
    decomposition (no MC error, never raises); batch → (N,).
    """
    Xb, single = _batch(X)
    if mode == "textbook":
        out = engine_for(models).ehvi_exact(Xb, max_point, PF).cpu().numpy()
        return float(out[0]) if single else out
    vals, raised = engine_for(models).ehvi3d(Xb, max_point, PF, cache)
    vals, raised = vals.cpu().numpy(), raised.cpu().numpy().astype(bool)
    if single:
        if raised[0]:
            raise ValueError("Reference point is invalid: a sample of the predictive distribution lies outside it")
        return float(vals[0])
    return vals, raised


def expected_decomposition(X, models, weights, agg_func, agg_function_min, cache):
    """util_functions.py:285-327.  One x: float; batch: (N,)."""
    Xb, single = _batch(X)
    out = engine_for(models).expected_decomposition(Xb, weights, agg_func, agg_function_min, cache).cpu().numpy()
    return float(out[0]) if single else out


def expected(X, models, agg_func, cache, weights):
    """util_functions.py:7-43 (plotting helper): mean and ±2σ band of the scalarised samples."""
    preds = [m.predict(np.asarray([X])) for m in models]
    vals = np.asarray(agg_func(change(preds, cache, len(models)), weights))
    total, std = np.mean(vals), np.std(vals)
    return total, total + 2 * std, total - 2 * std
