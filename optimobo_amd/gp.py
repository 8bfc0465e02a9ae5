"""Gaussian-process surrogate: host-side fit, device-side prediction.

Mirrors the part of GPy the reference uses (optimobo/algorithms/optimisers.py:223-231):

    model = GPRegression(X, y, Matern52(n_var, ARD=True))
    model.Gaussian_noise.variance.fix(0)
    model.optimize(messages=False, max_f_eval=1000)
    mu, var = model.predict(x[None, :])          # (1,1), (1,1)

The fit (kernel matrix, jittered Cholesky, α, L⁻¹, and the L-BFGS hyperparameter search) is
O(n³) per likelihood evaluation.  With a GPU it runs on the device: each
L-BFGS-B evaluation is one omb_gp_lml_grad call (K, Cholesky, L⁻¹, Ky⁻¹ and the gradient sums in
HIP; scipy's L-BFGS-B drives it on the host) and the final state is factorised in place by
omb_gp_fit_state.  Without a GPU (the CPU test suite) the same arithmetic runs in numpy.
``predict`` — the hot path — runs on the GPU through the HIP posterior kernel
(optimobo_amd.device); there is no CPU prediction path.
"""
import atexit
import concurrent.futures
import threading

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


class DeviceGPState:
    """Fitted state factorised on the device (omb_gp_fit_state): holds only X, y and θ on the host."""

    def __init__(self, X, y, lengthscale, variance, kernel="matern52", noise=0.0):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.y = np.asarray(y, np.float64).reshape(-1, 1)
        self.lengthscale = np.broadcast_to(np.asarray(lengthscale, np.float64), (self.X.shape[1],)).copy()
        self.variance = float(variance)
        self.kernel = kernel
        self.noise = float(noise)
        self.jitter = None

    @property
    def n(self):
        return self.X.shape[0]

    def upload(self, ctx, obj):
        self.jitter = ctx.gp_fit_state(obj, self.X, self.y, self.lengthscale, self.variance, self.noise, self.kernel)


def _device_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


# ----------------------------------------------------------------------------- concurrent fits
# The drivers fit one surrogate per objective from the same inputs (optimisers.py:223-231, called per
# objective at :186; emo.py:297-301).  The fits are independent and deterministic.  A device evaluation at
# the BO loop's sizes is ≈ 40 µs of launch and synchronisation that host threads do not overlap
# (tools/gpfit_threads_probe.py, profiles/r02_v64_threads_probe.txt), so the fits run in lockstep on ONE
# thread: each keeps its own L-BFGS-B state in scipy's reverse-communication routine (the loop of
# scipy.optimize._lbfgsb_py._minimize_lbfgsb, scipy 1.15, restated below), and every round of
# evaluations — one per fit still running — is one C call (omb_gp_lml_grad_batch: one launch with a
# workgroup per fit, one synchronisation).  Each fit takes exactly the path scipy.optimize.minimize takes
# for it alone (test_concurrent_fits_match_sequential: bitwise equal hyperparameters).


def _lbfgsb_routine():
    try:
        from scipy.optimize import _lbfgsb
        return _lbfgsb.setulb
    except Exception:  # pragma: no cover - another scipy layout: fit one after another
        return None


_LOCKSTEP_OK = None


def _lockstep_ok():
    """The restated loop matches this scipy's L-BFGS-B (checked once on a small problem); otherwise the
    fits run one after another through scipy.optimize.minimize."""
    global _LOCKSTEP_OK
    if _LOCKSTEP_OK is None:
        try:
            def fg(x):
                return float(np.sum((x - 1.5) ** 4) + np.sum(np.cos(x))), 4 * (x - 1.5) ** 3 - np.sin(x)
            x0 = np.array([0.3, -1.0, 2.0])
            ref = optimize.minimize(fg, x0, jac=True, method="L-BFGS-B", options={"maxfun": 1000, "maxiter": 1000})
            r = _LbfgsbRun(x0, *fg(x0), 1000, 1000)
            while True:
                x = r.advance()
                if x is None:
                    break
                r.supply(x, *fg(x))
            _LOCKSTEP_OK = bool(np.array_equal(ref.x, r.x) and ref.nfev == r.nfev)
        except Exception:  # pragma: no cover - no routine, or one with another signature
            _LOCKSTEP_OK = False
    return _LOCKSTEP_OK


class _LbfgsbRun:
    """scipy.optimize._lbfgsb_py._minimize_lbfgsb without bounds, driven from outside: ``advance``
    runs the routine until it needs f and g at a point not evaluated last (returned) or it stops (None);
    ScalarFunction's rule (re-use the last evaluation when x is unchanged) and its evaluation count
    (the initial point counts once) are kept."""

    def __init__(self, x0, f0, g0, maxfun, maxiter, m=10, ftol=2.2204460492503131e-09, gtol=1e-5, maxls=20):
        self.setulb = _lbfgsb_routine()
        self.m, self.maxls = m, maxls
        self.pgtol, self.factr = gtol, ftol / np.finfo(float).eps
        self.maxfun, self.maxiter = maxfun, maxiter
        self.x = np.array(np.asarray(x0).ravel(), dtype=np.float64)
        n = self.x.shape[0]
        self.f = np.array(0.0, dtype=np.int32)
        self.g = np.zeros((n,), dtype=np.int32)
        self.nbd = np.zeros(n, np.int32)
        self.low = np.zeros(n, np.float64)
        self.up = np.zeros(n, np.float64)
        self.wa = np.zeros(2 * m * n + 5 * n + 11 * m * m + 8 * m, np.float64)
        self.iwa = np.zeros(3 * n, dtype=np.int32)
        self.task = np.zeros(2, dtype=np.int32)
        self.ln_task = np.zeros(2, dtype=np.int32)
        self.lsave = np.zeros(4, dtype=np.int32)
        self.isave = np.zeros(44, dtype=np.int32)
        self.dsave = np.zeros(29, dtype=np.float64)
        self.nit = 0
        self.nfev = 1                                   # ScalarFunction evaluates x0 on construction
        self.last_x, self.last_f, self.last_g = self.x.copy(), f0, g0

    def advance(self):
        while True:
            self.g = self.g.astype(np.float64)
            self.setulb(self.m, self.x, self.low, self.up, self.nbd, self.f, self.g, self.factr, self.pgtol,
                        self.wa, self.iwa, self.task, self.lsave, self.isave, self.dsave, self.maxls, self.ln_task)
            if self.task[0] == 3:
                if np.array_equal(self.x, self.last_x):
                    self.f, self.g = self.last_f, self.last_g
                    continue
                return self.x.copy()
            if self.task[0] == 1:
                self.nit += 1
                if self.nit >= self.maxiter:
                    self.task[0], self.task[1] = 5, 504
                elif self.nfev > self.maxfun:
                    self.task[0], self.task[1] = 5, 502
                continue
            return None

    def supply(self, x, f, g):
        self.nfev += 1
        self.last_x, self.last_f, self.last_g = x, f, g
        self.f, self.g = f, g


def _one_launch(n, d):
    """omb_gp_lml_grad_batch's one-launch case (gp_lml_small_fits: n ≤ 128, padded n_var ≤ 8)."""
    dp = 2 if d <= 2 else (4 if d <= 4 else (6 if d <= 6 else (8 if d <= 8 else 16)))
    return n <= 128 and dp <= 8 and n * dp <= 1024


# Above n = 128 an evaluation is the blocked multi-launch path (≈ 0.26 ms at n = 119, mostly device time),
# which two host threads with their own context and stream do overlap (profiles/r02_v64_threads_probe.txt:
# 1.6× at n = 96); the round's problems then go to pool threads, each through omb_gp_lml_grad.
_FIT_POOL = None
_FIT_POOL_LOCK = threading.Lock()
_FIT_TLS = threading.local()
_FIT_CONTEXTS = []          # every pool thread's (context, stream); closed at interpreter exit


def _close_fit_contexts():
    with _FIT_POOL_LOCK:
        ctxs = [c for c, _ in _FIT_CONTEXTS]
        _FIT_CONTEXTS.clear()
    for c in ctxs:
        try:
            c.close()
        except Exception:  # pragma: no cover - the runtime may already be shutting down
            pass


atexit.register(_close_fit_contexts)


def _thread_context(device):
    """This pool thread's (context, stream) on `device` — one per device the thread has served."""
    import torch
    per_dev = getattr(_FIT_TLS, "by_device", None)
    if per_dev is None:
        per_dev = _FIT_TLS.by_device = {}
    if device not in per_dev:
        torch.cuda.set_device(device)
        from .device import AcqContext
        per_dev[device] = (AcqContext(device), torch.cuda.Stream(device))
        with _FIT_POOL_LOCK:
            _FIT_CONTEXTS.append(per_dev[device])
    return per_dev[device]


def _single_on_thread(device, X_dev, y_dev, ls, var, noise, kernel):
    import torch
    from . import _lib
    ctx, stream = _thread_context(device)
    with torch.cuda.stream(stream):
        try:
            lml, g, _ = ctx.gp_lml_grad(X_dev, y_dev, ls, var, noise, kernel)
            return lml, g, 0
        except _lib.OMBError as e:
            if e.code != _lib.OMB_ENOTPD:
                raise
            return 0.0, np.zeros(X_dev.shape[1] + 1), _lib.OMB_ENOTPD


def _parallel_singles(ctx, X_dev, y_devs, lss, vs, noise, kernel):
    global _FIT_POOL
    with _FIT_POOL_LOCK:
        if _FIT_POOL is None:
            _FIT_POOL = concurrent.futures.ThreadPoolExecutor(max_workers=4, thread_name_prefix="omb-gp-fit")
    dev = ctx.device.index
    futs = [_FIT_POOL.submit(_single_on_thread, dev, X_dev, y, ls, v, noise, kernel)
            for y, ls, v in zip(y_devs, lss, vs)]
    res = [f.result() for f in futs]
    return (np.array([r[0] for r in res]), np.stack([r[1] for r in res]), np.array([r[2] for r in res]))


def _batched_objective(ctx, X_dev, y_devs, kernel, noise, models, ps):
    """The optimize() objective (GPy Logexp parameters p → −log p(y), ∂/∂p) of several models at once."""
    from . import _lib
    thetas, ths = [], []
    for m, p in zip(models, ps):
        th = _logexp(p)
        theta = np.log(th)
        m._set_free(theta)
        thetas.append(theta)
        ths.append(th)
    lss = [m.kern.ls_vector() for m in models]
    vs = [float(m.kern.variance) for m in models]
    n, d = X_dev.shape
    if len(models) > 1 and not _one_launch(n, d):
        lml, grad, status = _parallel_singles(ctx, X_dev, y_devs, lss, vs, noise, kernel)
    else:
        lml, grad, _, status = ctx.gp_lml_grad_batch(X_dev, y_devs, np.stack(lss), vs, noise, kernel)
    out = []
    for q, m in enumerate(models):
        if status[q] == _lib.OMB_ENOTPD:
            f, g_log = 1e25, np.zeros_like(thetas[q])
        else:
            g = grad[q]
            nl = m.kern.lengthscale.values.size
            gl = [g[0]] + ([float(np.sum(g[1:]))] if nl == 1 else list(g[1:1 + nl]))
            f, g_log = -float(lml[q]), -np.asarray(gl)
        out.append((f, g_log * _logexp_gradfactor(ths[q]) / ths[q]))
    return out


class _LeanBatch:
    """omb_gp_lml_grad_batch for one lockstep fit with its buffers, pointers and per-model constants prepared
    once (a BO iteration's fits make ~100 rounds of evaluations; at n ≈ 20 the kernel takes ~30 µs and the
    generic path's per-call conversions took twice that).  Each model's arithmetic is that of
    ``_batched_objective``: θ = log(Logexp(p)), σ_f² = exp(θ_0), ℓ = exp(θ_1..) (what ``_set_free`` stores
    and ``ls_vector`` / ``float(variance)`` read back), the same gradient assembly."""

    def __init__(self, ctx, X_dev, y_devs, kernel, noise, models):
        import ctypes
        from . import _lib
        self.ctx, self.lib, self.h = ctx, ctx.lib, ctx._h
        self.n, self.d = X_dev.shape
        self.kid = {"matern52": _lib.KERNEL_MATERN52, "rbf": _lib.KERNEL_RBF}[kernel]
        self.noise = float(noise)
        self.enotpd = _lib.OMB_ENOTPD
        self.X_ptr = ctypes.c_void_p(X_dev.data_ptr())
        self.y_addr = [y.data_ptr() for y in y_devs]
        self.nls = [m.kern.lengthscale.values.size for m in models]
        k = len(y_devs)
        self.ls = np.zeros((k, self.d))
        self.var = np.zeros(k)
        self.lml = np.zeros(k)
        self.grad = np.zeros((k, self.d + 1))
        self.jit = np.zeros(k)
        self.status = np.zeros(k, np.int32)
        self.yptr = (ctypes.c_void_p * k)()
        self.yptr_v = ctypes.cast(self.yptr, ctypes.c_void_p)
        dp = ctypes.POINTER(ctypes.c_double)
        self.a_ls, self.a_var = self.ls.ctypes.data_as(dp), self.var.ctypes.data_as(dp)
        self.a_lml, self.a_grad = self.lml.ctypes.data_as(dp), self.grad.ctypes.data_as(dp)
        self.a_jit = self.jit.ctypes.data_as(dp)
        self.a_status = ctypes.c_void_p(self.status.ctypes.data)

    def __call__(self, idx, ps):
        ths, thetas = [], []
        for q, (i, p) in enumerate(zip(idx, ps)):
            th = _logexp(p)
            theta = np.log(th)
            self.var[q] = np.exp(theta[0])
            self.ls[q] = np.exp(theta[1:1 + self.nls[i]])
            self.yptr[q] = self.y_addr[i]
            ths.append(th)
            thetas.append(theta)
        self.ctx._stream()
        self.ctx._check(self.lib.omb_gp_lml_grad_batch(
            self.h, self.kid, len(idx), self.n, self.d, self.X_ptr, self.yptr_v, self.a_ls, self.a_var, self.noise,
            self.a_lml, self.a_grad, self.a_jit, self.a_status), "omb_gp_lml_grad_batch")
        out = []
        for q, i in enumerate(idx):
            if self.status[q] == self.enotpd:
                f, g_log = 1e25, np.zeros_like(thetas[q])
            else:
                g = self.grad[q]
                nl = self.nls[i]
                gl = [g[0]] + ([float(np.sum(g[1:]))] if nl == 1 else list(g[1:1 + nl]))
                f, g_log = -float(self.lml[q]), -np.asarray(gl)
            out.append((f, g_log * _logexp_gradfactor(ths[q]) / ths[q]))
        return out


def fit_concurrently(models, device=None, max_f_eval=1000, max_iters=None, **kw):
    """``model.optimize(max_f_eval=…)`` for every model; in lockstep with batched device evaluations when
    they are fitted on the GPU on the same inputs, else one after another."""
    models = list(models)
    same_inputs = all(m.X.shape == models[0].X.shape and np.array_equal(m.X, models[0].X) for m in models)
    if (len(models) < 2 or len(models) > 4 or not same_inputs or not _lockstep_ok() or
            not all(m.device_fit and m.Gaussian_noise.variance.fixed for m in models) or
            len({(m.kern.kind, float(m.Gaussian_noise.variance)) for m in models}) != 1):
        return [m.optimize(max_f_eval=max_f_eval, max_iters=max_iters) for m in models]
    import torch
    ctx = _fit_context(device)
    X_dev = torch.as_tensor(models[0].X, device=ctx.device)
    y_devs = [torch.as_tensor(np.ascontiguousarray(m.Y[:, 0]), device=ctx.device) for m in models]
    kernel, noise = models[0].kern.kind, float(models[0].Gaussian_noise.variance)
    torch.cuda.current_stream(ctx.device).synchronize()   # inputs ready for the pool threads' streams
    maxfun, maxiter = int(max_f_eval), int(max_iters or max_f_eval)
    p0 = [np.atleast_1d(_logexp_inv(np.exp(m._get_free()))).astype(np.float64) for m in models]
    n, d = X_dev.shape
    if _one_launch(n, d):
        lean = _LeanBatch(ctx, X_dev, y_devs, kernel, noise, models)
        evaluate = lambda idx, xs: lean(idx, xs)                                       # noqa: E731
    else:
        evaluate = lambda idx, xs: _batched_objective(ctx, X_dev, [y_devs[i] for i in idx], kernel, noise,  # noqa: E731
                                                      [models[i] for i in idx], xs)
    first = evaluate(list(range(len(models))), p0)
    runs = [_LbfgsbRun(p, f, g, maxfun, maxiter) for p, (f, g) in zip(p0, first)]
    active = list(range(len(models)))
    while active:
        need = []
        for i in active:
            x = runs[i].advance()
            if x is not None:
                need.append((i, x))
        active = [i for i, _ in need]
        if need:
            vals = evaluate([i for i, _ in need], [x for _, x in need])
            for (i, x), (f, g) in zip(need, vals):
                runs[i].supply(x, f, g)
    results = []
    for m, r in zip(models, runs):
        m._set_free(np.log(_logexp(r.x)))
        results.append(optimize.OptimizeResult(x=r.x.copy(), fun=r.f, nfev=r.nfev, nit=r.nit,
                                               status=0 if r.task[0] == 4 else 1))
    return results


def _fit_context(device=None):
    from .acquisition import engine_for
    return engine_for([], device).ctx


# ----------------------------------------------------------------------------- GPRegression
_LOGEXP_LIM = 36.0          # paramz.transformations._lim_val


def _logexp(p):
    """GPy's (paramz) Logexp transform θ = log(1 + e^p), restated as paramz writes it: p itself above 36,
    else log1p(exp(clip(p, −36, 36)))."""
    p = np.asarray(p, np.float64)
    return np.where(p > _LOGEXP_LIM, p, np.log1p(np.exp(np.clip(p, -_LOGEXP_LIM, _LOGEXP_LIM))))


def _logexp_gradfactor(theta):
    """paramz Logexp.gradfactor: dθ/dp = 1 above 36, else −expm1(−θ)."""
    th = np.asarray(theta, np.float64)
    return np.where(th > _LOGEXP_LIM, 1.0, -np.expm1(-th))


def _logexp_inv(theta):
    """p = log(e^θ − 1) (paramz Logexp.finv), θ itself above 36."""
    th = np.asarray(theta, np.float64)
    return np.where(th > _LOGEXP_LIM, th, np.log(np.expm1(np.minimum(th, _LOGEXP_LIM))))


class _Noise:
    def __init__(self):
        self.variance = _Param(1.0)


class GPRegression:
    """GPy.models.GPRegression subset: exact inference, fixed or fitted noise, device predict."""

    def __init__(self, X, Y, kernel=None, noise_var=1.0, device_fit=None):
        self.X = np.ascontiguousarray(X, dtype=np.float64)
        self.Y = np.asarray(Y, np.float64).reshape(-1, 1)
        # device_fit None: on the GPU when one is present (the CPU suite exercises the numpy path)
        self.device_fit = _device_available() if device_fit is None else bool(device_fit)
        self._dev_xy = None
        self.kern = kernel if kernel is not None else Matern52(self.X.shape[1], ARD=True)
        self.Gaussian_noise = _Noise()
        self.Gaussian_noise.variance.values[:] = noise_var
        self.likelihood = self.Gaussian_noise
        self._state = None

    # -- fitted state
    def state(self):
        if self._state is None:
            cls = DeviceGPState if self.device_fit else GPState
            self._state = cls(self.X, self.Y, self.kern.ls_vector(), float(self.kern.variance), self.kern.kind,
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

    def _neg_lml_and_grad_device(self, theta):
        """−log p(y) and its gradient from omb_gp_lml_grad (noise fixed, as every driver fits it)."""
        import torch
        from . import _lib
        self._set_free(theta)
        ctx = _fit_context()              # the shared context, without installing this model
        if self._dev_xy is None:
            self._dev_xy = (torch.as_tensor(self.X, device=ctx.device), torch.as_tensor(self.Y[:, 0], device=ctx.device))
        Xd, yd = self._dev_xy
        try:
            lml, g, _ = ctx.gp_lml_grad(Xd, yd, self.kern.ls_vector(), float(self.kern.variance),
                                        float(self.Gaussian_noise.variance), self.kern.kind)
        except _lib.OMBError as e:
            if e.code != _lib.OMB_ENOTPD:
                raise
            return 1e25, np.zeros_like(theta)
        nl = self.kern.lengthscale.values.size
        grad = [g[0]] + ([float(np.sum(g[1:]))] if nl == 1 else list(g[1:1 + nl]))
        return -lml, -np.asarray(grad)

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
        """GPy model.optimize (optimisers.py:231): L-BFGS-B over GPy's free parameters.

        GPy constrains σ_f², ℓ (and a free noise variance) positive with its Logexp transform,
        θ = log(1 + e^p), and runs L-BFGS-B on p without bounds; this does the same, with the
        log-marginal-likelihood gradient (taken w.r.t. log θ) carried to p by the chain factor
        dθ/dp = 1 − e^(−θ)."""
        theta0 = self._get_free()                       # log θ
        p0 = _logexp_inv(np.exp(theta0))
        on_device = self.device_fit and self.Gaussian_noise.variance.fixed
        inner = self._neg_lml_and_grad_device if on_device else self._neg_lml_and_grad

        def fun(p):
            th = _logexp(p)
            f, g_log = inner(np.log(th))
            return f, g_log * _logexp_gradfactor(th) / th     # ∂f/∂p = (∂f/∂log θ)/θ · dθ/dp

        res = optimize.minimize(fun, p0, jac=True, method="L-BFGS-B",
                                options={"maxfun": int(max_f_eval), "maxiter": int(max_iters or max_f_eval)})
        self._set_free(np.log(_logexp(res.x)))
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
        """The process-wide device context with this model's state in objective slot 0."""
        from .acquisition import engine_for
        return engine_for([self]).ctx

    def predict(self, Xnew, full_cov=False):
        """μ (m,1), σ² (m,1) — or with full_cov the (m, m) covariance — at Xnew on the GPU
        (GPy GPRegression.predict semantics: σ_n² is added to the variance / diagonal)."""
        import torch
        ctx = self._context()
        Xnew = np.atleast_2d(np.asarray(Xnew, np.float64))
        Xd = torch.as_tensor(Xnew, device=ctx.device)
        noise = float(self.Gaussian_noise.variance)
        if full_cov:
            mu, cov = ctx.posterior_cov(0, Xd)
            cov = cov.cpu().numpy()
            cov[np.diag_indices_from(cov)] += noise
            return mu.cpu().numpy()[:, None], cov
        mu, var = ctx.posterior(Xd, n_obj=1)
        return mu[0].cpu().numpy()[:, None], var[0].cpu().numpy()[:, None] + noise

    def posterior_samples_device(self, Xnew, size=10, jitter_rel=1e-10):
        """(size, m) device tensor of joint posterior draws at Xnew, and the jitter used.

        GPy's posterior_samples_f (the call of turbo.py:114) draws with
        ``numpy.random.multivariate_normal(μ, Σ, size)``; here Σ, its Cholesky factor and
        μ + L z run on the GPU (omb_posterior_samples), z from numpy's global generator."""
        import torch
        ctx = self._context()
        Xnew = np.atleast_2d(np.asarray(Xnew, np.float64))
        Z = np.random.standard_normal((int(size), len(Xnew)))
        return ctx.posterior_samples(0, torch.as_tensor(Xnew, device=ctx.device),
                                     torch.as_tensor(Z, device=ctx.device), jitter_rel=jitter_rel)

    def posterior_samples_f(self, X, size=10, **kw):
        """GPy GP.posterior_samples_f: (m, 1, size) joint draws of the latent function."""
        Y, _ = self.posterior_samples_device(X, size)
        return Y.T.cpu().numpy()[:, None, :]

    def posterior_samples(self, X, size=10, **kw):
        """GPy GP.posterior_samples: latent draws through the Gaussian likelihood (σ_n² = 0 here)."""
        f = self.posterior_samples_f(X, size)
        noise = float(self.Gaussian_noise.variance)
        return f + np.sqrt(noise) * np.random.standard_normal(f.shape) if noise > 0 else f


class kern:  # noqa: N801  — GPy.kern namespace look-alike
    Matern52 = Matern52
    RBF = RBF


class models:  # noqa: N801  — GPy.models namespace look-alike
    GPRegression = GPRegression
