"""Device context: torch tensors as device-memory holders around the HIP C-ABI.

``AcqContext`` owns one ``omb_ctx`` (one per GPU) and runs every call on torch's current
stream, so torch events time the kernels exactly.  All arrays are fp64 CUDA (HIP) tensors;
the context never copies candidates to the host.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _dev_f64(x, device):
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=torch.float64)
    else:
        t = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=device)
    return t.contiguous()


class AcqContext:
    """One HIP context on ``device`` holding the fitted GPs of up to 8 objectives."""

    def __init__(self, device=0):
        if not torch.cuda.is_available():
            raise RuntimeError("AcqContext needs a ROCm GPU (torch.cuda.is_available() is False); "
                               "the acquisition hot path has no CPU fallback")
        self.lib = _lib.load()
        self.device = torch.device("cuda", device if isinstance(device, int) else torch.device(device).index or 0)
        h = ctypes.c_void_p()
        rc = self.lib.omb_create(self.device.index, ctypes.byref(h))
        if rc != 0:
            raise _lib.OMBError(rc, f"omb_create(device={self.device.index}) failed")
        self._h = h
        self._gp_keep = {}     # device tensors referenced by the packed GP state
        self.gp_info = {}

    # ------------------------------------------------------------------ plumbing
    def _check(self, rc, what):
        if rc != 0:
            msg = self.lib.omb_last_error(self._h)
            raise _lib.OMBError(rc, f"{what}: {msg.decode() if msg else ''}")

    def _stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != getattr(self, "_cur_stream", None):     # one C call per stream change, not per call
            self._check(self.lib.omb_set_stream(self._h, ctypes.c_void_p(s)), "omb_set_stream")
            self._cur_stream = s

    def close(self):
        if getattr(self, "_h", None):
            self.lib.omb_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        self._check(self.lib.omb_synchronize(self._h), "omb_synchronize")

    def debug_set(self, what, value):
        """omb_debug_set: ("spin_limit", polls) bounds the posterior's LDS-counter waits; ("cov_table", 0/1)
        builds K(X, X) / K(X*, X*) with the posterior's table-driven Matern transform; ("fused_chain", 0/1/2) runs
        EHVI-2D and the arg-max as separate launches / as one ticketed launch / as EHVI with per-workgroup pairs
        and the arg-max's second pass; ("argmax_passes", 1/2) runs the arg-max as one
        launch / as two; ("chol_mode", 0/1/2 [+ 4]) factors auto / by per-step launches / in one persistent launch
        [with release-acquire hand-offs];
        ("timing_stride", s) records the timing events on every s-th chain only; ("select_seq", 0/1) picks the
        Thompson selection's parallel rounds (default) / its sequential walk for B <= 64."""
        code = {"spin_limit": _lib.DEBUG_SPIN_LIMIT, "cov_table": _lib.DEBUG_COV_TABLE,
                "fused_chain": _lib.DEBUG_FUSED_CHAIN, "argmax_passes": _lib.DEBUG_ARGMAX_PASSES,
                "chol_mode": _lib.DEBUG_CHOL_MODE, "timing_stride": _lib.DEBUG_TIMING_STRIDE,
                "cov_fused": _lib.DEBUG_COV_FUSED,
                "select_seq": _lib.DEBUG_SELECT_SEQ, "syrk_glds": _lib.DEBUG_SYRK_GLDS}[what]
        self._check(self.lib.omb_debug_set(self._h, code, int(value)), "omb_debug_set")

    # ------------------------------------------------------------------ GP state
    def set_gp(self, obj, X, lengthscale, variance, alpha, Linv, kernel="matern52"):
        """Upload one fitted GP (see optimobo_amd.gp.GPState) for objective ``obj``."""
        X = _dev_f64(X, self.device)
        alpha = _dev_f64(np.asarray(alpha).reshape(-1) if not isinstance(alpha, torch.Tensor) else alpha.reshape(-1),
                         self.device)
        Linv = _dev_f64(Linv, self.device)
        n, d = X.shape
        if Linv.shape != (n, n) or alpha.shape[0] != n:
            raise ValueError(f"set_gp: shapes X{tuple(X.shape)} alpha{tuple(alpha.shape)} Linv{tuple(Linv.shape)}")
        ls = np.broadcast_to(np.asarray(lengthscale, np.float64), (d,))
        kid = {"matern52": _lib.KERNEL_MATERN52, "rbf": _lib.KERNEL_RBF}[kernel]
        self._stream()
        self._check(self.lib.omb_set_gp(self._h, obj, kid, n, d, _ptr(X), _lib.darr(ls), float(variance),
                                        _ptr(alpha), _ptr(Linv)), "omb_set_gp")
        self._gp_keep[obj] = (X, alpha, Linv)
        self.gp_info[obj] = dict(n=n, d=d, variance=float(variance), kernel=kernel)

    def set_gp_state(self, obj, state):
        if hasattr(state, "upload"):          # DeviceGPState: factorised on the device
            state.upload(self, obj)
            return
        self.set_gp(obj, state.X, state.lengthscale, state.variance, state.alpha, state.Linv, state.kernel)

    # ------------------------------------------------------------------ posterior
    def _check_width(self, Xc, obj=0):
        """The C-ABI takes no candidate width: the kernels read Xc (N, d) with the installed GP's d."""
        info = self.gp_info.get(obj)
        if Xc.dim() != 2:
            raise ValueError(f"candidates must be (N, d), got shape {tuple(Xc.shape)}")
        if info is not None and Xc.shape[1] != info["d"]:
            raise ValueError(f"candidates have {Xc.shape[1]} columns but objective {obj}'s GP has n_var={info['d']}")

    def kernel_block(self, obj, Xc, out=None):
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc, obj)
        n = self.gp_info[obj]["n"]
        N = Xc.shape[0]
        K = out if out is not None else torch.empty((n, N), dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_kernel_block(self._h, obj, _ptr(Xc), N, _ptr(K)), "omb_kernel_block")
        return K

    def posterior(self, Xc, n_obj=None, out=None):
        """μ, σ² (n_obj, N) of objectives 0..n_obj-1 at candidates Xc (N, d)."""
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc)
        n_obj = n_obj if n_obj is not None else len(self.gp_info)
        N = Xc.shape[0]
        if out is None:
            mu = torch.empty((n_obj, N), dtype=torch.float64, device=self.device)
            var = torch.empty_like(mu)
        else:
            mu, var = out
        self._stream()
        self._check(self.lib.omb_posterior(self._h, n_obj, _ptr(Xc), N, _ptr(mu), _ptr(var)), "omb_posterior")
        return mu, var

    # ------------------------------------------------------------------ acquisitions
    def ehvi2d(self, mu, var, pf_sorted, r, s00, s01, mode="reference", out=None):
        N = mu.shape[1]
        pf = _dev_f64(pf_sorted, self.device)
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        m = {"reference": _lib.EHVI_REFERENCE, "textbook": _lib.EHVI_TEXTBOOK, "sigma": _lib.EHVI_SIGMA}[mode]
        self._stream()
        self._check(self.lib.omb_ehvi2d(self._h, _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(pf), pf.shape[0],
                                        _lib.darr(r), float(s00), float(s01), m, _ptr(out)), "omb_ehvi2d")
        return out

    def ehvi_mc(self, mu, var, cache, r, hv_pf, out=None, raised=None):
        """EHVI_3D's Monte-Carlo form over k = cache.shape[1] objectives (rows 0..k-1 of mu/var):
        (values (N,), raised (N,) int32); NaN and raised = 1 where pygmo would raise."""
        N = mu.shape[1]
        cache = _dev_f64(cache, self.device)
        if cache.dim() != 2 or not 2 <= cache.shape[1] <= mu.shape[0] or len(r) != cache.shape[1]:
            raise ValueError(f"ehvi_mc: cache {tuple(cache.shape)}, r of {len(r)}, mu {tuple(mu.shape)} disagree on k")
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        raised = raised if raised is not None else torch.empty(N, dtype=torch.int32, device=self.device)
        self._stream()
        self._check(self.lib.omb_ehvi_mc(self._h, cache.shape[1], _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(cache),
                                         cache.shape[0], _lib.darr(r), float(hv_pf), _ptr(out), _ptr(raised)),
                    "omb_ehvi_mc")
        return out, raised

    def ehvi3d_mc(self, mu, var, cache, r, hv_pf, out=None, raised=None):
        N = mu.shape[1]
        cache = _dev_f64(cache, self.device)
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        raised = raised if raised is not None else torch.empty(N, dtype=torch.int32, device=self.device)
        self._stream()
        self._check(self.lib.omb_ehvi3d_mc(self._h, _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(cache), cache.shape[0],
                                           _lib.darr(r), float(hv_pf), _ptr(out), _ptr(raised)), "omb_ehvi3d_mc")
        return out, raised

    def ehvi_boxes(self, mu, var, coords, boxes, out=None):
        """Exact EHVI over a box decomposition (optimobo_amd.pareto.box_decomposition)."""
        k, N = mu.shape
        coords = _dev_f64(coords, self.device)
        if not isinstance(boxes, torch.Tensor):
            # uint16 indices < 32768 travel as int16 (torch has no uint16 on every build)
            b = np.ascontiguousarray(boxes, dtype=np.uint16)
            boxes = torch.as_tensor(b.view(np.int16), device=self.device)
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_ehvi_boxes(self._h, k, _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(coords),
                                            coords.shape[1], _ptr(boxes), boxes.shape[0], _ptr(out)),
                    "omb_ehvi_boxes")
        return out

    def hvpoi(self, mu, var, cells, out=None):
        N = mu.shape[1]
        cells = _dev_f64(cells, self.device)
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_hvpoi(self._h, _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(cells), cells.shape[0],
                                       _ptr(out)), "omb_hvpoi")
        return out

    def expdec(self, mu, var, cache, scal_id, params, weights, ideal, max_point, agg_min, out=None):
        k, N = mu.shape
        cache = _dev_f64(cache, self.device)
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_expdec(self._h, k, _ptr(mu), _ptr(var), mu.stride(0), N, _ptr(cache), cache.shape[0],
                                        int(scal_id), _lib.darr(params), _lib.darr(weights), _lib.darr(ideal),
                                        _lib.darr(max_point), float(agg_min), _ptr(out)), "omb_expdec")
        return out

    def ei(self, mu, var, best, var_eps=0.0, out=None):
        mu = mu.reshape(-1)
        var = var.reshape(-1)
        N = mu.shape[0]
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_ei(self._h, _ptr(mu), _ptr(var), N, float(best), float(var_eps), _ptr(out)), "omb_ei")
        return out

    def ei_ext(self, kind, mu, var, best, var_eps=0.0, pof_eps=0.0, out=None):
        """EI family over rows 0..k-1 of (mu, var): kind "plain" | "pareto" (KEEP) | "constrained" (cParEGO)."""
        k, N = mu.shape
        kid = {"plain": _lib.EI_PLAIN, "pareto": _lib.EI_PARETO, "constrained": _lib.EI_CONSTRAINED}[kind]
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_ei_ext(self._h, kid, k, _ptr(mu), _ptr(var), mu.stride(0), N, float(best),
                                        float(var_eps), float(pof_eps), _ptr(out)), "omb_ei_ext")
        return out

    def argmax_dev(self, vals, offset=0, out=None):
        out = out if out is not None else torch.empty(2, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_argmax_dev(self._h, _ptr(vals), vals.numel(), int(offset), _ptr(out)), "omb_argmax_dev")
        return out

    def argmax(self, vals, offset=0):
        v = ctypes.c_double()
        i = ctypes.c_int64()
        self._stream()
        self._check(self.lib.omb_argmax(self._h, _ptr(vals), vals.numel(), int(offset), ctypes.byref(v),
                                        ctypes.byref(i)), "omb_argmax")
        return v.value, i.value

    # ------------------------------------------------------------------ fused chain (plans)
    def _plan(self, fn, *args):
        self._stream()
        self._check(getattr(self.lib, fn)(self._h, *args), fn)

    def plan_ehvi2d(self, pf_sorted, r, s00, s01, mode="reference"):
        pf = np.ascontiguousarray(pf_sorted, dtype=np.float64).reshape(-1, 2)
        m = {"reference": _lib.EHVI_REFERENCE, "textbook": _lib.EHVI_TEXTBOOK, "sigma": _lib.EHVI_SIGMA}[mode]
        self._plan("omb_plan_ehvi2d", _lib.host_ptr(pf), pf.shape[0], _lib.darr(r), float(s00), float(s01), m)

    def plan_ehvi_mc(self, cache, r, hv_pf):
        """EHVI_3D's Monte-Carlo form for k = cache.shape[1] objectives (cache (M, k), r (k,))."""
        c = np.ascontiguousarray(cache, dtype=np.float64)
        if c.ndim != 2 or len(r) != c.shape[1]:
            raise ValueError(f"plan_ehvi_mc: cache {c.shape} and r of {len(r)} disagree on k")
        self._plan("omb_plan_ehvi_mc", c.shape[1], _lib.host_ptr(c), c.shape[0], _lib.darr(r), float(hv_pf))

    def plan_ehvi3d_mc(self, cache, r, hv_pf):
        c = np.ascontiguousarray(cache, dtype=np.float64).reshape(-1, 3)
        self._plan("omb_plan_ehvi3d_mc", _lib.host_ptr(c), c.shape[0], _lib.darr(r), float(hv_pf))

    def plan_ehvi_boxes(self, coords, boxes):
        c = np.ascontiguousarray(coords, dtype=np.float64)
        b = np.ascontiguousarray(boxes, dtype=np.uint16)
        self._plan("omb_plan_ehvi_boxes", c.shape[0], _lib.host_ptr(c), c.shape[1], _lib.host_ptr(b), b.shape[0])

    def plan_hvpoi(self, cells):
        c = np.ascontiguousarray(cells, dtype=np.float64).reshape(-1, 2, 2)
        self._plan("omb_plan_hvpoi", _lib.host_ptr(c), c.shape[0])

    def plan_expdec(self, cache, scal_id, params, weights, ideal, max_point, agg_min):
        c = np.ascontiguousarray(cache, dtype=np.float64)
        self._plan("omb_plan_expdec", c.shape[1], _lib.host_ptr(c), c.shape[0], int(scal_id), _lib.darr(params),
                   _lib.darr(weights), _lib.darr(ideal), _lib.darr(max_point), float(agg_min))

    def plan_ei(self, best, var_eps=0.0):
        self._plan("omb_plan_ei", float(best), float(var_eps))

    def plan_ei_ext(self, kind, k, best, var_eps=0.0, pof_eps=0.0):
        kid = {"plain": _lib.EI_PLAIN, "pareto": _lib.EI_PARETO, "constrained": _lib.EI_CONSTRAINED}[kind]
        self._plan("omb_plan_ei_ext", kid, int(k), float(best), float(var_eps), float(pof_eps))

    def set_sobol(self, d, lo, hi, seed=None, scramble=True, state=None):
        """Device Sobol' engine = scipy qmc.Sobol(d, scramble=scramble, seed=seed) over [lo, hi]."""
        from .sobol import engine_state
        sv, shift, bits = state if state is not None else engine_state(d, seed, scramble)
        lo = np.broadcast_to(np.asarray(lo, np.float64), (d,))
        hi = np.broadcast_to(np.asarray(hi, np.float64), (d,))
        self._stream()
        self._check(self.lib.omb_set_sobol(self._h, d, bits, _lib.host_ptr(sv), _lib.host_ptr(shift), _lib.darr(lo),
                                           _lib.darr(hi)), "omb_set_sobol")
        self.sobol_dim = d

    def sobol(self, start, N, out=None):
        out = out if out is not None else torch.empty((N, self.sobol_dim), dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_sobol(self._h, int(start), int(N), _ptr(out)), "omb_sobol")
        return out

    def eval(self, Xc, out=None):
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc)
        N = Xc.shape[0]
        out = out if out is not None else torch.empty(N, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_eval(self._h, _ptr(Xc), N, _ptr(out)), "omb_eval")
        return out

    def eval_argmax(self, Xc, offset=0, out=None):
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc)
        out = out if out is not None else torch.empty(2, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_eval_argmax(self._h, _ptr(Xc), Xc.shape[0], int(offset), _ptr(out)),
                    "omb_eval_argmax")
        return out

    def eval_argmax_sobol(self, start, N, out=None):
        out = out if out is not None else torch.empty(2, dtype=torch.float64, device=self.device)
        self._stream()
        self._check(self.lib.omb_eval_argmax_sobol(self._h, int(start), int(N), _ptr(out)), "omb_eval_argmax_sobol")
        return out

    # ------------------------------------------------------------------ GP fit on the device
    def gp_lml_grad(self, X, y, lengthscale, variance, noise=0.0, kernel="matern52"):
        """GPy's exact-inference log marginal likelihood at (σ_f², ℓ) with the noise fixed, its gradient
        w.r.t. (log σ_f², log ℓ_1..d) and jitchol's extra jitter: (lml, grad (d+1,), jitter)."""
        X = _dev_f64(X, self.device)
        y = _dev_f64(y, self.device).reshape(-1)
        n, d = X.shape
        if y.shape[0] != n:
            raise ValueError(f"gp_lml_grad: y has {y.shape[0]} values for {n} inputs")
        ls = np.broadcast_to(np.asarray(lengthscale, np.float64), (d,))
        kid = {"matern52": _lib.KERNEL_MATERN52, "rbf": _lib.KERNEL_RBF}[kernel]
        lml, jit = ctypes.c_double(), ctypes.c_double()
        grad = (ctypes.c_double * (d + 1))()
        self._stream()
        self._check(self.lib.omb_gp_lml_grad(self._h, kid, n, d, _ptr(X), _ptr(y), _lib.darr(ls), float(variance),
                                             float(noise), ctypes.byref(lml), grad, ctypes.byref(jit)),
                    "omb_gp_lml_grad")
        return lml.value, np.array(grad[:]), jit.value

    def gp_lml_grad_batch(self, X, ys, lengthscales, variances, noise=0.0, kernel="matern52"):
        """omb_gp_lml_grad_batch: k ≤ 4 GPs on the same inputs in one call — (lml (k,), grad (k, d+1),
        jitter (k,), status (k,)); status[p] is 0 or OMB_ENOTPD for problem p."""
        X = _dev_f64(X, self.device)
        ys = [_dev_f64(y, self.device).reshape(-1) for y in ys]
        n, d = X.shape
        k = len(ys)
        if any(y.shape[0] != n for y in ys):
            raise ValueError("gp_lml_grad_batch: every y needs one value per input row")
        ls = np.ascontiguousarray(np.broadcast_to(np.asarray(lengthscales, np.float64), (k, d)))
        var = np.ascontiguousarray(np.asarray(variances, np.float64).reshape(k))
        kid = {"matern52": _lib.KERNEL_MATERN52, "rbf": _lib.KERNEL_RBF}[kernel]
        yptr = (ctypes.c_void_p * k)(*[y.data_ptr() for y in ys])
        lml = np.zeros(k)
        grad = np.zeros((k, d + 1))
        jit = np.zeros(k)
        status = np.zeros(k, np.int32)
        dp = ctypes.POINTER(ctypes.c_double)
        self._stream()
        self._check(self.lib.omb_gp_lml_grad_batch(
            self._h, kid, k, n, d, _ptr(X), ctypes.cast(yptr, ctypes.c_void_p), ls.ctypes.data_as(dp),
            var.ctypes.data_as(dp), float(noise), lml.ctypes.data_as(dp), grad.ctypes.data_as(dp),
            jit.ctypes.data_as(dp), ctypes.c_void_p(status.ctypes.data)), "omb_gp_lml_grad_batch")
        return lml, grad, jit, status

    def gp_fit_state(self, obj, X, y, lengthscale, variance, noise=0.0, kernel="matern52"):
        """Factorise on the device and install objective ``obj`` (omb_gp_fit_state); returns the jitter."""
        X = _dev_f64(X, self.device)
        y = _dev_f64(y, self.device).reshape(-1)
        n, d = X.shape
        ls = np.broadcast_to(np.asarray(lengthscale, np.float64), (d,))
        kid = {"matern52": _lib.KERNEL_MATERN52, "rbf": _lib.KERNEL_RBF}[kernel]
        jit = ctypes.c_double()
        self._stream()
        self._check(self.lib.omb_gp_fit_state(self._h, int(obj), kid, n, d, _ptr(X), _ptr(y), _lib.darr(ls),
                                              float(variance), float(noise), ctypes.byref(jit)), "omb_gp_fit_state")
        self._gp_keep[obj] = (X, y)
        self.gp_info[obj] = dict(n=n, d=d, variance=float(variance), kernel=kernel)
        return jit.value

    # ------------------------------------------------------------------ Thompson sampling (TuRBO)
    def posterior_cov(self, obj, Xc, out=None):
        """μ (N,), Σ (N, N): GPy predict(Xc, full_cov=True) of objective ``obj`` (σ_n² = 0)."""
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc, obj)
        N = Xc.shape[0]
        mu, cov = out if out is not None else (torch.empty(N, dtype=torch.float64, device=self.device),
                                               torch.empty((N, N), dtype=torch.float64, device=self.device))
        self._stream()
        self._check(self.lib.omb_posterior_cov(self._h, int(obj), _ptr(Xc), N, _ptr(mu), _ptr(cov)),
                    "omb_posterior_cov")
        return mu, cov

    def cholesky(self, A, jitter=0.0):
        """In place: lower triangle of A (N, N) ← chol(A + jitter·I); returns LAPACK's info (0 = ok)."""
        if A.dtype != torch.float64 or A.dim() != 2 or A.shape[0] != A.shape[1] or A.stride(1) != 1:
            raise ValueError("cholesky: A must be a square fp64 device matrix with unit column stride")
        info = ctypes.c_int()
        self._stream()
        self._check(self.lib.omb_cholesky(self._h, _ptr(A), A.shape[0], A.stride(0), float(jitter), ctypes.byref(info)),
                    "omb_cholesky")
        return info.value

    def posterior_samples(self, obj, Xc, Zt, jitter_rel=1e-10, max_tries=8, out=None):
        """Y (B, N): B joint posterior samples μ + chol(Σ + jI) z_b at Xc, z_b = row b of Zt (B, N).

        Returns (Y, j) with j the absolute jitter that made Σ + jI factorisable."""
        Xc = _dev_f64(Xc, self.device)
        self._check_width(Xc, obj)
        Zt = _dev_f64(Zt, self.device)
        N = Xc.shape[0]
        B = Zt.shape[0]
        if Zt.dim() != 2 or Zt.shape[1] != N:
            raise ValueError(f"Zt must be (B, {N}), got {tuple(Zt.shape)}")
        Y = out if out is not None else torch.empty((B, N), dtype=torch.float64, device=self.device)
        used = ctypes.c_double()
        self._stream()
        self._check(self.lib.omb_posterior_samples(self._h, int(obj), _ptr(Xc), N, _ptr(Zt), B, float(jitter_rel),
                                                   int(max_tries), _ptr(Y), ctypes.byref(used)),
                    "omb_posterior_samples")
        return Y, used.value

    def thompson_select(self, Y, out=None):
        """TuRBO's greedy per-sample arg-min over Y (B, N) → indices (B,) int64 (device)."""
        Y = _dev_f64(Y, self.device)
        B, N = Y.shape
        idx = out if out is not None else torch.empty(B, dtype=torch.int64, device=self.device)
        self._stream()
        self._check(self.lib.omb_thompson_select(self._h, _ptr(Y), B, N, _ptr(idx)), "omb_thompson_select")
        return idx

    def ea_search(self, pop, tape, best, lower, upper, mode=0, var_eps=1e-6):
        """ParEGO (mode 0: EI of objective 0) / KEEP (mode 1: μ of objective 1 · EI of objective 0)
        evolutionary acquisition search (omb_ea_search) from the temporary population `pop` (P, d) and
        a tape of the reference's random draws (optimobo_amd.ea.ea_tape) → (best x (d,), best fitness),
        host numpy.  Synchronises."""
        pop = np.ascontiguousarray(pop, np.float64)
        P, d = pop.shape
        if tape.beta.shape[1:] != (d,) or tape.mut.shape[1:] != (d,) or tape.sel.shape[1:] != (4,):
            raise ValueError("tape does not match the population width")
        sel = tape.sel
        if len(sel) and (sel[:, :2].min() < 1 or sel[:, :2].max() > P - 1 or sel[:, 2:].min() < 1
                         or sel[:, 2:].max() > P - 2):
            raise ValueError("tournament samples outside range(1, P) / range(1, P - 1)")
        dv = self.device
        t_pop = torch.as_tensor(pop, device=dv)
        self._check_width(t_pop)
        if mode == _lib.EA_PARETO_EI:
            self._check_width(t_pop, 1)
        t_sel = torch.as_tensor(np.ascontiguousarray(sel, np.int32), device=dv)
        t_cross = torch.as_tensor(np.ascontiguousarray(tape.cross, np.int8), device=dv)
        t_beta = torch.as_tensor(np.ascontiguousarray(tape.beta, np.float64), device=dv)
        t_mut = torch.as_tensor(np.ascontiguousarray(tape.mut, np.int8), device=dv)
        t_lo = torch.as_tensor(np.ascontiguousarray(lower, np.float64).reshape(d), device=dv)
        t_hi = torch.as_tensor(np.ascontiguousarray(upper, np.float64).reshape(d), device=dv)
        out = torch.empty(d + 1, dtype=torch.float64, device=dv)
        self._stream()
        self._check(self.lib.omb_ea_search(self._h, int(mode), float(best), float(var_eps), _ptr(t_pop), P,
                                           int(tape.iters), _ptr(t_sel), _ptr(t_cross), _ptr(t_beta), _ptr(t_mut),
                                           _ptr(t_lo), _ptr(t_hi), _ptr(out)), "omb_ea_search")
        o = out.cpu().numpy()
        return o[:d].copy(), float(o[d])

    def timing(self, level=2):
        """0 off, 1 posterior only, 2 every stage of the fused chain (see omb_timing)."""
        self._stream()
        self._check(self.lib.omb_timing(self._h, int(level)), "omb_timing")

    def timing_read(self):
        """{stage: summed ms} over the fused chains since the last read, and their count."""
        ms = (ctypes.c_double * 4)()
        n = ctypes.c_int64()
        self._stream()
        self._check(self.lib.omb_timing_read(self._h, ms, ctypes.byref(n)), "omb_timing_read")
        return dict(zip(("sobol", "posterior", "acquisition", "argmax"), list(ms))), n.value
