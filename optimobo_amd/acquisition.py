"""Batched acquisition engine: the device replacement for the reference's maximiser loop.

The reference maximises every acquisition with ``scipy.optimize.differential_evolution``,
calling ``acq(x)`` one candidate at a time (optimisers.py:87,118,366; emo.py:240).  Here one
BO iteration uploads the fitted surrogates once, scores a large quasi-random candidate batch
on the GPU (Sobol generation → posterior → acquisition) and reduces it with the device arg-max.  With
torch.distributed initialised, every rank scores its own contiguous shard of the Sobol
sequence and the ranks exchange one {value, index} pair (optimobo_amd.parallel); the winning
point is regenerated from its Sobol index on every rank, so no coordinates are broadcast.
"""
import numpy as np
import torch

from . import pareto
from .device import AcqContext
from .gp import GPState
from .parallel import global_argmax, shard_range, world


def _state_of(model):
    if isinstance(model, GPState):
        return model
    if hasattr(model, "state"):
        return model.state()
    raise TypeError(f"unsupported surrogate {type(model).__name__}: expected optimobo_amd.gp.GPRegression/GPState")


class AcquisitionEngine:
    """Owns one AcqContext and the fitted GP state currently resident on the device."""

    def __init__(self, device=None):
        if device is None:
            device = torch.cuda.current_device() if torch.cuda.is_available() else 0
        self.ctx = AcqContext(device)
        self.device = self.ctx.device
        self._resident = {}
        self.n_obj = 0

    # ------------------------------------------------------------------ model state
    def load_models(self, models):
        for o, m in enumerate(models):
            st = _state_of(m)
            if self._resident.get(o) is not st:
                self.ctx.set_gp_state(o, st)
                self._resident[o] = st
        self.n_obj = len(models)
        return self

    def _dev(self, x):
        return torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=self.device)

    def posterior(self, Xc):
        Xc = Xc if isinstance(Xc, torch.Tensor) else self._dev(np.atleast_2d(Xc))
        return self.ctx.posterior(Xc, self.n_obj)

    # ------------------------------------------------------------------ acquisitions on a batch
    def ehvi(self, Xc, max_point, PF, cache, mode="reference"):
        """util_functions.EHVI (2 objectives) on every row of Xc."""
        mu, var = self.posterior(Xc)
        s00, s01 = pareto.cache_stats(np.asarray(cache, np.float64))
        pf = pareto.stripes_2d(PF)
        return self.ctx.ehvi2d(mu, var, pf, np.asarray(max_point, np.float64), s00, s01, mode=mode)

    def ehvi_2d_aux(self, PF, r, mu, sigma):
        """EHVI_2D_aux(PF, r, μ, σ) with σ given directly (util_functions.py:81), batched: (2, N)."""
        mu = self._dev(np.asarray(mu, np.float64).reshape(2, -1))
        sig = self._dev(np.asarray(sigma, np.float64).reshape(2, -1))
        return self.ctx.ehvi2d(mu, sig, pareto.stripes_2d(PF), np.asarray(r, np.float64), 1.0, 1.0, mode="sigma")

    def ehvi_exact(self, Xc, max_point, PF):
        """Exact EHVI (2 or 3 objectives) over the box decomposition — "textbook" mode."""
        mu, var = self.posterior(Xc)
        coords, _, boxes = pareto.box_decomposition(PF, max_point)
        return self.ctx.ehvi_boxes(mu, var, coords, boxes)

    def ehvi3d(self, Xc, max_point, PF, cache):
        """util_functions.EHVI_3D (Monte-Carlo form) on every row of Xc, for k = n_obj ≥ 3 objectives (the
        reference calls it for every n_obj != 2): (values (N,), raised (N,) int32)."""
        mu, var = self.posterior(Xc)
        hv = pareto.hypervolume(PF, max_point)
        return self.ctx.ehvi_mc(mu, var, np.asarray(cache, np.float64), np.asarray(max_point, np.float64), hv)

    def expected_decomposition(self, Xc, weights, agg_func, agg_min, cache):
        mu, var = self.posterior(Xc)
        sid, params = agg_func.device_spec()
        return self.ctx.expdec(mu, var, np.asarray(cache, np.float64), sid, params, np.asarray(weights, np.float64),
                               np.asarray(agg_func.ideal_point, np.float64), np.asarray(agg_func.max_point, np.float64),
                               float(agg_min))

    def hvpoi(self, Xc, cells):
        mu, var = self.posterior(Xc)
        return self.ctx.hvpoi(mu, var, np.ascontiguousarray(cells, dtype=np.float64))

    def ei(self, Xc, best, var_eps=0.0):
        mu, var = self.posterior(Xc)
        return self.ctx.ei(mu[0], var[0], float(best), float(var_eps))

    def pareto_ei(self, Xc, best, var_eps=1e-6):
        """KEEP's μ_pareto · EI (keep.py:142-151); models = [scalarised, pareto membership]."""
        mu, var = self.posterior(Xc)
        return self.ctx.ei_ext("pareto", mu, var, float(best), float(var_eps))

    def constrained_ei(self, Xc, best, var_eps=0.0, pof_eps=1e-5):
        """ParEGO_C2's EI · Π PoF (cparego.py:486-496); models = [aggregate, constraint_1, ...]."""
        mu, var = self.posterior(Xc)
        return self.ctx.ei_ext("constrained", mu, var, float(best), float(var_eps), float(pof_eps))

    # ------------------------------------------------------------------ plans (fused chain)
    # One plan per BO iteration; each candidate batch is then a single omb_eval_argmax_sobol
    # (Sobol generation → posterior → acquisition → arg-max on the device).
    def plan_ehvi(self, max_point, PF, cache, mode="reference"):
        s00, s01 = pareto.cache_stats(np.asarray(cache, np.float64))
        self.ctx.plan_ehvi2d(pareto.stripes_2d(PF), np.asarray(max_point, np.float64), s00, s01, mode=mode)

    def plan_ehvi_exact(self, max_point, PF):
        coords, _, boxes = pareto.box_decomposition(PF, max_point)
        self.ctx.plan_ehvi_boxes(coords, boxes)

    def plan_ehvi3d(self, max_point, PF, cache):
        self.ctx.plan_ehvi_mc(np.asarray(cache, np.float64), np.asarray(max_point, np.float64),
                              pareto.hypervolume(PF, max_point))

    def plan_expected_decomposition(self, weights, agg_func, agg_min, cache):
        sid, params = agg_func.device_spec()
        self.ctx.plan_expdec(np.asarray(cache, np.float64), sid, params, np.asarray(weights, np.float64),
                             np.asarray(agg_func.ideal_point, np.float64), np.asarray(agg_func.max_point, np.float64),
                             float(agg_min))

    def plan_hvpoi(self, cells):
        self.ctx.plan_hvpoi(np.ascontiguousarray(cells, dtype=np.float64))

    def plan_ei(self, best, var_eps=0.0):
        self.ctx.plan_ei(float(best), float(var_eps))

    def plan_pareto_ei(self, best, var_eps=1e-6):
        self.ctx.plan_ei_ext("pareto", 2, float(best), float(var_eps))

    def plan_constrained_ei(self, best, var_eps=0.0, pof_eps=1e-5):
        self.ctx.plan_ei_ext("constrained", self.n_obj, float(best), float(var_eps), float(pof_eps))

    # ------------------------------------------------------------------ maximiser
    def score(self, acq_fn, X):
        """Acquisition values at host points X (m, d) → numpy (m,); NaN reads as −inf."""
        Xd = self._dev(np.atleast_2d(X))
        v = (self.ctx.eval(Xd) if acq_fn is None else acq_fn(Xd)).cpu().numpy().astype(np.float64)
        return np.where(np.isnan(v), -np.inf, v)

    def polish(self, acq_fn, x0, v0, lower, upper, maxiter=100):
        """Local L-BFGS-B finish from (x0, v0) — what ``differential_evolution(polish=True)`` does to its
        best member (scipy's default; optimisers.py:87,118 use it).  The objective and its central-
        difference gradient come from ONE batched device evaluation of the (2d+1)-point stencil per
        L-BFGS-B step (one-sided at the bounds).  Keeps x0 unless the polished point scores higher.
        The objective is scaled by 1/|v0|: L-BFGS-B's stopping test compares the decrease of f with
        ftol·max(|f|, 1), so an unscaled acquisition of magnitude 1e-3 would stop at a relative accuracy
        of ~1e-6 (the README run's expected decomposition is 1e-4 to 1e-2)."""
        from scipy.optimize import minimize
        lower = np.asarray(lower, np.float64)
        upper = np.asarray(upper, np.float64)
        d = lower.size
        h = 1e-6 * np.maximum(upper - lower, 1e-12)
        scale = 1.0 / abs(v0) if np.isfinite(v0) and v0 != 0.0 else 1.0

        def fg(x):
            x = np.clip(x, lower, upper)
            P = np.repeat(x[None, :], 2 * d + 1, axis=0)
            for j in range(d):
                P[1 + 2 * j, j] = min(x[j] + h[j], upper[j])
                P[2 + 2 * j, j] = max(x[j] - h[j], lower[j])
            v = self.score(acq_fn, P)
            if not np.isfinite(v[0]):
                return np.inf, np.zeros(d)
            g = np.zeros(d)
            for j in range(d):
                a, b = v[1 + 2 * j], v[2 + 2 * j]
                step = P[1 + 2 * j, j] - P[2 + 2 * j, j]
                if np.isfinite(a) and np.isfinite(b) and step > 0:
                    g[j] = (a - b) / step
            return -v[0] * scale, -g * scale

        res = minimize(fg, np.asarray(x0, np.float64), jac=True, method="L-BFGS-B",
                       bounds=list(zip(lower, upper)), options={"maxiter": int(maxiter)})
        x1 = np.clip(res.x, lower, upper)
        v1 = float(self.score(acq_fn, x1[None, :])[0])
        return (x1, v1) if v1 > v0 else (np.asarray(x0, np.float64), float(v0))

    def _starts(self, acq_fn, lower, upper, n_candidates, seed, k, pool=64, sep=0.1):
        """Round 0 of a multi-start search: the ``n_candidates`` Sobol points scored on the device, every rank's
        ``pool`` best (value, global index) pairs gathered, then up to ``k`` starts picked greedily in
        (value desc, index asc) order — the arg-max rule, so start 0 is round 0's arg-max — each at least ``sep``
        (in units of the box) from the starts already taken.  Returns [(x, v)], best first."""
        d = lower.size
        W, rank = world()
        start, count = shard_range(n_candidates, W, rank)
        self.ctx.set_sobol(d, lower, upper, seed=seed)
        vals = self.ctx.eval(self.ctx.sobol(start, count)) if acq_fn is None else acq_fn(self.ctx.sobol(start, count))
        v = torch.nan_to_num(vals, nan=-float("inf"))
        # start 0 is round 0's arg-max by the device rule (value desc, lowest index; NaN never wins): torch.topk does
        # not promise which of several equal values it returns, so the pool alone could miss it on a flat
        # region (e.g. reference-mode EHVI <= 0 with many ties at 0)
        best = global_argmax(self.ctx.argmax_dev(vals, offset=start)).cpu().numpy()
        top = torch.topk(v, min(pool, count))
        pairs = torch.stack([top.values, top.indices.to(torch.float64) + start], 1)
        if W > 1:
            pad = torch.full((pool, 2), -float("inf"), dtype=torch.float64, device=pairs.device)
            pad[:pairs.shape[0]] = pairs
            pad[pairs.shape[0]:, 1] = -1.0
            if torch.distributed.get_backend() == "gloo":
                pad = pad.cpu()
            gathered = [torch.empty_like(pad) for _ in range(W)]
            torch.distributed.all_gather(gathered, pad)
            pairs = torch.cat(gathered)
        P = pairs.cpu().numpy()
        P = P[(P[:, 1] >= 0) & np.isfinite(P[:, 0])]
        P = P[np.lexsort((P[:, 1], -P[:, 0]))]
        if best[1] >= 0 and np.isfinite(best[0]):
            P = np.concatenate([best[None, :], P[P[:, 1] != best[1]]])
        span = np.maximum(upper - lower, 1e-300)
        out = []
        for val, idx in P:
            x = self.ctx.sobol(int(idx), 1).cpu().numpy()[0]
            if all(np.max(np.abs(x - y) / span) >= sep for y, _ in out):
                out.append((x, float(val)))
            if len(out) == k:
                break
        return out

    def maximise(self, acq_fn, lower, upper, n_candidates=1 << 16, seed=0, refine_rounds=2, shrink=0.1,
                 polish=True, starts=None):
        """Arg-max of the acquisition over [lower, upper]^d.

        ``acq_fn`` is None for the current plan (fused chain, one C call per batch) or a callable
        ``acq_fn(Xc_tensor (N, d)) -> (N,) tensor``.  Round 0 scores the first ``n_candidates``
        points of a scrambled Sobol sequence generated on the device (seeded, so every rank sees
        the same sequence and owns one contiguous shard).  Each refinement round re-centres a box
        ``shrink`` times smaller on the incumbent and keeps it if it improves.  ``polish`` then
        finishes with L-BFGS-B from the incumbent, as scipy's differential_evolution does by
        default (``polish``); with several ranks rank 0 polishes and broadcasts the point.
        ``starts`` (default: 1 for n_var ≤ 2, 4 above): independent incumbents refined and polished from
        round 0's best well-separated points (_starts) — round 0's arg-max alone stopped 1.2% short of
        scipy's DE on a 6-D expected decomposition (tests/test_gpu_config1.py); the first start is the
        single-start search's, so the result is never worse.
        Returns (x_best (d,), value).
        """
        lower = np.asarray(lower, np.float64)
        upper = np.asarray(upper, np.float64)
        d = lower.size
        W, rank = world()
        k = (1 if d <= 2 else 4) if starts is None else int(starts)
        if k > 1:
            cands = self._starts(acq_fn, lower, upper, n_candidates, seed, k)
        else:
            start, count = shard_range(n_candidates, W, rank)
            self.ctx.set_sobol(d, lower, upper, seed=seed)
            if acq_fn is None:
                pair = self.ctx.eval_argmax_sobol(start, count)
            else:
                pair = self.ctx.argmax_dev(acq_fn(self.ctx.sobol(start, count)), offset=start)
            g = global_argmax(pair).cpu().numpy()
            cands = [(self.ctx.sobol(int(g[1]), 1).cpu().numpy()[0], float(g[0]))] if g[1] >= 0 else []
        if not cands:   # every candidate was NaN/−inf: fall back to the first Sobol point
            self.ctx.set_sobol(d, lower, upper, seed=seed)
            return self.ctx.sobol(0, 1).cpu().numpy()[0], -np.inf
        results = []
        for best_x, best_v in cands:
            for rnd in range(1, refine_rounds + 1):
                half = shrink ** rnd * (upper - lower) / 2
                lo = np.maximum(lower, best_x - half)
                hi = np.minimum(upper, best_x + half)
                start, count = shard_range(n_candidates, W, rank)
                self.ctx.set_sobol(d, lo, hi, seed=seed + rnd)
                if acq_fn is None:
                    pair = self.ctx.eval_argmax_sobol(start, count)
                else:
                    pair = self.ctx.argmax_dev(acq_fn(self.ctx.sobol(start, count)), offset=start)
                g = global_argmax(pair).cpu().numpy()
                if g[1] >= 0 and g[0] > best_v:
                    best_x = self.ctx.sobol(int(g[1]), 1).cpu().numpy()[0]   # the winner, regenerated
                    best_v = float(g[0])
            if polish:
                if W == 1:
                    best_x, best_v = self.polish(acq_fn, best_x, best_v, lower, upper)
                else:
                    box = [None]
                    if rank == 0:
                        box[0] = self.polish(acq_fn, best_x, best_v, lower, upper)
                    torch.distributed.broadcast_object_list(box, src=0)
                    best_x, best_v = np.asarray(box[0][0], np.float64), float(box[0][1])
            results.append((best_x, best_v))
        # the best start; ties to the earliest (the single-start search's when it ties)
        return max(results, key=lambda r: r[1])


_ENGINES = {}


def engine_for(models, device=None):
    """Process-wide engine per device with ``models`` resident."""
    if device is None:
        device = torch.cuda.current_device() if torch.cuda.is_available() else 0
    eng = _ENGINES.get(device)
    if eng is None:
        eng = _ENGINES[device] = AcquisitionEngine(device)
    return eng.load_models(models)
