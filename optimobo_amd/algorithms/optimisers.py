"""Drop-in ``optimobo.algorithms.optimisers`` (optimisers.py:18-527).

``MultiSurrogateOptimiser(problem, ideal, max).solve(budget, n_init_samples,
sample_exponent, acquisition_func)`` and ``MonoSurrogateOptimiser(...).solve(aggregation_func,
budget, n_init_samples)`` keep the reference signatures and return ``Res``.  Extra keyword
arguments select the device maximiser: ``mode`` ("reference" = bug-compatible acquisition
values, "textbook" = exact EHVI), ``n_candidates`` (Sobol batch per iteration), ``refine_rounds``,
``seed`` and ``device``.
"""
import numpy as np

from .. import pareto
from ..refdirs import get_reference_directions
from ._base import BODriver


class MultiSurrogateOptimiser(BODriver):
    """One GP per objective; EHVI (2-D / 3-D) or expected decomposition as the acquisition."""

    def _get_cached_samples(self, dimensions, sample_exponent):
        """optimisers.py:121-141 — scrambled Sobol mapped through the normal ppf."""
        return pareto.cached_samples(dimensions, sample_exponent, seed=self.seed)

    def _get_proposed_EHVI(self, function, models, ideal_point, max_point, pf, cache):
        """optimisers.py:91-119 on the device: returns (x, −EHVI(x))."""
        from ..acquisition import engine_for
        eng = engine_for(models, self.device)
        mc = function == "EHVI_3D" or self.n_obj >= 3          # optimisers.py:245-248: EHVI_3D for n_obj != 2
        if mc and self.mode == "textbook" and self.n_obj <= 3:
            eng.plan_ehvi_exact(max_point, pf)          # exact EHVI in place of the MC estimate (k = 2, 3)
        elif mc:
            eng.plan_ehvi3d(max_point, pf, cache)       # the reference's Monte-Carlo form, any k ≥ 3
        else:
            eng.plan_ehvi(max_point, pf, cache, mode=self.mode)
        x, v = self._maximise(models, None)
        return x, -v

    def _get_proposed_scalarisation(self, function, models, min_val, scalar_func, ref_dir, cache):
        """optimisers.py:62-88 on the device: returns (x, −value, ref_dir)."""
        from ..acquisition import engine_for
        eng = engine_for(models, self.device)
        eng.plan_expected_decomposition(ref_dir, scalar_func, min_val, cache)
        x, v = self._maximise(models, None)
        return x, -v, ref_dir

    def solve(self, budget=100, n_init_samples=5, sample_exponent=5, acquisition_func=None):
        problem = self.test_problem
        Xsample, ysample = self._initial_samples(n_init_samples)
        cached_samples = self._get_cached_samples(self.n_obj, sample_exponent)
        ref_dirs = get_reference_directions("das-dennis", self.n_obj, n_partitions=100)
        hypervolume_convergence = []
        for _ in range(budget):
            self._update_bounds(ysample, acquisition_func)
            hypervolume_convergence.append(self._hypervolume(ysample))
            models = self._fit_many(Xsample, ysample[:, :problem.n_obj])
            ref_dir = np.asarray(ref_dirs[np.random.randint(0, len(ref_dirs))])
            if acquisition_func is None:
                pf = pareto.calc_pf(ysample)
                fn = "EHVI" if problem.n_obj == 2 else "EHVI_3D"
                X_next, _ = self._get_proposed_EHVI(fn, models, self.ideal_point, self.max_point, pf, cached_samples)
            else:
                min_scalar = np.min([acquisition_func(y, ref_dir) for y in ysample])
                X_next, _, _ = self._get_proposed_scalarisation("expected_decomposition", models, min_scalar,
                                                                acquisition_func, ref_dir, cached_samples)
            y_next = self._objective_function(problem, X_next)
            ysample = np.vstack((ysample, y_next))
            Xsample = np.vstack((Xsample, X_next))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)


class MonoSurrogateOptimiser(BODriver):
    """One GP on scalarised objectives; EI as the acquisition (optimisers.py:283-527)."""

    def _expected_improvement(self, X, model, opt_value, kappa=0.01):
        """optimisers.py:325-344 (σ = sqrt(σ²)); X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([model], self.device).ei(Xb, opt_value, 0.0).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def _get_proposed(self, function, models, current_best):
        from ..acquisition import engine_for
        eng = engine_for([models], self.device)
        eng.plan_ei(current_best, 0.0)
        x, v = self._maximise([models], None)
        return x, -v

    def _normalize_data(self, data):
        return (data - np.min(data)) / (np.max(data) - np.min(data))

    def solve(self, aggregation_func, budget=100, n_init_samples=5):
        problem = self.test_problem
        weights = np.asarray([1 / problem.n_obj] * problem.n_obj)
        Xsample, ysample = self._initial_samples(n_init_samples)
        self._update_bounds(ysample, aggregation_func)
        aggregated_samples = np.asarray([aggregation_func(i, weights) for i in ysample]).flatten()
        ref_dirs = get_reference_directions("das-dennis", problem.n_obj, n_partitions=100)
        hypervolume_convergence = []
        for _ in range(budget):
            self._update_bounds(ysample, aggregation_func)
            hypervolume_convergence.append(self._hypervolume(ysample))
            current_best = aggregated_samples[np.argmin(aggregated_samples)]
            model = self._fit(Xsample, aggregated_samples)
            next_X, _ = self._get_proposed(self._expected_improvement, model, current_best)
            next_y = self._objective_function(problem, next_X)
            ysample = np.vstack((ysample, next_y))
            ref_dir = ref_dirs[np.random.randint(0, len(ref_dirs))]
            aggregated_samples = np.append(aggregated_samples, aggregation_func(next_y, ref_dir))
            Xsample = np.vstack((Xsample, next_X))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)
