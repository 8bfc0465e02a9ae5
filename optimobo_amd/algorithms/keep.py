"""``optimobo.algorithms.keep.KEEP`` (keep.py:12-320) with a device maximiser.

KEEP is ParEGO with a second GP: besides the model of the scalarised archive it fits a model
of Pareto-set membership (1 for archive points in the current front, 0 otherwise,
keep.py:227-238) and ranks candidates by μ_pareto(x) · EI(x) with σ = sqrt(σ² + 1e-6)
(pareto_expected_improvement, keep.py:142-151).  The host loop follows the reference; the
acquisition search is the reference's 20-member evolutionary search with 1,000 generations
(keep.py:240-287) run on the device (omb_ea_search mode OMB_EA_PARETO_EI, draws from the global
generators in the reference's order).  `acq_search = "batch"` uses the batched device arg-max of the
same fitness instead (omb_plan_ei_ext, kind "pareto": both posteriors and the product in one chain).
"""
import numpy as np

from .. import ea, pareto
from ..refdirs import get_reference_directions
from ._base import BODriver


class KEEP(BODriver):
    acq_search = "ea"
    def _expected_improvement(self, X, model, opt_value, kappa=0.01):
        """keep.py:118-137 (σ = sqrt(σ² + 1e-6)); X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([model], self.device).ei(Xb, opt_value, 1e-6).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def pareto_expected_improvement(self, X, pareto_model, scalarised_model, opt_value):
        """keep.py:142-151: μ_pareto · EI.  X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([scalarised_model, pareto_model], self.device).pareto_ei(Xb, opt_value).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def _get_proposed(self, pareto_model, scalar_model, current_best, Xsample=None):
        from ..acquisition import engine_for
        eng = engine_for([scalar_model, pareto_model], self.device)
        if self.acq_search == "ea" and Xsample is not None and ea.device_search_fits(len(Xsample)):
            lower = np.asarray(self.test_problem.xl, np.float64)
            upper = np.asarray(self.test_problem.xu, np.float64)
            pop = ea.initial_population(Xsample, lower, upper)           # keep.py:246-252
            tape = ea.ea_tape(len(pop), Xsample.shape[1])               # keep.py:256-290
            return eng.ctx.ea_search(pop, tape, current_best, lower, upper, mode=1)
        if self.acq_search == "ea" and Xsample is not None:
            ea.warn_batch_fallback("KEEP", len(Xsample))
        eng.plan_pareto_ei(current_best)
        return self._maximise([scalar_model, pareto_model], None)

    @staticmethod
    def _membership(Xsample, ysample):
        """keep.py:228-234, including numpy's `row in array` (any element equal)."""
        pareto_set = pareto.calc_pf(ysample)
        probs = np.zeros(len(Xsample))
        for i in range(len(Xsample)):
            if ysample[i] in pareto_set:
                probs[i] = 1
        return probs

    def solve(self, aggregation_func, budget=100, n_init_samples=5):
        problem = self.test_problem
        Xsample, ysample = self._initial_samples(n_init_samples)
        ref_dirs = get_reference_directions("das-dennis", problem.n_obj, n_partitions=100)
        hypervolume_convergence = []
        for _ in range(budget):
            self._update_bounds(ysample, aggregation_func)
            hypervolume_convergence.append(self._hypervolume(ysample))
            ref_dir = ref_dirs[np.random.randint(0, len(ref_dirs))]
            aggregated = np.asarray([aggregation_func(y, ref_dir) for y in ysample]).flatten()
            scalar_model = self._fit(Xsample, aggregated)
            pareto_model = self._fit(Xsample, self._membership(Xsample, ysample))
            current_best = aggregated[np.argmin(aggregated)]
            next_X, _ = self._get_proposed(pareto_model, scalar_model, current_best, Xsample)
            next_y = self._objective_function(problem, next_X)
            ysample = np.vstack((ysample, next_y))
            Xsample = np.vstack((Xsample, next_X))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)
