"""``optimobo.algorithms.parego.ParEGO`` (parego.py:12-298) with a device maximiser.

The host loop (random Das-Dennis weight, scalarised archive, one GP on it, EI with
σ = sqrt(σ² + 1e-6)) follows the reference.  The acquisition search is the reference's own
20-member evolutionary search with 1,000 generations (parego.py:223-271), run on the device
(omb_ea_search, optimobo_amd/ea.py): the temporary population and the search's random draws come
from numpy's and Python's global generators in the reference's call order, so with the same
surrogate it returns the reference's proposal.  `acq_search = "batch"` uses the batched device
arg-max of the same EI over a Sobol batch instead.
"""
import numpy as np

from .. import ea
from ..refdirs import get_reference_directions
from ._base import BODriver


class ParEGO(BODriver):
    acq_search = "ea"
    def _expected_improvement(self, X, model, opt_value, kappa=0.01):
        """parego.py:126-145; X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([model], self.device).ei(Xb, opt_value, 1e-6).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def _get_proposed(self, model, current_best, Xsample=None):
        from ..acquisition import engine_for
        eng = engine_for([model], self.device)
        if self.acq_search == "ea" and Xsample is not None and ea.device_search_fits(len(Xsample)):
            lower = np.asarray(self.test_problem.xl, np.float64)
            upper = np.asarray(self.test_problem.xu, np.float64)
            pop = ea.initial_population(Xsample, lower, upper)           # parego.py:229-235
            tape = ea.ea_tape(len(pop), Xsample.shape[1])               # the search's draws, parego.py:238-269
            return eng.ctx.ea_search(pop, tape, current_best, lower, upper, mode=0)
        if self.acq_search == "ea" and Xsample is not None:
            ea.warn_batch_fallback("ParEGO", len(Xsample))
        eng.plan_ei(current_best, 1e-6)
        return self._maximise([model], None)

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
            model = self._fit(Xsample, aggregated)
            current_best = aggregated[np.argmin(aggregated)]
            next_X, _ = self._get_proposed(model, current_best, Xsample)
            next_y = self._objective_function(problem, next_X)
            ysample = np.vstack((ysample, next_y))
            Xsample = np.vstack((Xsample, next_X))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)
