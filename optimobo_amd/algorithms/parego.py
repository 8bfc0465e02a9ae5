"""``optimobo.algorithms.parego.ParEGO`` (parego.py:12-298) with a device maximiser.

The host loop (random Das-Dennis weight, scalarised archive, one GP on it, EI with
σ = sqrt(σ² + 1e-6)) follows the reference.  The reference's 20-member evolutionary
search with 1,000 sequential re-mutations (~26,000 single-point predictions, parego.py:228-271)
is replaced by the batched device arg-max of the same EI over a Sobol batch.
"""
import numpy as np

from ..refdirs import get_reference_directions
from ._base import BODriver


class ParEGO(BODriver):
    def _expected_improvement(self, X, model, opt_value, kappa=0.01):
        """parego.py:126-145; X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([model], self.device).ei(Xb, opt_value, 1e-6).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def _get_proposed(self, model, current_best):
        from ..acquisition import engine_for
        eng = engine_for([model], self.device)
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
            next_X, _ = self._get_proposed(model, current_best)
            next_y = self._objective_function(problem, next_X)
            ysample = np.vstack((ysample, next_y))
            Xsample = np.vstack((Xsample, next_X))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)
