"""Drop-in ``optimobo.algorithms.emo.EMO`` (emo.py:14-333): hypervolume-based PoI.

Cells come from the reference-exact 2-D decomposition (optimobo_amd.pareto); the HV-PoI of a
candidate batch runs in the omb_hvpoi kernel and is maximised by the device arg-max.
"""
import numpy as np

from .. import pareto
from ._base import BODriver


class EMO(BODriver):
    def decompose_into_cells(self, data_points):
        """emo.py:55-152 (2 objectives)."""
        return pareto.decompose_into_cells(data_points, self.ideal_point, self.max_point)

    def vol5(self, mu, lower, upper):
        """emo.py:176-189: volume of the part of cell [lower, upper] dominated by μ."""
        mu, lower, upper = (np.asarray(a, np.float64) for a in (mu, lower, upper))
        if not np.all(upper > mu):
            return 0
        return np.prod(upper - np.maximum(lower, mu))

    def hypervolume_improvement(self, query_point, P, ref_point):
        """emo.py:155-174: HV(P ∪ {q}) − HV(P), clipped at 0."""
        before = pareto.hypervolume(P, ref_point)
        after = pareto.hypervolume(np.vstack((P, query_point)), ref_point)
        return max(after - before, 0)

    def hypervolume_based_PoI(self, X, models, P, cells):
        """emo.py:192-228 on the device. X (d,) → float; X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for(models, self.device).hvpoi(Xb, cells).cpu().numpy()
        return float(out[0]) if np.ndim(X) == 1 else out

    def get_proposed(self, function, P, cells, models):
        """emo.py:231-241: maximise HV-PoI with the device arg-max."""
        from ..acquisition import engine_for
        engine_for(models, self.device).plan_hvpoi(cells)
        x, v = self._maximise(models, None)
        return x, -v

    def solve(self, budget=100, n_init_samples=5):
        problem = self.test_problem
        Xsample, ysample = self._initial_samples(n_init_samples)
        hypervolume_convergence = []
        for _ in range(budget):
            # emo.py:264-285 updates the bounds without a scalarisation object
            if not self.is_ideal_known:
                self.ideal_point = ysample.min(axis=0).astype(float)
            if not self.is_max_known:
                self.max_point = ysample.max(axis=0).astype(float)
            hypervolume_convergence.append(self._hypervolume(ysample))
            models = self._fit_many(Xsample, ysample[:, :self.n_obj])
            cells = self.decompose_into_cells(pareto.calc_pf(ysample))
            X_next, _ = self.get_proposed(self.hypervolume_based_PoI, ysample, cells, models)
            y_next = self._objective_function(problem, X_next)
            ysample = np.vstack((ysample, y_next))
            Xsample = np.vstack((Xsample, X_next))
        return self._result(ysample, Xsample, hypervolume_convergence, n_init_samples)
