"""Shared BO-driver plumbing of the drop-in optimisers.

The loop structure, bounds bookkeeping, hypervolume trace, surrogate fitting and result
assembly follow the reference drivers (optimisers.py:144-277, 373-527; emo.py:244-328;
parego.py:148-298).  What changes is the acquisition maximiser: the reference's per-candidate
``differential_evolution`` is replaced by the batched device arg-max
(optimobo_amd.acquisition.AcquisitionEngine.maximise).
"""
import numpy as np

from .. import pareto
from .. import util_functions
from ..acquisition import engine_for
from ..gp import GPRegression, Matern52, fit_concurrently
from ..parallel import agree_host_rng
from ..result import Res


class BODriver:
    def __init__(self, test_problem, ideal_point=None, max_point=None, mode="reference", n_candidates=1 << 14,
                 refine_rounds=2, seed=None, device=None):
        self.test_problem = test_problem
        self.max_point = max_point
        self.ideal_point = ideal_point
        self.n_vars = test_problem.n_var
        self.n_obj = test_problem.n_obj
        self.upper = test_problem.xu
        self.lower = test_problem.xl
        self.is_ideal_known = ideal_point is not None
        self.is_max_known = max_point is not None
        # device-maximiser settings (not in the reference, which uses scipy DE)
        if mode not in ("reference", "textbook"):
            raise ValueError("mode must be 'reference' or 'textbook'")
        self.mode = mode
        self.n_candidates = int(n_candidates)
        self.refine_rounds = int(refine_rounds)
        # several ranks (torch.distributed initialised): one seed and one numpy state for all of them
        self.seed = agree_host_rng(seed)
        self.device = device
        self._iteration = 0

    def _objective_function(self, problem, x):
        return problem.evaluate(x)

    # -- optimisers.py:189-213 (the AttributeError for an unset acquisition_func is the reference's)
    def _update_bounds(self, ysample, scal):
        if not self.is_ideal_known and not self.is_max_known:
            self.max_point = ysample.max(axis=0).astype(float)
            self.ideal_point = ysample.min(axis=0).astype(float)
            self._set_bounds(scal, self.ideal_point, self.max_point)
        elif not self.is_ideal_known:
            self.ideal_point = ysample.min(axis=0).astype(float)
            self._set_bounds(scal, self.ideal_point, self.max_point)
        elif not self.is_max_known:
            self.max_point = ysample.max(axis=0).astype(float)
            self._set_bounds(scal, self.ideal_point, self.max_point)

    def _set_bounds(self, scal, lo, hi):
        if scal is None and self.mode == "textbook":
            return
        scal.set_bounds(lo, hi)       # reference mode: None raises AttributeError, as the reference does

    def _hypervolume(self, ysample):
        return pareto.hypervolume(ysample, self.max_point)

    def _model(self, X, y):
        model = GPRegression(X, np.reshape(y, (-1, 1)), Matern52(self.n_vars, ARD=True))
        model.Gaussian_noise.variance.fix(0)
        return model

    def _fit(self, X, y):
        model = self._model(X, y)
        model.optimize(messages=False, max_f_eval=1000)
        return model

    def _fit_many(self, X, ys):
        """One surrogate per column of ``ys`` on the same inputs, as the reference's per-objective
        loop does (optimisers.py:186, emo.py:297-301); the independent fits run concurrently on the
        GPU (gp.fit_concurrently), each taking the path it takes alone."""
        models = [self._model(X, ys[:, i]) for i in range(ys.shape[1])]
        fit_concurrently(models, device=self.device, messages=False, max_f_eval=1000)
        return models

    def _maximise(self, models, acq_fn):
        """acq_fn None: the plan set on the engine (fused chain); else a batched callable."""
        eng = engine_for(models, self.device)
        seed = (self.seed if self.seed is not None else np.random.randint(0, 2 ** 31 - 1)) + 7919 * self._iteration
        self._iteration += 1
        return eng.maximise(acq_fn, self.test_problem.xl, self.test_problem.xu, n_candidates=self.n_candidates,
                            seed=seed, refine_rounds=self.refine_rounds)

    def _result(self, ysample, Xsample, hypervolume_convergence, n_init_samples):
        pf_approx = util_functions.calc_pf(ysample)
        # optimisers.py:269-273 (numpy `in`: any coordinate of the row appears in pf_approx)
        indicies = [i for i, item in enumerate(ysample) if item in pf_approx]
        return Res(pf_approx, Xsample[indicies], ysample, Xsample, hypervolume_convergence, self.n_obj,
                   n_init_samples)

    def _initial_samples(self, n_init_samples):
        ranges = list(zip(self.test_problem.xl, self.test_problem.xu))
        Xsample = util_functions.generate_latin_hypercube_samples(n_init_samples, ranges)
        ysample = np.asarray([self._objective_function(self.test_problem, x) for x in Xsample])
        return Xsample, ysample
