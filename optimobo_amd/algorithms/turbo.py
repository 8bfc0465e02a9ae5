"""``optimobo.algorithms.turbo.TuRBO_1`` / ``TuRBO_M`` (turbo.py:17-574) with device Thompson sampling.

TuRBO fits one GP to the scalarised local history of a trust region and scores up to 5,000
candidates inside it by Thompson sampling: ``batch_size`` joint posterior draws
(``create_candidates``, turbo.py:75-117 — GPy ``posterior_samples``: a full posterior
covariance and ``numpy.random.multivariate_normal``, an O(N³) SVD on the host), then the
greedy per-draw arg-min (``select_candidates`` :142-153, ``TuRBO_M._select_candidates``
:365-383).  Here the covariance (FP64 MFMA GEMM), its Cholesky factor (blocked, in HIP), the
draws μ + L z and the greedy selection run on the GPU (omb_posterior_samples,
omb_thompson_select).  The trust-region bookkeeping follows the reference line by line,
including its quirks (TuRBO_M judges success on column 0 of the objective archive,
turbo.py:350; TuRBO_1 appends the initial aggregated values to the global history, :261).
"""
import math
from copy import deepcopy

import numpy as np
from scipy.stats import qmc

from .. import pareto
from .. import util_functions
from ..gp import GPRegression, Matern52
from ..refdirs import get_reference_directions
from ..result import Res


class TuRBO_1:  # noqa: N801 — reference class name
    """https://doi.org/10.48550/arXiv.1910.01739 — one trust region (turbo.py:17-304)."""

    def __init__(self, test_problem, batch_size, ideal_point=None, max_point=None, device=None):
        self.test_problem = test_problem
        self.max_point = max_point
        self.ideal_point = ideal_point
        self.n_vars = test_problem.n_var
        self.n_obj = test_problem.n_obj
        self.upper = test_problem.xu
        self.lower = test_problem.xl
        self.n_evals = 0
        self.budget = 100
        self.Xsample = np.zeros((0, self.n_vars))
        self.ysample = np.zeros((0, self.n_obj))
        self.aggregated_samples = np.zeros((0, 1))
        self.batch_size = batch_size
        self.n_cand = min(100 * self.n_vars, 5000)
        self.length_min = 0.5 ** 7
        self.length_max = 1.6
        self.length_init = 0.4
        self.length = self.length_init
        self.ref_dirs = get_reference_directions("das-dennis", self.n_obj, n_partitions=10)
        self.failtol = np.ceil(np.max([4.0 / batch_size, self.n_vars / batch_size]))
        self.succtol = 3
        self.is_ideal_known = ideal_point is not None
        self.is_max_known = max_point is not None
        self.device = device            # not in the reference: GPU of the sampling path

    def _objective_function(self, problem, x):
        return problem.evaluate(x)

    def normalise(self, X):
        return (np.asarray(X) - np.asarray(self.lower)) / (np.asarray(self.upper) - np.asarray(self.lower))

    def denormalise(self, X):
        return (X * (self.upper - self.lower)) + self.lower

    def _fit(self, X, y):
        model = GPRegression(X, np.reshape(y, (-1, 1)), Matern52(self.n_vars, ARD=True))
        model.Gaussian_noise.variance.fix(0)
        model.optimize(messages=False, max_f_eval=1000)
        return model

    def _candidate_points(self, Xsample, ysample, GP, length):
        """turbo.py:79-111: Sobol points in the ℓ-shaped box around the incumbent, perturbing
        min(20/d, 1) of the coordinates of the centre (numpy's global generator, as the reference)."""
        assert Xsample.min() >= 0.0 and Xsample.max() <= 1.0
        x_center = Xsample[ysample.argmin().item(), :][None, :]
        weights = np.asarray(GP.kern.lengthscale.values if hasattr(GP.kern.lengthscale, "values")
                             else GP.kern.lengthscale, np.float64)
        weights = np.broadcast_to(weights, (self.n_vars,)).astype(np.float64)
        weights = weights / weights.mean()
        weights = weights / np.prod(np.power(weights, 1.0 / len(weights)))
        lb = np.clip(x_center - weights * length / 2.0, 0.0, 1.0)
        ub = np.clip(x_center + weights * length / 2.0, 0.0, 1.0)
        sample = qmc.Sobol(d=self.n_vars, scramble=False).random(n=self.n_cand)
        sample = qmc.scale(sample, lb[0], ub[0])
        prob_perturb = min(20.0 / self.n_vars, 1.0)
        mask = np.random.rand(self.n_cand, self.n_vars) <= prob_perturb
        ind = np.where(np.sum(mask, axis=1) == 0)[0]
        mask[ind, np.random.randint(0, self.n_vars - 1, size=len(ind))] = 1
        X_cand = x_center.copy() * np.ones((self.n_cand, self.n_vars))
        X_cand[mask] = sample[mask]
        return X_cand

    def create_candidates(self, Xsample, ysample, GP, length):
        """turbo.py:75-117 → (X_cand (n_cand, d), y_cand (n_cand, 1, batch_size)); draws on the GPU."""
        X_cand = self._candidate_points(Xsample, ysample, GP, length)
        y_cand = GP.posterior_samples(X_cand, size=self.batch_size)
        return X_cand, y_cand

    def _thompson(self, GP, X_cand):
        """(batch_size, n_cand) device tensor of joint draws at X_cand."""
        Y, _ = GP.posterior_samples_device(X_cand, self.batch_size)
        return Y

    def select_candidates(self, X_cand, y_cand):
        """turbo.py:142-153: the arg-min of every draw, never picking a point twice.
        y_cand is (n_cand, 1, batch_size) host values or a (batch_size, n_cand) device tensor."""
        idx = _select(y_cand, self.batch_size, self.device)
        return np.asarray(X_cand)[idx].copy()

    def _restart(self):
        self._Xsample = []
        self._ysample = []
        self.failcount = 0
        self.succcount = 0
        self.length = self.length_init

    def _adjust_length(self, fX_next):
        """turbo.py:127-140."""
        best = np.min(self._aggregated_samples)
        if np.min(fX_next) < best - 1e-3 * math.fabs(best):
            self.succcount += 1
            self.failcount = 0
        else:
            self.succcount = 0
            self.failcount += 1
        if self.succcount == self.succtol:
            self.length = min([2.0 * self.length, self.length_max])
            self.succcount = 0
        elif self.failcount == self.failtol:
            self.length /= 2.0
            self.failcount = 0

    def get_random_weight(self):
        return self.ref_dirs[np.random.randint(0, len(self.ref_dirs))]

    def _hypervolume(self):
        ref = self.max_point if self.max_point is not None else (
            self.ysample.max(axis=0) if len(self.ysample) else None)
        return 0.0 if ref is None else pareto.hypervolume(self.ysample, ref)

    def solve(self, aggregation_func, budget=100, n_init_samples=5):
        """turbo.py:158-304."""
        self.budget = budget
        hypervolume_convergence = []
        while self.n_evals < self.budget:
            hypervolume_convergence.append(self._hypervolume())
            self._restart()
            variable_ranges = list(zip(self.test_problem.xl, self.test_problem.xu))
            Xsample = util_functions.generate_latin_hypercube_samples(n_init_samples, variable_ranges)
            ysample = np.asarray([self._objective_function(self.test_problem, x) for x in Xsample])
            aggregated_samples = np.asarray([aggregation_func(i, [0.5, 0.5]) for i in ysample]).flatten()
            self.n_evals = self.n_evals + n_init_samples
            self._Xsample = deepcopy(Xsample)
            self._ysample = deepcopy(ysample)
            self._aggregated_samples = np.reshape(aggregated_samples, (-1, 1))
            self.Xsample = np.vstack((self.Xsample, deepcopy(Xsample)))
            self.ysample = np.vstack((self.ysample, deepcopy(ysample)))
            self.aggregated_samples = np.vstack((self.aggregated_samples,
                                                 np.reshape(deepcopy(aggregated_samples), (-1, 1))))
            while self.n_evals < self.budget and self.length >= self.length_min:
                Xsample_normed = self.normalise(self._Xsample)
                aggre = self._aggregated_samples
                GP = self._fit(Xsample_normed, aggre)
                X_cand = self._candidate_points(Xsample_normed, aggre, GP, self.length)
                X_next = self.select_candidates(X_cand, self._thompson(GP, X_cand))
                X_next = self.denormalise(X_next)
                ref_dir = self.get_random_weight()
                y_next = np.array([self._objective_function(self.test_problem, x) for x in X_next])
                aggregated_next = np.array([aggregation_func(y, ref_dir) for y in y_next])
                self._adjust_length(aggregated_next)
                self.n_evals += self.batch_size
                self._Xsample = np.vstack((self._Xsample, X_next))
                self._ysample = np.vstack((self._ysample, y_next))
                self._aggregated_samples = np.vstack((self._aggregated_samples, aggregated_next))
                self.Xsample = np.vstack((self.Xsample, deepcopy(X_next)))
                self.ysample = np.vstack((self.ysample, deepcopy(y_next)))
                # turbo.py:261 appends the initial aggregated values, not aggregated_next
                self.aggregated_samples = np.vstack((self.aggregated_samples,
                                                     np.reshape(deepcopy(aggregated_samples), (-1, 1))))
        return self._result(hypervolume_convergence, n_init_samples)

    def _result(self, hypervolume_convergence, n_init_samples):
        pf_approx = util_functions.calc_pf(self.ysample)
        indicies = [i for i, item in enumerate(self.ysample) if item in pf_approx]
        return Res(pf_approx, self.Xsample[indicies], self.ysample, self.Xsample, hypervolume_convergence,
                   self.n_obj, n_init_samples)


class TuRBO_M(TuRBO_1):  # noqa: N801 — reference class name
    """TuRBO-m: several trust regions competing for one batch (turbo.py:307-574)."""

    def __init__(self, test_problem, ideal_point, max_point, batch_size, n_trust_regions, device=None):
        self.n_trust_regions = n_trust_regions
        super().__init__(test_problem=test_problem, ideal_point=ideal_point, max_point=max_point,
                         batch_size=batch_size, device=device)
        self.succtol = 3
        self.failtol = max(5, self.n_vars)
        self.hypers = [{} for _ in range(self.n_trust_regions)]
        self._restart()

    def _restart(self):
        self._idx = np.zeros((0, 1), dtype=int)
        self.failcount = np.zeros(self.n_trust_regions, dtype=int)
        self.succcount = np.zeros(self.n_trust_regions, dtype=int)
        self.length = self.length_init * np.ones(self.n_trust_regions)

    def _adjust_length(self, fX_next, i):
        """turbo.py:347-363 (the target is column 0 of the objective archive, as the reference)."""
        assert 0 <= i <= self.n_trust_regions - 1
        fX_min = self.ysample[self._idx[:, 0] == i, 0].min()
        if fX_next.min() < fX_min - 1e-3 * math.fabs(fX_min):
            self.succcount[i] += 1
            self.failcount[i] = 0
        else:
            self.succcount[i] = 0
            self.failcount[i] += len(fX_next)
        if self.succcount[i] == self.succtol:
            self.length[i] = min([2.0 * self.length[i], self.length_max])
            self.succcount[i] = 0
        elif self.failcount[i] >= self.failtol:
            self.length[i] /= 2.0
            self.failcount[i] = 0

    def _select_candidates(self, X_cand, y_cand):
        """turbo.py:365-383: X_cand (T, n_cand, d); y_cand (T, n_cand, B) host values or a
        (B, T·n_cand) device tensor → (X_next (B, d), idx_next (B, 1) trust region of each pick)."""
        T, n = X_cand.shape[0], X_cand.shape[1]
        if not hasattr(y_cand, "device"):
            assert y_cand.shape == (self.n_trust_regions, self.n_cand, self.batch_size)
            assert np.all(np.isfinite(y_cand))
        assert X_cand.min() >= 0.0 and X_cand.max() <= 1.0
        flat = _select(y_cand, self.batch_size, self.device)
        i, j = np.unravel_index(flat, (T, n))
        X_next = np.asarray(X_cand)[i, j, :].copy()
        return X_next, i.reshape(-1, 1).astype(int)

    def solve(self, aggregation_func, budget, n_init_samples):
        """turbo.py:385-574."""
        import torch
        hypervolume_convergence = []
        self.budget = budget
        assert self.n_trust_regions > 1 and isinstance(budget, int)
        assert self.budget > self.n_trust_regions * n_init_samples, "Not enough trust regions to do initial evaluations"
        assert budget > self.batch_size, "Not enough evaluations to do a single batch"
        variable_ranges = list(zip(self.test_problem.xl, self.test_problem.xu))
        for i in range(self.n_trust_regions):
            ref_dir = self.get_random_weight()
            Xsample = util_functions.generate_latin_hypercube_samples(n_init_samples, variable_ranges)
            ysample = np.asarray([self._objective_function(self.test_problem, x) for x in Xsample])
            aggregated_samples = np.asarray([aggregation_func(i, ref_dir) for i in ysample]).flatten()
            self.n_evals = self.n_evals + n_init_samples
            self._idx = np.vstack((self._idx, i * np.ones((n_init_samples, 1), dtype=int)))
            self.Xsample = np.vstack((self.Xsample, deepcopy(Xsample)))
            self.ysample = np.vstack((self.ysample, deepcopy(ysample)))
            self.aggregated_samples = np.vstack((self.aggregated_samples,
                                                 np.reshape(deepcopy(aggregated_samples), (-1, 1))))
        while self.n_evals < self.budget:
            X_cand = np.zeros((self.n_trust_regions, self.n_cand, self.n_vars))
            draws = []
            for i in range(self.n_trust_regions):
                idx = np.where(self._idx == i)[0]
                Xsample_normed = self.normalise(self.Xsample[idx, :])
                aggre = self.aggregated_samples[idx, :]
                GP = self._fit(Xsample_normed, aggre)
                X_cand[i, :, :] = self._candidate_points(Xsample_normed, aggre, GP, self.length[i])
                draws.append(self._thompson(GP, X_cand[i]))
            # (B, T·n_cand) in the row-major (region, candidate) order np.unravel_index reads
            y_dev = torch.cat(draws, dim=1)
            X_next, idx_next = self._select_candidates(X_cand, y_dev)
            assert X_next.min() >= 0.0 and X_next.max() <= 1.0
            X_next = self.denormalise(X_next)
            ref_dir = self.get_random_weight()
            y_next = np.array([self._objective_function(self.test_problem, x) for x in X_next])
            aggregated_next = np.array([aggregation_func(y, ref_dir) for y in y_next])
            for i in range(self.n_trust_regions):
                idx_i = np.where(idx_next == i)[0]
                if len(idx_i) > 0:
                    self.hypers[i] = {}
                    self._adjust_length(aggregated_next[idx_i], i)
            self.n_evals += self.batch_size
            self.Xsample = np.vstack((self.Xsample, deepcopy(X_next)))
            self.ysample = np.vstack((self.ysample, deepcopy(y_next)))
            self.aggregated_samples = np.vstack((self.aggregated_samples,
                                                 np.reshape(deepcopy(aggregated_next), (-1, 1))))
            self._idx = np.vstack((self._idx, deepcopy(idx_next)))
            for i in range(self.n_trust_regions):
                if self.length[i] < self.length_min:
                    idx_i = self._idx[:, 0] == i
                    self.length[i] = self.length_init
                    self.succcount[i] = 0
                    self.failcount[i] = 0
                    self._idx[idx_i, 0] = -1
                    self.hypers[i] = {}
                    Xsample = util_functions.generate_latin_hypercube_samples(n_init_samples, variable_ranges)
                    ysample = np.asarray([self._objective_function(self.test_problem, x) for x in Xsample])
                    aggregated_samples = np.asarray([aggregation_func(i, [0.5, 0.5]) for i in ysample]).flatten()
                    self.Xsample = np.vstack((self.Xsample, Xsample))
                    self.ysample = np.vstack((self.ysample, ysample))
                    self.aggregated_samples = np.vstack((self.aggregated_samples,
                                                         np.reshape(aggregated_samples, (-1, 1))))
                    self._idx = np.vstack((self._idx, i * np.ones((n_init_samples, 1), dtype=int)))
                    self.n_evals += n_init_samples
        return self._result(hypervolume_convergence, n_init_samples)


def _select(y_cand, batch_size, device):
    """Flat pick indices: host (…, B) values are uploaded as (B, ·); device (B, ·) tensors are used as is."""
    import torch
    from ..acquisition import engine_for
    if isinstance(y_cand, torch.Tensor):
        Y = y_cand
        eng_dev = Y.device.index
    else:
        y = np.asarray(y_cand, np.float64)
        Y = np.ascontiguousarray(np.moveaxis(y, -1, 0).reshape(y.shape[-1], -1))
        eng_dev = device
    eng = engine_for([], eng_dev)
    return eng.ctx.thompson_select(Y).cpu().numpy()
