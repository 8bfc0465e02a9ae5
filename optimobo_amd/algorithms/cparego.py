"""``optimobo.algorithms.cparego.ParEGO_C1`` / ``ParEGO_C2`` (cparego.py:12-874) with a device maximiser.

Constrained ParEGO (Duro et al. 2022).  Every iteration walks a shuffled set of Das-Dennis weights;
for each weight the archive is scalarised, infeasible points get a penalised fitness, at most
``N_max`` points are kept (``select_subset``) and GPs are fitted on them.  C1 maximises EI of the
scalarised model; C2 maximises EI × Π_c PoF_c with one GP per constraint
(``consraint_ei``, cparego.py:486-496).  The reference maximises with
``differential_evolution`` one candidate at a time (cparego.py:94, 544); here the same acquisition
runs as a fused device plan (omb_plan_ei / omb_plan_ei_ext kind "constrained": every posterior and
the product in one chain) over a Sobol batch.  The host bookkeeping — penalisation, subset
selection, the incumbent — follows the reference, including its quirks:

* ``xi_bar`` divides only ``min(scores)`` by the score range (operator precedence, cparego.py:322);
* the penalty is ``exp(2(s̄ + ξ̄) − 1)/(e² − 1)`` with the −1 inside the exponential (:328);
* ``select_subset`` re-evaluates the constraints of infeasible points through the problem (:109);
* ParEGO_C2 takes the *largest* scalarised value as the incumbent (``select_current_best``, :511);
* the result's ``pf_inputs`` are objective vectors, and the feasible split is the last
  iteration's (:395-403).
"""
import numpy as np

from .. import pareto
from .. import util_functions
from ..refdirs import get_reference_directions
from ..result import Constrained_Res
from ._base import BODriver


def _infeasible_mask(gsample):
    """cparego.py:270-274: a row is infeasible when any constraint value is > 0."""
    return np.asarray([bool(np.any(g > 0)) for g in np.atleast_2d(gsample)], dtype=bool)


def _penalise(aggregated, gsample, mask, feasible_pairs, infeasible_pairs, n_vars):
    """cparego.py:289-349: penalised fitness of the infeasible points (aggregated[mask])."""
    v_max = [max(col) for col in zip(*gsample)]

    def xi_single(J):
        return sum(max(v, 0) / v_max[c] for c, v in enumerate(J)) / len(J)

    workable = gsample[mask]
    scores = [xi_single(g) for g in workable]
    lo, hi = min(aggregated), max(aggregated)
    # np.any(X_feasible) in the reference: any non-zero decision variable among the feasible rows
    if np.any(feasible_pairs[:, :n_vars]):
        x_star = feasible_pairs[np.argmin(feasible_pairs[:, -1])]
    else:
        x_star = infeasible_pairs[np.argmin(scores)]
    out = []
    for row, g in zip(infeasible_pairs, workable):
        s_dot = x_star[-1] if row[-1] < x_star[-1] else row[-1]
        s_bar = (row[-1] - lo) / (hi - lo)
        if len(scores) == 1:
            xi_bar = (xi_single(g) - lo) / (hi - lo)
        else:
            xi_bar = xi_single(g) - min(scores) / (max(scores) - min(scores))
        out.append(s_dot + np.exp(2 * (s_bar + xi_bar) - 1) / (np.exp(2) - 1))
    return np.asarray(out).flatten()


class ParEGO_C1(BODriver):  # noqa: N801 — reference class name
    """ParEGO-C1: penalised scalarisation, subset selection, EI on the scalarised model."""

    _rows_have_g = False      # C1 keeps [X | y | S] rows, C2 [X | y | g | S]

    def __init__(self, test_problem, ideal_point=None, max_point=None, **kw):
        super().__init__(test_problem, ideal_point, max_point, **kw)
        self.aggregation_func = None
        self.n_eq_constr = getattr(test_problem, "n_eq_constr", 0)
        self.n_ieq_constr = getattr(test_problem, "n_ieq_constr", 0)

    def _constraint_function(self, problem, x):
        return problem.evaluate_constraints(x)

    def _xi(self, x):
        """Sum of the positive constraint values of x, re-evaluated through the problem (cparego.py:104-111)."""
        return sum(max(c, 0) for c in np.atleast_1d(self._constraint_function(self.test_problem, x)))

    def _expected_improvement(self, X, model, opt_value, kappa=0.01):
        """cparego.py:52-71 (σ = sqrt(σ²)); X (d,) → (1,), X (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        out = engine_for([model], self.device).ei(Xb, opt_value, 0.0).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def _get_proposed(self, function, models, current_best):
        """cparego.py:74-95 on the device: EI of the scalarised model → (x, −EI)."""
        from ..acquisition import engine_for
        eng = engine_for([models], self.device)
        eng.plan_ei(current_best, 0.0)
        x, v = self._maximise([models], None)
        return x, -v

    # -- subset selection (cparego.py:98-189 / 548-644)
    def _best_performing(self, X, N, ref_dir):
        X_sorted = X[X[:, -1].argsort()]
        head, tail = X_sorted[0:(N // 2)], X_sorted[(N // 2):]
        n_constr = (self.n_ieq_constr + self.n_eq_constr) if self._rows_have_g else 0
        y_end = -1 - n_constr
        deltas = [np.linalg.norm(x[self.n_vars:y_end] - ref_dir) for x in tail]
        aux = np.hstack((tail, np.reshape(deltas, (-1, 1))))
        by_delta = aux[aux[:, -1].argsort()]
        return np.vstack((head, by_delta[0:(N - N // 2)][:, :-1]))

    def select_subset(self, X_feasible, X_infeasible, ref_dir, N_max):
        x_end = self.n_vars if self._rows_have_g else -1 - self.n_obj
        scores = [self._xi(x[:x_end]) for x in X_infeasible]
        scored = np.hstack((X_infeasible, np.reshape(scores, (-1, 1))))
        by_score = scored[scored[:, -1].argsort()]
        H = N_max // 2
        nf, ni = len(X_feasible), len(X_infeasible)
        if nf + ni < N_max:
            return np.vstack((X_feasible, X_infeasible))
        if ni == 0:
            return self._best_performing(X_feasible, N_max, ref_dir)
        if nf == 0:
            first = by_score[0:H][:, :-1]
            taken = set(tuple(r) for r in first)
            rest = np.array(list(set(tuple(r) for r in X_infeasible) - taken))
            return np.vstack((first, self._best_performing(rest, N_max - len(first), ref_dir)))
        if ni >= H and nf >= H:
            head = self._best_performing(X_feasible, H, ref_dir)
            worst = by_score[0:(N_max - len(head))][:, :-1]
            return worst if len(head) == 0 else np.vstack((head, worst))
        if ni < H and nf >= H:
            return np.vstack((X_infeasible, self._best_performing(X_feasible, N_max - ni, ref_dir)))
        if ni >= H and nf < H:
            return np.vstack((X_feasible, by_score[0:(N_max - nf)][:, :-1]))
        return np.vstack((X_infeasible, X_feasible))

    # -- one weight of one iteration: scalarise, penalise, split (cparego.py:251-362 / 705-816)
    def _weight_step(self, aggregation_func, ref_dir, Xsample, ysample, gsample):
        upper = ysample.max(axis=0).astype(float)
        lower = ysample.min(axis=0).astype(float)
        aggregation_func.set_bounds(lower, upper)
        aggregated = np.asarray([aggregation_func(y, ref_dir) for y in ysample]).flatten()
        current_best = aggregated[np.argmin(aggregated)]
        mask = _infeasible_mask(gsample)
        feasible_pairs = np.hstack((Xsample[~mask], ysample[~mask], np.reshape(aggregated[~mask], (-1, 1))))
        infeasible_pairs = np.hstack((Xsample[mask], ysample[mask], np.reshape(aggregated[mask], (-1, 1))))
        if len(infeasible_pairs) > 0:
            aggregated[mask] = _penalise(aggregated, gsample, mask, feasible_pairs, infeasible_pairs, self.n_vars)
        blocks_f = [Xsample[~mask], ysample[~mask]]
        blocks_i = [Xsample[mask], ysample[mask]]
        if self._rows_have_g:
            blocks_f.append(gsample[~mask])
            blocks_i.append(gsample[mask])
        feasible_pairs = np.hstack(blocks_f + [np.reshape(aggregated[~mask], (-1, 1))])
        infeasible_pairs = np.hstack(blocks_i + [np.reshape(aggregated[mask], (-1, 1))])
        return current_best, mask, feasible_pairs, infeasible_pairs

    def _propose(self, X_prime, feasible_pairs, infeasible_pairs, current_best):
        model = self._fit(X_prime[:, :self.n_vars], X_prime[:, -1])
        next_X, _ = self._get_proposed(self._expected_improvement, model, current_best)
        return next_X

    def solve(self, aggregation_func, budget=50, n_init_samples=5, N_max=100):
        self.aggregation_func = aggregation_func
        problem = self.test_problem
        ranges = list(zip(problem.xl, problem.xu))
        Xsample = util_functions.generate_latin_hypercube_samples(n_init_samples, ranges)
        ysample = np.asarray([self._objective_function(problem, x) for x in Xsample])
        gsample = np.asarray([np.atleast_1d(self._constraint_function(problem, x)) for x in Xsample])
        ref_dirs = get_reference_directions("das-dennis", problem.n_obj, n_partitions=10)
        hypervolume_convergence = []
        n_iters = budget // len(ref_dirs)
        assert budget >= len(ref_dirs), "For " + str(self.n_obj) + " dimensions, the budget must be above " + \
            str(len(ref_dirs))
        mask = _infeasible_mask(gsample)
        for _ in range(n_iters):
            hypervolume_convergence.append(pareto.hypervolume(ysample, ysample.max(axis=0).astype(float)))
            np.random.shuffle(ref_dirs)
            for ref_dir in ref_dirs:
                current_best, mask, fp, ip = self._weight_step(aggregation_func, ref_dir, Xsample, ysample, gsample)
                X_prime = self.select_subset(fp, ip, ref_dir, N_max)
                next_X = self._propose(X_prime, fp, ip, current_best)
                next_y = self._objective_function(problem, next_X)
                ysample = np.vstack((ysample, next_y))
                Xsample = np.vstack((Xsample, next_X))
                gsample = np.vstack((gsample, np.atleast_1d(self._constraint_function(problem, next_X))))
        # the last weight step's split, as the reference reports it (cparego.py:395-403)
        n_last = len(mask)
        y_feasible, y_infeasible = ysample[:n_last][~mask], ysample[:n_last][mask]
        X_feasible, X_infeasible = Xsample[:n_last][~mask], Xsample[:n_last][mask]
        pf_approx = util_functions.calc_pf(y_feasible)
        indicies = [i for i, item in enumerate(y_feasible) if item in pf_approx]
        return Constrained_Res(y_infeasible, y_feasible, X_infeasible, X_feasible, pf_approx, y_feasible[indicies],
                               ysample, Xsample, hypervolume_convergence, problem.n_obj, n_init_samples)


class ParEGO_C2(ParEGO_C1):  # noqa: N801 — reference class name
    """ParEGO-C2: as C1, plus one GP per constraint and EI × Π PoF as the acquisition."""

    _rows_have_g = True

    def probability_of_feasibility(self, X, model):
        """cparego.py:471-484: Φ(−μ / sqrt(σ² + 1e-5)); X (d,) → (1,), X (N, d) → (N,)."""
        from scipy.stats import norm
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        mu, var = engine_for([model], self.device).posterior(Xb)
        out = norm.cdf((0 - mu[0].cpu().numpy()) / np.sqrt(var[0].cpu().numpy() + 1e-5))
        return out[:1] if np.ndim(X) == 1 else out

    def consraint_ei(self, X, aggregate_model, constraint_models, current_best):
        """cparego.py:486-496 on the device (omb_ei_ext kind "constrained"); X (d,) → (1,), (N, d) → (N,)."""
        from ..acquisition import engine_for
        Xb = np.atleast_2d(np.asarray(X, np.float64))
        eng = engine_for([aggregate_model] + list(constraint_models), self.device)
        out = eng.constrained_ei(Xb, current_best, 0.0, 1e-5).cpu().numpy()
        return out[:1] if np.ndim(X) == 1 else out

    def select_current_best(self, X_feasible, X_infeasible):
        """cparego.py:498-512 (the largest scalarised value, as the reference takes it)."""
        if len(X_feasible) == 0:
            scores = [self._xi(x[:self.n_vars]) for x in X_infeasible]
            return X_infeasible[int(np.argmax(scores))][-1]
        return X_feasible[int(np.argmax(X_feasible[:, -1]))][-1]

    def xi(self, x):
        return self._xi(x)

    def _get_proposed(self, function, models, constraint_models, current_best):
        from ..acquisition import engine_for
        eng = engine_for([models] + list(constraint_models), self.device)
        eng.plan_constrained_ei(current_best, 0.0, 1e-5)
        x, v = self._maximise([models] + list(constraint_models), None)
        return x, -v

    def _propose(self, X_prime, feasible_pairs, infeasible_pairs, current_best):
        model_input = X_prime[:, :self.n_vars]
        agg_model = self._fit(model_input, X_prime[:, -1])
        constraints = X_prime[:, self.n_vars + self.n_obj:-1]
        constraint_models = [self._fit(model_input, constraints[:, i])
                             for i in range(self.n_eq_constr + self.n_ieq_constr)]
        best = self.select_current_best(feasible_pairs, infeasible_pairs)
        next_X, _ = self._get_proposed(self.consraint_ei, agg_model, constraint_models, best)
        return next_X
