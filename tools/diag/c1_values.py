"""Diagnostic (GPU box): README run; at 5 iterations compare the device posterior at the proposal with the
oracle's, and report cond(Ky)."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import optimobo_amd.algorithms.optimisers as opti
import optimobo_amd.scalarisations as sc
from optimobo_amd.problem import ElementwiseProblem
from oracle import gp as ogp, acquisition as oacq, scalarisations as osc


class MyProblem(ElementwiseProblem):
    def __init__(self):
        super().__init__(n_var=2, n_obj=2, xl=np.array([-2, -2]), xu=np.array([2, 2]))

    def _evaluate(self, x, out, *a, **k):
        out["F"] = [100 * (x[0] ** 2 + x[1] ** 2), (x[0] - 1) ** 2 + x[1] ** 2]


np.random.seed(0)
opt = opti.MultiSurrogateOptimiser(MyProblem(), [0, 0], [700, 12], seed=1)
orig = opt._get_proposed_scalarisation
it = [0]
tch = osc.Tchebicheff(np.array([0.0, 0.0]), np.array([700.0, 12.0]))


def rec(function, models, min_val, scalar_func, ref_dir, cache):
    x, negv, rd = orig(function, models, min_val, scalar_func, ref_dir, cache)
    if it[0] % 12 == 0 or it[0] == 99:
        from optimobo_amd.acquisition import engine_for
        eng = engine_for(models)
        dm, dv = [], []
        for o, m in enumerate(models):
            mu, var = m.predict(x[None, :])
            dm.append(mu[0, 0]); dv.append(var[0, 0])
        gps = [ogp.ExactGP(models[0].X, m.Y[:, 0], m.kern.ls_vector(), float(m.kern.variance)) for m in models]
        om = [g.predict(x[None, :]) for g in gps]
        K = [g.K if hasattr(g, "K") else None for g in gps]
        conds = []
        for g, m in zip(gps, models):
            from oracle.gp import matern52_K
            try:
                Kx = matern52_K(models[0].X, models[0].X, m.kern.ls_vector(), float(m.kern.variance))
                conds.append(float(np.linalg.cond(Kx + 1e-8 * np.eye(len(Kx)))))
            except Exception as e:
                conds.append(str(e))
        mu_o = np.array([o[0][0, 0] for o in om]); var_o = np.array([o[1][0, 0] for o in om])
        v_o = oacq.expected_decomposition(mu_o[:, None], var_o[:, None], np.array(cache), tch, np.asarray(ref_dir), float(min_val))[0]
        print(f"it {it[0]} n {len(models[0].X)} v_dev {-negv:.6e} v_oracle {v_o:.6e} mu_dev {dm} mu_o {mu_o.tolist()} "
              f"var_dev {dv} var_o {var_o.tolist()} ls {[m.kern.ls_vector().tolist() for m in models]} "
              f"sf2 {[float(m.kern.variance) for m in models]} cond {conds}", flush=True)
    it[0] += 1
    return x, negv, rd


opt._get_proposed_scalarisation = rec
res = opt.solve(budget=100, n_init_samples=20, sample_exponent=3, acquisition_func=sc.Tchebicheff([0, 0], [700, 12]))
