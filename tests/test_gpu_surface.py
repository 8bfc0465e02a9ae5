"""GPU tests of the drop-in surface: reference-signature acquisition calls (one candidate and
batches) against the oracle chain, and short solve() runs of every driver."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import acquisition as oacq  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import pareto as opar  # noqa: E402


def zdt1(X):
    f1 = X[:, 0]
    g = 1 + 9.0 / (X.shape[1] - 1) * X[:, 1:].sum(1)
    return np.column_stack([f1, g * (1 - np.sqrt(f1 / g))])


@pytest.fixture(scope="module")
def fitted():
    from optimobo_amd.gp import GPRegression, Matern52
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 1, (48, 4))
    Y = zdt1(X)
    ls = np.array([0.4, 0.8, 1.1, 1.5])
    models = []
    for o in range(2):
        m = GPRegression(X, Y[:, o:o + 1], Matern52(4, variance=float(np.var(Y[:, o])), lengthscale=ls, ARD=True))
        m.Gaussian_noise.variance.fix(0)
        models.append(m)
    return X, Y, ls, models


def oracle_moments(X, Y, ls, Xc):
    mus, vs = [], []
    for o in range(2):
        m, v = ogp.ExactGP(X, Y[:, o], ls, float(np.var(Y[:, o]))).predict(Xc)
        mus.append(m[:, 0])
        vs.append(v[:, 0])
    return np.array(mus), np.array(vs)


def test_predict_matches_oracle(fitted):
    X, Y, ls, models = fitted
    Xc = np.random.default_rng(0).uniform(0, 1, (300, 4))
    mu, var = models[1].predict(Xc)
    mo, vo = oracle_moments(X, Y, ls, Xc)
    np.testing.assert_allclose(mu[:, 0], mo[1], rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(var[:, 0], vo[1], rtol=1e-6, atol=1e-10)
    assert mu.shape == (300, 1) and var.shape == (300, 1)


@pytest.mark.parametrize("mode", ["reference", "textbook"])
def test_util_ehvi_single_and_batch(fitted, mode):
    import optimobo_amd.util_functions as uf
    X, Y, ls, models = fitted
    pf = opar.calc_pf(Y)
    r = Y.max(0) + 0.1
    cache = np.random.default_rng(1).standard_normal((32, 2))
    Xc = np.random.default_rng(2).uniform(0, 1, (257, 4))
    batch = uf.EHVI(Xc, models, r, pf, cache, mode=mode)
    one = uf.EHVI(Xc[5], models, r, pf, cache, mode=mode)
    assert one.shape == (1,) and batch.shape == (257,)
    mo, vo = oracle_moments(X, Y, ls, Xc)
    ref = oacq.ehvi2d(mo, vo, pf, r, cache, mode=mode)
    np.testing.assert_allclose(batch, ref, rtol=1e-5, atol=1e-10)
    assert one[0] == pytest.approx(batch[5], rel=1e-14)


def test_util_ehvi_2d_aux_sigma(fitted):
    import optimobo_amd.util_functions as uf
    pf = np.array([[0.1, 0.9], [0.4, 0.5], [0.8, 0.1]])
    r = np.array([1.0, 1.0])
    mu = np.array([0.3, 0.4])
    cov = np.array([[0.04, -0.01], [-0.01, 0.02]])
    got = uf.EHVI_2D_aux(pf, r, mu, cov)
    ref = oacq.ehvi2d_aux(pf, r, mu[:1], mu[1:], np.array([0.04]), np.array([-0.01]))
    np.testing.assert_allclose(got, ref, rtol=1e-12)


def test_util_expdec_and_ehvi3d(fitted):
    import optimobo_amd.scalarisations as sc
    import optimobo_amd.util_functions as uf
    from oracle import scalarisations as osc
    X, Y, ls, models = fitted
    Xc = np.random.default_rng(4).uniform(0, 1, (100, 4))
    cache = np.random.default_rng(5).standard_normal((8, 2))
    w = np.array([0.3, 0.7])
    s = sc.Tchebicheff(Y.min(0), Y.max(0))
    agg_min = float(np.min(s(Y, w)))
    got = uf.expected_decomposition(Xc, models, w, s, agg_min, cache)
    mo, vo = oracle_moments(X, Y, ls, Xc)
    ref = oacq.expected_decomposition(mo, vo, cache, osc.Tchebicheff(Y.min(0), Y.max(0)), w, agg_min)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-12)
    assert isinstance(uf.expected_decomposition(Xc[0], models, w, s, agg_min, cache), float)


def _myproblem():
    from optimobo_amd.problem import ElementwiseProblem

    class MyProblem(ElementwiseProblem):        # README.md:28-39
        def __init__(self):
            super().__init__(n_var=2, n_obj=2, xl=np.array([-2, -2]), xu=np.array([2, 2]))

        def _evaluate(self, x, out, *args, **kwargs):
            out["F"] = [100 * (x[0] ** 2 + x[1] ** 2), (x[0] - 1) ** 2 + x[1] ** 2]
    return MyProblem()


def test_solve_multi_surrogate_tchebicheff():
    import optimobo_amd.algorithms.optimisers as opti
    import optimobo_amd.scalarisations as sc
    np.random.seed(0)
    opt = opti.MultiSurrogateOptimiser(_myproblem(), [0, 0], [700, 12], n_candidates=4096, seed=1)
    out = opt.solve(budget=4, n_init_samples=10, sample_exponent=3, acquisition_func=sc.Tchebicheff([0, 0], [700, 12]))
    assert out.ysample.shape == (14, 2) and out.Xsample.shape == (14, 2)
    assert len(out.hypervolume_convergence) == 4
    assert np.all(np.diff(out.hypervolume_convergence) >= -1e-12)
    assert np.all(np.abs(out.Xsample) <= 2 + 1e-12)


@pytest.mark.parametrize("mode", ["reference", "textbook"])
def test_solve_multi_surrogate_ehvi(mode):
    import optimobo_amd.algorithms.optimisers as opti
    np.random.seed(1)
    opt = opti.MultiSurrogateOptimiser(_myproblem(), [0, 0], [700, 12], mode=mode, n_candidates=4096, seed=2)
    out = opt.solve(budget=3, n_init_samples=8)
    assert out.ysample.shape == (11, 2) and out.pf_approx.shape[1] == 2


def test_solve_mono_emo_parego():
    from optimobo_amd.algorithms import EMO, MonoSurrogateOptimiser, ParEGO
    import optimobo_amd.scalarisations as sc
    np.random.seed(2)
    p = _myproblem()
    r1 = MonoSurrogateOptimiser(p, [0, 0], [700, 12], n_candidates=2048, seed=3).solve(
        sc.Tchebicheff([0, 0], [700, 12]), budget=2, n_init_samples=8)
    r2 = EMO(p, [0, 0], [700, 12], n_candidates=2048, seed=4).solve(budget=2, n_init_samples=8)
    # the evolutionary search (the reference's) samples 10 archive members: n_init ≥ 10, as in the reference
    r3 = ParEGO(p, [0, 0], [700, 12], n_candidates=2048, seed=5).solve(sc.Tchebicheff([0, 0], [700, 12]), budget=2,
                                                                        n_init_samples=10)
    for r in (r1, r2):
        assert r.ysample.shape == (10, 2)
    assert r3.ysample.shape == (12, 2) and np.all(np.abs(r3.Xsample) <= 2 + 1e-12)
    r4 = ParEGO(p, [0, 0], [700, 12], n_candidates=2048, seed=5)
    r4.acq_search = "batch"
    assert r4.solve(sc.Tchebicheff([0, 0], [700, 12]), budget=2, n_init_samples=8).ysample.shape == (10, 2)


def test_keep_solve_and_fitness(fitted):
    from optimobo_amd.algorithms import KEEP
    import optimobo_amd.scalarisations as sc
    np.random.seed(3)
    p = _myproblem()
    keep = KEEP(p, [0, 0], [700, 12], n_candidates=2048, seed=6)
    r = keep.solve(sc.Tchebicheff([0, 0], [700, 12]), budget=2, n_init_samples=10)
    assert r.ysample.shape == (12, 2) and np.all(np.abs(r.Xsample) <= 2 + 1e-12)
    # the fitness KEEP maximises, batched and single, against the oracle chain
    X, Y, ls, models = fitted
    Xc = np.random.default_rng(4).uniform(0, 1, (500, 4))
    got = keep.pareto_expected_improvement(Xc, models[1], models[0], 0.3)
    mo, vo = oracle_moments(X, Y, ls, Xc)
    ref = oacq.pareto_ei(mo, vo, 0.3)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-12)
    one = keep.pareto_expected_improvement(Xc[7], models[1], models[0], 0.3)
    assert one.shape == (1,) and one[0] == pytest.approx(ref[7], rel=1e-6, abs=1e-12)


def test_cparego_c1_c2_solve():
    """Constrained ParEGO end to end: device fit, device EI / EI·PoF plans, Constrained_Res."""
    from optimobo_amd.algorithms import ParEGO_C1, ParEGO_C2
    from optimobo_amd.problem import ElementwiseProblem
    import optimobo_amd.scalarisations as sc

    class BNH(ElementwiseProblem):          # optimobo/problem.py BNH demo, 2 inequality constraints
        def __init__(self):
            super().__init__(n_var=2, n_obj=2, n_ieq_constr=2, xl=np.array([0.0, 0.0]), xu=np.array([5.0, 3.0]))

        def _evaluate(self, x, out, *args, **kwargs):
            out["F"] = [4 * x[0] ** 2 + 4 * x[1] ** 2, (x[0] - 5) ** 2 + (x[1] - 5) ** 2]

        def _evaluate_constraints(self, x, out, *args, **kwargs):
            out["G"] = [(x[0] - 5) ** 2 + x[1] ** 2 - 9.0, 7.7 - (x[0] - 8) ** 2 - (x[1] + 3) ** 2]

    for cls in (ParEGO_C1, ParEGO_C2):
        np.random.seed(4)
        r = cls(BNH(), n_candidates=2048, seed=9).solve(sc.Tchebicheff(), budget=11, n_init_samples=8, N_max=10)
        assert r.ysample.shape == (19, 2) and r.Xsample.shape == (19, 2)
        assert np.all((r.Xsample >= 0) & (r.Xsample <= np.array([5.0, 3.0]) + 1e-12))
        assert len(r.X_feasible) + len(r.X_infeasible) == 18    # the last weight step's split
        assert len(r.hypervolume_convergence) == 1


def test_cparego_constraint_ei_matches_oracle(fitted):
    """ParEGO_C2.consraint_ei (cparego.py:486-496) on the device against the oracle chain."""
    from optimobo_amd.algorithms import ParEGO_C2
    X, Y, ls, models = fitted
    Xc = np.random.default_rng(11).uniform(0, 1, (400, 4))
    c2 = object.__new__(ParEGO_C2)
    c2.device = None
    got = c2.consraint_ei(Xc, models[0], [models[1]], 0.2)
    mo, vo = oracle_moments(X, Y, ls, Xc)
    ref = oacq.constrained_ei(mo, vo, 0.2)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-12)
