"""The bench's own workloads (bench.py CONFIGS 2, 3 and 5, built by bench.setup_problem) through the fused
chain bench.py times (omb_eval_argmax): the arg-max is an interior candidate (not Sobol index 0, where the
unexplored corner x = 0 and the lowest-index tie rule both land), positive and unique, equal to the arg-max
of the device values, and the oracle chain over the device's 256 best candidates picks the same one at the
same value (1e-5 relative, north_star's acquisition tolerance)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import bench  # noqa: E402
from oracle import acquisition as oacq  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import pareto as opar  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    from optimobo_amd.device import AcqContext
    c = AcqContext(0)
    yield c
    c.close()


@pytest.mark.parametrize("config", [2, 3, 5])
def test_bench_workload_interior_argmax(ctx, config):
    from optimobo_amd import pareto
    from optimobo_amd import scalarisations as sc
    from optimobo_amd.gp import GPState
    cfg = bench.CONFIGS[config]
    n, d, N = cfg["n"], cfg["d"], 1 << cfg["log2"]
    X, Y, ls, variances = bench.setup_problem(n, d, problem=cfg["problem"], tail_hi=cfg["tail_hi"])
    if cfg["acq"] == "ei_tch":
        tch = sc.Tchebicheff(Y.min(axis=0), Y.max(axis=0))
        T = tch(Y, np.array([0.5, 0.5]))[:, None]
        Tvar = [float(np.var(T))]
        best_y = float(T.min())
        ctx.set_gp_state(0, GPState(X, T[:, 0], ls, Tvar[0]))
        ctx.plan_ei(best_y, 1e-6)
    else:
        T, Tvar = Y, variances
        for o in range(2):
            ctx.set_gp_state(o, GPState(X, Y[:, o], ls, variances[o]))
        pf = opar.calc_pf(Y)
        r = Y.max(axis=0) + 0.1 * (Y.max(axis=0) - Y.min(axis=0))
        cache = pareto.cached_samples(2, 5, seed=1)
        s00, s01 = pareto.cache_stats(cache)
        assert s01 > 0
        ctx.plan_ehvi2d(pareto.stripes_2d(pf), r, s00, s01, mode="reference")
    Xc = bench.candidates(d, 0, N)
    Xd = torch.as_tensor(Xc, device="cuda:0")
    pair = ctx.eval_argmax(Xd, offset=0).cpu().numpy()
    vals = ctx.eval(Xd).cpu().numpy()
    ov, oi = oacq.argmax(vals)
    assert (pair[0], int(pair[1])) == (ov, oi)
    assert oi != 0 and ov > 0 and np.count_nonzero(vals == ov) == 1, (oi, ov)
    top = np.argsort(-vals, kind="stable")[:256]
    mus, vs = [], []
    for o in range(T.shape[1]):
        m, v = ogp.ExactGP(X, T[:, o], ls, Tvar[o]).predict(Xc[top])
        mus.append(m[:, 0])
        vs.append(v[:, 0])
    mus, vs = np.array(mus), np.array(vs)
    if cfg["acq"] == "ei_tch":
        ref = oacq.ei(mus[0], vs[0], best_y, 1e-6)
    else:
        ref = oacq.ehvi2d(mus, vs, pf, r, cache, mode="reference")
    np.testing.assert_allclose(vals[top], ref, rtol=1e-5, atol=1e-12)
    assert top[int(np.argmax(ref))] == oi
