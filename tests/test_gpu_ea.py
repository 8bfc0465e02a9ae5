"""GPU: the ParEGO / KEEP evolutionary acquisition search (omb_ea_search) against the
reference's own solve() (tests/golden/ea.npz, make_golden.py make_ea) and the oracle's restatement.
Cases 4 and 5 are runs where the reference's proposal is a view of a population row that was replaced
after it was recorded (parego.py:248-251 / :270, keep.py:268-271 / :292).

With both generators restored to the reference's state at the start of the search, the host tape
(optimobo_amd.ea.ea_tape) plus the device search must return the reference's proposal exactly; the best
fitness agrees with the oracle's to 1e-12 relative (the device computes the same fitness in a different
summation order).
"""
import os
import random

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import ea as oea  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from test_ea import N_CASES, _case, _restore, fitness_for  # noqa: E402


@pytest.fixture(scope="module")
def ea_golden(golden_dir):
    return np.load(os.path.join(golden_dir, "ea.npz"), allow_pickle=False)


def _ctx_for(cs):
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState
    ctx = AcqContext(0)
    X = cs["X"]
    ctx.set_gp_state(0, GPState(X, cs["y0"], np.ones(X.shape[1]), 1.0))
    if str(cs["kind"]) == "keep":
        ctx.set_gp_state(1, GPState(X, cs["y1"], np.ones(X.shape[1]), 1.0))
    return ctx


@pytest.mark.parametrize("c", range(N_CASES))
def test_device_search_matches_reference(ea_golden, c):
    from optimobo_amd import ea
    cs = _case(ea_golden, c)
    _restore(cs)
    tape = ea.ea_tape(len(cs["pop"]), int(cs["d"]))
    ctx = _ctx_for(cs)
    mode = 0 if str(cs["kind"]) == "parego" else 1
    x, f = ctx.ea_search(cs["pop"], tape, float(cs["best"]), cs["lower"], cs["upper"], mode=mode)
    np.testing.assert_array_equal(x, cs["next_x"])
    _, f_o = oea.search(cs["pop"], fitness_for(cs), tape, cs["lower"], cs["upper"])
    assert abs(f - f_o) <= 1e-12 * abs(f_o) + 1e-300
    ctx.close()


def test_device_search_random_tapes_match_oracle():
    """Fresh surrogates and tapes (several seeds, d = 3 and 7, n = 40 and 150): the device search and the
    oracle's make the same choices."""
    from optimobo_amd import ea
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState
    for seed, d, n in [(11, 3, 40), (12, 7, 150), (13, 5, 90), (14, 100, 60), (15, 256, 30)]:
        rng = np.random.default_rng(seed)
        X = rng.uniform(0, 1, (n, d))
        y = np.sin(4 * X).sum(1) + X[:, 0]
        ls = rng.uniform(0.3, 1.2, d)
        var = float(np.var(y))
        ctx = AcqContext(0)
        ctx.set_gp_state(0, GPState(X, y, ls, var))
        lower, upper = np.zeros(d), np.ones(d)
        pop = ea.initial_population(X, lower, upper, nprand=np.random.RandomState(seed), pyrand=random.Random(seed))
        tape = ea.ea_tape(len(pop), d, iters=400, nprand=np.random.RandomState(seed + 1), pyrand=random.Random(seed + 1))
        best = float(y.min())
        x, f = ctx.ea_search(pop, tape, best, lower, upper)
        gp = ogp.ExactGP(X, y, ls, var)
        x_o, f_o = oea.search(pop, oea.ei_fitness(gp, best), tape, lower, upper)
        np.testing.assert_array_equal(x, x_o)
        assert abs(f - f_o) <= 1e-12 * abs(f_o)
        ctx.close()


def test_search_argument_checks():
    from optimobo_amd import _lib, ea
    from optimobo_amd._lib import OMBError
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState
    rng = np.random.default_rng(3)
    X = rng.uniform(0, 1, (20, 2))
    ctx = AcqContext(0)
    ctx.set_gp_state(0, GPState(X, X.sum(1), np.ones(2), 1.0))
    tape = ea.ea_tape(20, 2, iters=5, nprand=np.random.RandomState(1), pyrand=random.Random(1))
    with pytest.raises(ValueError):
        ctx.ea_search(np.zeros((20, 3)), tape, 0.0, np.zeros(3), np.ones(3))          # wrong width
    bad = ea.EATape(np.full((5, 4), 19, np.int32), tape.cross, tape.beta, tape.mut)
    with pytest.raises(ValueError):
        ctx.ea_search(np.zeros((20, 2)), bad, 0.0, np.zeros(2), np.ones(2))           # second-tournament range
    with pytest.raises(OMBError) as e:
        ctx.ea_search(np.zeros((40, 2)), ea.ea_tape(40, 2, iters=1, nprand=np.random.RandomState(2),
                                                     pyrand=random.Random(2)), 0.0, np.zeros(2), np.ones(2))
    assert e.value.code == _lib.OMB_EINVAL                                              # P > 32
    with pytest.raises(OMBError) as e:
        ctx.ea_search(np.zeros((20, 2)), tape, 0.0, np.zeros(2), np.ones(2), mode=1)  # objective 1 not set
    assert e.value.code == _lib.OMB_ESTATE
    ctx.close()
