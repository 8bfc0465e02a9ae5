"""ParEGO / KEEP evolutionary acquisition search, host side.

Pins the tape generator (optimobo_amd.ea.ea_tape, replaying the reference's np.random / random calls)
and the oracle's restatement of the search loop (oracle/ea.py) against the reference's own solve():
tests/golden/ea.npz holds, per case, the temporary population and both generators' states at the start
of the search and the proposal the reference's 1,000-generation search returned (make_golden.py
make_ea; GPy's default hyperparameters through the oracle's GPy restatement).  Bit-exact.
"""
import os
import random

import numpy as np
import pytest

from oracle import ea as oea
from oracle import gp as ogp
from optimobo_amd import ea


def _case(z, c):
    k = f"c{c}"
    return {key[len(k) + 1:]: z[key] for key in z.files if key.startswith(k + "_")}


def _restore(cs):
    np.random.set_state(("MT19937", cs["np_keys"], int(cs["np_pos"]), int(cs["np_has_gauss"]), float(cs["np_gauss"])))
    random.setstate((int(cs["py_version"]), tuple(int(v) for v in cs["py_state"]), None))


def fitness_for(cs):
    X = cs["X"]
    scalar = ogp.ExactGP(X, cs["y0"], 1.0, 1.0)
    if str(cs["kind"]) == "parego":
        return oea.ei_fitness(scalar, float(cs["best"]))
    return oea.pareto_ei_fitness(scalar, ogp.ExactGP(X, cs["y1"], 1.0, 1.0), float(cs["best"]))


@pytest.fixture(scope="module")
def ea_golden(golden_dir):
    return np.load(os.path.join(golden_dir, "ea.npz"), allow_pickle=False)


N_CASES = 6      # tests/golden/ea.npz: 4 fixed seeds + one aliasing ParEGO and one aliasing KEEP run


def test_golden_has_alias_cases(ea_golden):
    assert int(ea_golden["n_cases"]) == N_CASES
    kinds = [str(ea_golden[f"c{c}_kind"]) for c in range(N_CASES) if int(ea_golden[f"c{c}_alias"])]
    assert sorted(kinds) == ["keep", "parego"]


@pytest.mark.parametrize("c", range(N_CASES))
def test_oracle_search_matches_reference(ea_golden, c):
    """The reference returns a view of the best row (parego.py:248-251, keep.py:268-271): in the alias
    cases the row was replaced after it was recorded, and a copy of it would be the wrong proposal."""
    cs = _case(ea_golden, c)
    d = int(cs["d"])
    _restore(cs)
    tape = ea.ea_tape(len(cs["pop"]), d)
    x, f = oea.search(cs["pop"], fitness_for(cs), tape, cs["lower"], cs["upper"])
    np.testing.assert_array_equal(x, cs["next_x"])
    if int(cs["alias"]):
        assert not np.array_equal(cs["next_x_if_copied"], cs["next_x"])


def test_tape_shapes_and_codes():
    rs = np.random.RandomState(5)
    tape = ea.ea_tape(20, 4, iters=300, nprand=rs, pyrand=random.Random(5))
    assert tape.sel.shape == (300, 4) and tape.beta.shape == (300, 4) and tape.mut.shape == (300, 4)
    assert tape.sel[:, :2].min() >= 1 and tape.sel[:, :2].max() <= 19
    assert tape.sel[:, 2:].min() >= 1 and tape.sel[:, 2:].max() <= 18
    assert np.all(tape.sel[:, 0] != tape.sel[:, 1]) and np.all(tape.sel[:, 2] != tape.sel[:, 3])
    assert set(np.unique(tape.mut)) <= {0, 1, 2}
    assert 0.1 < tape.cross.mean() < 0.3                       # crossover probability 0.2
    assert np.all(tape.beta[tape.cross == 0] == 0)


def test_initial_population_follows_reference_draws():
    """Mutants of 10 archive members then 10 Latin-hypercube points (parego.py:229-235), bounded."""
    rs = np.random.RandomState(7)
    X = rs.uniform(0, 1, (15, 3))
    pop = ea.initial_population(X, np.zeros(3), np.ones(3), nprand=np.random.RandomState(8), pyrand=random.Random(8))
    assert pop.shape == (20, 3) and np.all((pop >= 0) & (pop <= 1))


def test_batch_fallback_warns_once():
    """Above EA_MAX_TRAIN the drivers leave the reference's search: one RuntimeWarning per process."""
    import warnings
    from optimobo_amd import ea
    ea._FALLBACK_WARNED[0] = False
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        ea.warn_batch_fallback("ParEGO", ea.EA_MAX_TRAIN + 1)
        ea.warn_batch_fallback("KEEP", ea.EA_MAX_TRAIN + 5)
    assert len(rec) == 1 and issubclass(rec[0].category, RuntimeWarning)
    assert "random streams" in str(rec[0].message)
