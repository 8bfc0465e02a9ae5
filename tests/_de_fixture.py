"""The reference maximisers' DE proposals (tests/golden/de_proposals.npz, make_golden.py make_de_proposals):
the acquisition of each case restated by the oracle (test infrastructure)."""
import numpy as np

from oracle import acquisition as oacq
from oracle import gp as ogp
from oracle import scalarisations as osc

N_CASES = 14


def oracle_value(z, k, kind, x):
    """The reference arithmetic (oracle restatement) of the fixture's acquisition at x."""
    X, Y, ls, var = z[f"{k}_X"], z[f"{k}_Y"], z[f"{k}_ls"], z[f"{k}_variances"]
    if kind == "ei":
        m, s2 = ogp.ExactGP(X, z[f"{k}_yagg"], ls, float(z[f"{k}_agg_variance"])).predict(x[None, :])
        return oacq.ei(m[:, 0], s2[:, 0], float(z[f"{k}_best"]), 0.0)[0]
    mus, vs = [], []
    for o in range(Y.shape[1]):
        m, s2 = ogp.ExactGP(X, Y[:, o], ls, float(var[o])).predict(x[None, :])
        mus.append(m[:, 0])
        vs.append(s2[:, 0])
    mu, v = np.array(mus), np.array(vs)
    if kind == "ehvi":
        return oacq.ehvi2d(mu, v, z[f"{k}_pf"], z[f"{k}_r"], z[f"{k}_cache"])[0]
    if kind == "ehvi3d":
        from oracle import pareto as opar
        val, raised = oacq.ehvi3d_reference(mu, v, opar.hypervolume(z[f"{k}_pf"], z[f"{k}_r"]), z[f"{k}_r"],
                                            z[f"{k}_cache"])
        return np.nan if raised[0] else val[0]
    if kind == "hvpoi":
        return oacq.hvpoi(mu, v, z[f"{k}_cells"])[0]
    return oacq.expected_decomposition(mu, v, z[f"{k}_cache"], osc.Tchebicheff(z[f"{k}_ideal"], z[f"{k}_max"]),
                                       z[f"{k}_w"], float(z[f"{k}_agg_min"]))[0]


