"""CPU restatement of the ParEGO / KEEP evolutionary acquisition search — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, as the checker.

Follows ParEGO.solve's search loop (parego.py:238-269) with its operators (mutate :37-56,
simulated_binary_crossover :58-75, parego_binary_tournament_selection_without_replacment :78-111) and
KEEP's (keep.py:256-290, :73-104, fitness pareto_expected_improvement :142-151).  The random draws come
from a tape (optimobo_amd.ea.ea_tape replays the reference's np.random / random calls).  Pinned against
the reference's own solve() through tests/golden/ea.npz (tests/golden/make_golden.py make_ea).
"""
import numpy as np


def search(pop0, fitness, tape, lower, upper, alias=True):
    """→ (best_x, best_fitness).  fitness(X (m, d)) → (m,).

    The reference keeps ``best_solution_found = temporary_population[np.argmax(EIs)]``, a numpy *view*
    of a population row (parego.py:248-251, keep.py:268-271), so a later
    ``temporary_population[parent1_idx] = final`` into that row (:270 / :292) changes the proposal it
    returns.  The search therefore tracks the best row's *index* and reads the row after the last
    generation (``lower`` if no generation improved on best_EI = 0).  ``alias=False`` keeps a copy of the
    row instead; it exists only so tests/golden/make_golden.py can find runs where the two differ.
    """
    pop = np.array(pop0, np.float64, copy=True)
    lower = np.asarray(lower, np.float64)
    upper = np.asarray(upper, np.float64)
    F = np.asarray(fitness(pop), np.float64).reshape(-1)
    best_f, best_row, best_copy = 0.0, -1, lower.copy()  # best_EI = 0, best_solution_found = self.lower
    for it in range(tape.iters):
        fmax = np.max(F)                               # NaN if any fitness is NaN (np.max propagates it)
        if fmax > best_f:
            best_f, best_row = fmax, int(np.argmax(F))   # argmax: the first maximum
            best_copy = pop[best_row].copy()
        s = tape.sel[it]
        w1 = s[0] if F[s[0]] > F[s[1]] else s[1]       # tournament 1 over the whole population
        a = s[2] if s[2] < w1 else s[2] + 1            # tournament 2 over the population without w1
        b = s[3] if s[3] < w1 else s[3] + 1
        w2 = a if F[a] > F[b] else b
        p1, p2 = pop[w1], pop[w2]
        if tape.cross[it]:
            beta = tape.beta[it]
            child = np.clip(0.5 * ((1 + beta) * p1 + (1 - beta) * p2), lower, upper)
        else:
            child = p1.copy()
        m = tape.mut[it]
        child = np.where(m == 1, child * 1.05, np.where(m == 2, child * 0.95, child))
        child = np.clip(child, lower, upper)
        fc = float(np.asarray(fitness(child[None, :])).reshape(-1)[0])
        if not F[w1] > fc:                             # the parent stays only if strictly better
            pop[w1] = child
            F[w1] = fc
    if not alias:
        return best_copy, best_f
    return (pop[best_row].copy() if best_row >= 0 else lower.copy()), best_f


def ei_fitness(gp, best, var_eps=1e-6):
    """ParEGO._expected_improvement (parego.py:126-145) over rows of X."""
    from .acquisition import ei

    def f(X):   # one point per predict, as the reference calls it (batched BLAS may round differently)
        out = []
        for x in np.atleast_2d(X):
            mu, var = gp.predict(x[None, :])
            out.append(ei(mu[:, 0], var[:, 0], best, var_eps)[0])
        return np.array(out)
    return f


def pareto_ei_fitness(scalar_gp, pareto_gp, best, var_eps=1e-6):
    """KEEP.pareto_expected_improvement (keep.py:142-151): μ_pareto · EI_scalar."""
    from .acquisition import ei

    def f(X):
        out = []
        for x in np.atleast_2d(X):
            mu0, var0 = scalar_gp.predict(x[None, :])
            mu1, _ = pareto_gp.predict(x[None, :])
            out.append(mu1[0, 0] * ei(mu0[:, 0], var0[:, 0], best, var_eps)[0])
        return np.array(out)
    return f
