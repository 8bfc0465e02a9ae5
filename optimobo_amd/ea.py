"""ParEGO / KEEP evolutionary acquisition search — host side.

The reference maximises its acquisition with a steady-state genetic algorithm (ParEGO.solve,
parego.py:223-271; KEEP.solve, keep.py:240-292): a temporary population of 20 (10 mutants of archive
members + 10 Latin-hypercube points), then 1,000 generations of

    track the population's best fitness (before the generation's change),
    two binary tournaments without replacement (random.sample(range(1, len(pop)), 2); the first
        winner is removed before the second tournament)             parego.py:78-111
    simulated binary crossover with probability 0.2, η = 2 (one child, clipped)   parego.py:58-75
    per-gene mutation with probability 1/d (×1.05 or ×0.95), clipped            parego.py:37-56
    the child replaces the first parent unless the parent's fitness is strictly greater.

Fitness: ParEGO's EI with σ = sqrt(σ² + 1e-6) (parego.py:126-145); KEEP's μ_pareto · EI
(keep.py:142-151).  No random draw depends on a fitness value, so the draws can be replayed on the
host, in the reference's call order, into a *tape* (`ea_tape`), and the 1,000 generations then run
in one device workgroup (`omb_ea_search`), which evaluates only the child's fitness per generation
(the population's fitness is cached: the reference recomputes the same values every generation).
With the generators in the reference's state, the device search returns the reference's proposal.
"""
import random
import warnings

import numpy as np

EA_POP = 20              # 10 mutants + 10 Latin-hypercube points (parego.py:230-235)
EA_ITERS = 1000          # n_remutations (parego.py:241)
EA_ETA = 2.0             # parego.py:226
EA_CROSS_PROB = 0.2      # simulated_binary_crossover(..., crossover_prob=0.2) (parego.py:259)
EA_MAX_TRAIN = 2048      # omb_ea_search keeps one K* row in LDS (kEAMaxTrain, omb_internal.h)


def device_search_fits(n_train):
    """True when omb_ea_search takes a surrogate of `n_train` points; the drivers use the batched
    device arg-max of the same fitness above that (omb_ea_search returns OMB_EUNSUP there)."""
    return int(n_train) <= EA_MAX_TRAIN


_FALLBACK_WARNED = [False]


def warn_batch_fallback(driver, n_train):
    """Once per process: above EA_MAX_TRAIN the drivers maximise with the batched Sobol arg-max instead of the
    reference's evolutionary search (parego.py:223-271, keep.py:240-292), which makes none of its
    ``random.sample`` / numpy draws, so the host random streams depart from the reference's from then on."""
    if not _FALLBACK_WARNED[0]:
        _FALLBACK_WARNED[0] = True
        warnings.warn(f"{driver}: {n_train} training points exceed the device evolutionary search's {EA_MAX_TRAIN}; "
                      "using the batched arg-max of the same fitness instead, so the host random streams no "
                      "longer follow the reference's", RuntimeWarning, stacklevel=3)


class EATape:
    """Random draws of `iters` generations.

    sel   (iters, 4) int32: the two tournaments' random.sample pairs — the first over range(1, P),
          the second over range(1, P − 1), i.e. indices into the population without the first winner;
    cross (iters,) int8: 1 when the crossover happens (np.random.rand() ≤ crossover_prob);
    beta  (iters, d) float64: the crossover's β per gene (numpy's expression, so bit-identical);
    mut   (iters, d) int8: 0 no mutation, 1 ×1.05, 2 ×0.95.
    """

    def __init__(self, sel, cross, beta, mut):
        self.sel = np.ascontiguousarray(sel, np.int32)
        self.cross = np.ascontiguousarray(cross, np.int8)
        self.beta = np.ascontiguousarray(beta, np.float64)
        self.mut = np.ascontiguousarray(mut, np.int8)

    @property
    def iters(self):
        return len(self.cross)


def ea_tape(P, d, iters=EA_ITERS, mutation_rate=None, crossover_prob=EA_CROSS_PROB, eta=EA_ETA,
            nprand=np.random, pyrand=random):
    """Replay the search's draws from `nprand` (numpy's global generator by default) and `pyrand`
    (Python's `random`), consuming them exactly as the reference does, generation by generation:
    tournament 1 and 2 (parego.py:89), crossover (:60-63), mutation (:45-51)."""
    if mutation_rate is None:
        mutation_rate = 1.0 / d
    sel = np.empty((iters, 4), np.int32)
    cross = np.zeros(iters, np.int8)
    beta = np.zeros((iters, d), np.float64)
    mut = np.zeros((iters, d), np.int8)
    for it in range(iters):
        sel[it, :2] = pyrand.sample(range(1, P), 2)
        sel[it, 2:] = pyrand.sample(range(1, P - 1), 2)
        if not nprand.rand() > crossover_prob:
            cross[it] = 1
            u = nprand.rand(d)
            beta[it] = np.where(u <= 0.5, (2 * u) ** (1.0 / (eta + 1)), (1.0 / (2 - 2 * u)) ** (1.0 / (eta + 1)))
        for i in range(d):
            if nprand.rand() < mutation_rate:
                mut[it, i] = 1 if nprand.uniform() > 0.5 else 2
    return EATape(sel, cross, beta, mut)


def mutate(x, lower, upper, mutation_rate, nprand=np.random):
    """ParEGO.mutate (parego.py:37-56): per gene ×1.05 or ×0.95 with probability `mutation_rate`."""
    m = np.array(x, np.float64, copy=True)
    for i in range(len(m)):
        if nprand.rand() < mutation_rate:
            m[i] = m[i] * 1.05 if nprand.uniform() > 0.5 else m[i] * 0.95
    return np.clip(m, lower, upper)


def latin_hypercube(num_samples, lower, upper, nprand=np.random):
    """util_functions.generate_latin_hypercube_samples (util_functions.py:46-61)."""
    lower = np.asarray(lower, np.float64)
    upper = np.asarray(upper, np.float64)
    out = np.empty((num_samples, len(lower)))
    for i, (lo, hi) in enumerate(zip(lower, upper)):
        intervals = np.linspace(lo, hi, num_samples + 1)
        points = nprand.rand(num_samples) + np.arange(num_samples)
        points /= num_samples
        out[:, i] = nprand.permutation(intervals[:-1] + (intervals[1:] - intervals[:-1]) * points)
    return out


def initial_population(Xsample, lower, upper, nprand=np.random, pyrand=random):
    """The temporary population of parego.py:229-235 / keep.py:246-252: mutants of 10 archive members
    (random.sample) followed by 10 Latin-hypercube points."""
    d = Xsample.shape[1]
    idx = pyrand.sample(range(0, len(Xsample)), 10)
    mutants = [mutate(Xsample[i], lower, upper, 1.0 / d, nprand) for i in idx]
    return np.vstack((mutants, latin_hypercube(10, lower, upper, nprand)))
