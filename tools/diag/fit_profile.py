"""Diagnostic (GPU box): where the lockstep per-objective fits of the README run spend their time —
per-round wall time by n, and a cProfile of fit_concurrently at n = 20, 60, 96, 119."""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from optimobo_amd import gp  # noqa: E402


def models(n, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-2, 2, (n, 2))
    Y = np.column_stack([100 * (X ** 2).sum(1), (X[:, 0] - 1) ** 2 + X[:, 1] ** 2])
    ms = [gp.GPRegression(X, Y[:, i:i + 1], gp.Matern52(2, ARD=True)) for i in range(2)]
    for m in ms:
        m.Gaussian_noise.variance.fix(0)
    return ms


gp.fit_concurrently(models(20, 0))
for n in (20, 60, 96, 97, 119):
    t = time.perf_counter()
    nf = 0
    for r in range(5):
        res = gp.fit_concurrently(models(n, r + 1))
        nf += max(x.nfev for x in res)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 5
    print(f"n={n}: {dt * 1e3:.2f} ms per 2-objective fit, {nf / 5:.1f} rounds, {dt / (nf / 5) * 1e3:.3f} ms per round",
          flush=True)
for n in (20, 119):
    pr = cProfile.Profile()
    pr.enable()
    for r in range(3):
        gp.fit_concurrently(models(n, r + 10))
    pr.disable()
    print(f"--- cProfile n={n}")
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
