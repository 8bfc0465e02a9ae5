"""Timing of the device evolutionary acquisition search (omb_ea_search) against the oracle's restatement
of the reference's search run as the reference runs it (one GP prediction per fitness call, numpy).

Run on the GPU box: python tools/ea_timing.py > gpurun_out/.../ea_timing.jsonl
Each line: n_train, n_var, generations, device ms per search (mean of 5 after one warm-up), host ms per
search (oracle, timed over a bounded number of generations and scaled), and whether both searches chose
the same point.
"""
import json
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from oracle import ea as oea  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from optimobo_amd import ea  # noqa: E402
from optimobo_amd.device import AcqContext  # noqa: E402
from optimobo_amd.gp import GPState  # noqa: E402


def main():
    ctx = AcqContext(0)
    for n, d in [(20, 2), (120, 2), (120, 6), (500, 6), (1000, 30)]:
        rng = np.random.default_rng(n + d)
        X = rng.uniform(0, 1, (n, d))
        y = np.sin(4 * X).sum(1) + X[:, 0]
        ls = rng.uniform(0.3, 1.2, d)
        var = float(np.var(y))
        ctx.set_gp_state(0, GPState(X, y, ls, var))
        lower, upper = np.zeros(d), np.ones(d)
        pop = ea.initial_population(X, lower, upper, nprand=np.random.RandomState(1), pyrand=random.Random(1))
        tape = ea.ea_tape(len(pop), d, nprand=np.random.RandomState(2), pyrand=random.Random(2))
        best = float(y.min())
        ctx.ea_search(pop, tape, best, lower, upper)
        t0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            x, f = ctx.ea_search(pop, tape, best, lower, upper)
        dev_ms = (time.perf_counter() - t0) * 1e3 / reps
        # host: the same search with one prediction per fitness call; a bounded number of generations
        gens = 100 if n <= 200 else 20
        short = ea.EATape(tape.sel[:gens], tape.cross[:gens], tape.beta[:gens], tape.mut[:gens])
        gp = ogp.ExactGP(X, y, ls, var)
        fit = oea.ei_fitness(gp, best)
        t0 = time.perf_counter()
        oea.search(pop, fit, short, lower, upper)
        host_per_gen = (time.perf_counter() - t0) / gens
        # the reference also re-evaluates the population (20) and both tournaments (4) every generation
        host_ms = host_per_gen * 1e3 * tape.iters * (1 + 24)
        same = None
        if n <= 200:
            x_o, _ = oea.search(pop, fit, tape, lower, upper)
            same = bool(np.array_equal(x, x_o))
        print(json.dumps({"n_train": n, "n_var": d, "generations": tape.iters, "device_ms": dev_ms,
                          "reference_style_host_ms_est": host_ms, "same_choice_as_oracle": same}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
