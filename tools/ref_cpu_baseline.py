"""The reference's OWN per-candidate acquisition path, timed on this container's CPU (BASELINE.md §3
item 1; SURVEY.md §8(d) "CPU timing beside it" (i)).  Container-only: it imports /root/reference.

What is timed is exactly what scipy's differential_evolution calls once per candidate in the
reference: ``obj(x) = -acq(x, ...)`` with the reference's own acquisition functions
  * ``util_functions.EHVI``                 (util_functions.py:136-167; BASELINE configs 2, 3)
  * ``util_functions.EHVI_3D``              (util_functions.py:170-214; config 4)
  * ``EMO.hypervolume_based_PoI``           (emo.py:192-228)
  * ``ParEGO._expected_improvement``        (parego.py:126-145; config 5)
  * ``util_functions.expected_decomposition`` with Tchebicheff (util_functions.py:285-327; config 1)
The fitted GPy models they call ``predict`` on are replaced by the oracle's restatement of GPy's
exact-inference posterior (oracle/gp.py: GPy is not installed), which has less per-call overhead than
GPy/paramz — so these rates are UPPER bounds on the reference's speed.  pygmo / pymoo are replaced
by the test doubles of tests/golden/make_golden.py (exact hypervolume, first-front filter).
Single Python thread, BLAS pinned to 1 thread (the reference calls predict on one row at a time).

Usage: python tools/ref_cpu_baseline.py [seconds_per_case] > profiles/r02_ref_cpu_baseline.jsonl
"""
import json
import os
import platform
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import make_golden as mg  # noqa: E402  (installs the pygmo/GPy/pymoo doubles)
from oracle import gp as ogp  # noqa: E402
from oracle import pareto as opar  # noqa: E402


def zdt1(X):
    f1 = X[:, 0]
    g = 1 + 9.0 / (X.shape[1] - 1) * np.sum(X[:, 1:], axis=1)
    return np.column_stack([f1, g * (1 - np.sqrt(f1 / g))])


def dtlz2(X, k=3):
    g = np.sum((X[:, k - 1:] - 0.5) ** 2, axis=1)
    th = X[:, :k - 1] * np.pi / 2
    F = np.empty((len(X), k))
    for i in range(k):
        f = 1 + g
        for j in range(k - 1 - i):
            f = f * np.cos(th[:, j])
        if i > 0:
            f = f * np.sin(th[:, k - 1 - i])
        F[:, i] = f
    return F


def setup(n, d, problem):
    """bench.py's synthetic workload (same seeds)."""
    rng = np.random.default_rng(0)
    X = rng.uniform(0.0, 1.0, (n, d))
    Y = zdt1(X) if problem == "zdt1" else dtlz2(X)
    ls = np.random.default_rng(1).uniform(0.2, 2.0, d)
    return X, Y, ls


def candidates(d, count):
    from scipy.stats import qmc
    return qmc.Sobol(d=d, scramble=False).random(count)


def time_calls(fn, Xc, seconds):
    done = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn(Xc[done % len(Xc)])
        done += 1
    dt = time.perf_counter() - t0
    return done, dt


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    from threadpoolctl import threadpool_limits
    mg._install_doubles()
    import optimobo.util_functions as uf
    import optimobo.scalarisations as sc
    import optimobo.algorithms.emo as emo_mod
    import optimobo.algorithms.parego as parego_mod
    host = {"cpu": platform.processor() or platform.machine(), "os_cpu_count": os.cpu_count(),
            "python": platform.python_version(), "numpy": np.__version__}
    out = []
    with threadpool_limits(limits=1):
        cases = []
        for cfg, n, d, k, problem in [(2, 128, 6, 2, "zdt1"), (3, 512, 6, 2, "zdt1"), (4, 256, 6, 3, "dtlz2")]:
            X, Y, ls = setup(n, d, problem)
            models = [ogp.ExactGP(X, Y[:, o], ls, float(np.var(Y[:, o]))) for o in range(k)]
            pf = opar.calc_pf(Y)
            r = Y.max(0) + 0.1 * (Y.max(0) - Y.min(0))
            cache = mg.cached_samples(k, 5, seed=1)
            Xc = candidates(d, 4096)
            if k == 2:
                cases.append((f"EHVI (util_functions.py:136) config {cfg}", cfg, n, d,
                              lambda x, m=models, r=r, pf=pf, c=cache: -uf.EHVI(x, m, r, pf, c), Xc))
                obj = object.__new__(emo_mod.EMO)
                obj.ideal_point, obj.max_point, obj.n_obj = Y.min(0), Y.max(0), 2
                cells = obj.decompose_into_cells(pf)
                cases.append((f"EMO.hypervolume_based_PoI (emo.py:192) config {cfg} shape", cfg, n, d,
                              lambda x, o=obj, m=models, c=cells: -o.hypervolume_based_PoI(x, m, None, c), Xc))
            else:
                # in-box candidates only raise rarely; a raise is what pygmo does and DE would see it
                def ehvi3(x, m=models, r=r, pf=pf, c=cache):
                    try:
                        return -uf.EHVI_3D(x, m, r, pf, c)
                    except ValueError:
                        return np.nan
                cases.append((f"EHVI_3D (util_functions.py:170) config {cfg}", cfg, n, d, ehvi3, Xc))
        # config 5: ParEGO mono surrogate EI, n = 1024, d = 30
        X, Y, ls = setup(1024, 30, "zdt1")
        tch = sc.Tchebicheff(Y.min(0), Y.max(0))
        yagg = np.asarray([tch(y, np.array([0.5, 0.5])) for y in Y]).reshape(-1)
        model = ogp.ExactGP(X, yagg, ls, float(np.var(yagg)))
        par = object.__new__(parego_mod.ParEGO)
        best = float(yagg.min())
        cases.append(("ParEGO._expected_improvement (parego.py:126) config 5", 5, 1024, 30,
                      lambda x, m=model, b=best: -par._expected_improvement(x, m, b), candidates(30, 4096)))
        # config 1: README MyProblem, Tchebicheff expected decomposition (n grows 20 -> 119; n = 120 here)
        rng = np.random.default_rng(0)
        X = rng.uniform(-2, 2, (120, 2))
        Y = np.column_stack([100 * (X[:, 0] ** 2 + X[:, 1] ** 2), (X[:, 0] - 1) ** 2 + X[:, 1] ** 2])
        models = [ogp.ExactGP(X, Y[:, o], np.array([0.8, 0.8]), float(np.var(Y[:, o]))) for o in range(2)]
        tch = sc.Tchebicheff(np.array([0.0, 0.0]), np.array([700.0, 12.0]))
        w = np.array([0.3, 0.7])
        agg_min = float(np.min([tch(y, w) for y in Y]))
        cache = mg.cached_samples(2, 3, seed=1)
        cases.append(("expected_decomposition + Tchebicheff (util_functions.py:285) config 1, n=120", 1, 120, 2,
                      lambda x, m=models: -uf.expected_decomposition(x, m, w, tch, agg_min, cache),
                      4 * candidates(2, 4096) - 2))
        for name, cfg, n, d, fn, Xc in cases:
            with np.errstate(all="ignore"):
                fn(Xc[0])                                   # warm up
                done, dt = time_calls(fn, Xc, seconds)
            rec = {"what": name, "config": cfg, "n_train": n, "n_var": d, "calls": done, "seconds": dt,
                   "value": done / dt, "unit": "candidates/s", "cores": 1, "kind": "reference",
                   "note": "reference acquisition code per candidate (as differential_evolution calls it); "
                           "GPy predict replaced by oracle/gp.py (upper bound on the reference speed)",
                   "host": host}
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
