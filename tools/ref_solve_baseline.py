"""BASELINE config 1 — the README run (README.md:21-45) — through the reference's OWN
``MultiSurrogateOptimiser.solve`` (optimisers.py:144-277), timed on this container's CPU.  Container-only:
it imports /root/reference.

    MultiSurrogateOptimiser(MyProblem(), [0, 0], [700, 12]).solve(budget=100, n_init_samples=20,
        sample_exponent=3, acquisition_func=Tchebicheff([0, 0], [700, 12]))

Everything the reference does runs as written: Latin-hypercube design, the per-objective GP fits, scipy
``differential_evolution`` over ``util_functions.expected_decomposition`` (one candidate per call) and the
hypervolume trace.  Third-party packages absent here are test doubles (tests/golden/make_golden.py):
  * GPy ``GPRegression(...).optimize(max_f_eval=1000)`` → the build's numpy fit (optimobo_amd.gp.GPRegression
    with device_fit=False: GPy's Logexp parameters, scipy L-BFGS-B on −log p(y)), and ``predict`` → the
    oracle's restatement of GPy's exact-inference posterior (oracle/gp.py) at the fitted hyperparameters;
  * pymoo ``HV`` → exact hypervolume (oracle/pareto.py); ``get_reference_directions`` → Das-Dennis restated;
  * the problem is a duck-typed MyProblem (the reference's Problem base class needs pymoo).
GPy/paramz add per-call overhead the doubles do not have, so the rate is an UPPER bound on the reference's.

Usage: python tools/ref_solve_baseline.py [budget] [seed] > profiles/r04_ref_solve_c1.json
"""
import json
import os
import platform
import sys
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

import make_golden as mg  # noqa: E402
from oracle import gp as ogp  # noqa: E402
from oracle import pareto as opar  # noqa: E402


class MyProblem:
    """README.md:28-39."""
    n_var, n_obj = 2, 2
    xl = np.array([-2, -2])
    xu = np.array([2, 2])

    def evaluate(self, x):
        x = np.asarray(x, np.float64)
        return np.array([100 * (x[0] ** 2 + x[1] ** 2), (x[0] - 1) ** 2 + x[1] ** 2])


def main():
    budget = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    mg._install_doubles()
    from optimobo_amd import gp as hgp
    split = {"fit": 0.0, "predict_calls": 0}

    class GPyDouble:
        def __init__(self, X, Y, kern=None):
            self.X, self.Y = np.array(X, np.float64), np.array(Y, np.float64)
            self._m = hgp.GPRegression(self.X, self.Y, hgp.Matern52(self.X.shape[1], ARD=True), device_fit=False)
            self.Gaussian_noise = self._m.Gaussian_noise
            self._gp = None

        def optimize(self, messages=False, max_f_eval=1000):
            t = time.perf_counter()
            self._m.optimize(max_f_eval=max_f_eval)
            self._gp = ogp.ExactGP(self.X, self.Y[:, 0], self._m.kern.ls_vector(), float(self._m.kern.variance))
            split["fit"] += time.perf_counter() - t

        def predict(self, X):
            split["predict_calls"] += 1
            X = np.atleast_2d(np.asarray(X, np.float64))
            if not np.all(np.isfinite(X)):          # GPy propagates NaN (DE's polish can step to NaN after a
                nan = np.full((len(X), 1), np.nan)  # NaN objective); scipy's triangular solve would raise
                return nan, nan.copy()
            return self._gp.predict(X)

    sys.modules["GPy"].models.GPRegression = GPyDouble
    sys.modules["GPy"].kern.Matern52 = lambda *a, **k: None

    class HV:
        def __init__(self, ref_point):
            self.r = np.asarray(ref_point, np.float64)

        def __call__(self, Y):
            return opar.hypervolume(Y, self.r)
    import optimobo.algorithms.optimisers as opti
    import optimobo.scalarisations as sc
    opti.HV = HV
    opti.get_reference_directions = lambda name, n_dim, n_partitions=None: mg._das_dennis(n_dim, n_partitions)
    np.random.seed(seed)
    opt = opti.MultiSurrogateOptimiser(MyProblem(), [0, 0], [700, 12])
    # one BLAS thread, enforced and read back ("cores" was hard-coded)
    from threadpoolctl import threadpool_info, threadpool_limits
    with threadpool_limits(limits=1):
        threads = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
        t0 = time.perf_counter()
        res = opt.solve(budget=budget, n_init_samples=20, sample_exponent=3,
                        acquisition_func=sc.Tchebicheff([0, 0], [700, 12]))
        el = time.perf_counter() - t0
    print(json.dumps({
        "what": "reference MultiSurrogateOptimiser.solve (README run, BASELINE config 1): budget "
                f"{budget}, n_init 20, sample_exponent 3, Tchebicheff; scipy DE one candidate per call",
        "value": budget / el, "unit": "iterations/s", "seconds": el, "cores": int(threads), "kind": "reference",
        "measured_in": f"build container ({os.cpu_count()} vCPU), not the GPU box's host",
        "split_s": {"gp_fit": split["fit"], "de_and_rest": el - split["fit"]},
        "predict_calls": split["predict_calls"], "final_hv": float(res.hypervolume_convergence[-1]),
        "n_evaluations": int(len(res.ysample)), "np_seed": seed,
        "doubles": "GPy fit = optimobo_amd.gp numpy L-BFGS-B, predict = oracle/gp.py; pymoo HV = exact HV",
        "host": platform.processor() or platform.machine(), "host_cpu_count": os.cpu_count(),
    }))


if __name__ == "__main__":
    main()
