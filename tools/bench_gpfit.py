"""Time the GP hyperparameter fit: one log-marginal-likelihood + gradient evaluation on the device
(omb_gp_lml_grad) vs the host numpy evaluation (optimobo_amd.gp, 16 BLAS threads on the GPU box),
and a whole L-BFGS-B fit (GPy's max_f_eval=1000 budget) both ways.  Prints one JSON line per n."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from optimobo_amd.gp import GPRegression, Matern52
    for n in (32, 64, 96, 128, 512, 1024):
        rng = np.random.default_rng(n)
        X = rng.uniform(0, 1, (n, 6))
        y = (np.sin(3 * X).sum(1) + 0.3 * X[:, 0] ** 2)[:, None]
        row = {"n_train": n, "n_var": 6}
        for dev in (True, False):
            m = GPRegression(X, y, Matern52(6, variance=float(np.var(y)), lengthscale=np.full(6, 0.7), ARD=True),
                             device_fit=dev)
            m.Gaussian_noise.variance.fix(0)
            f = m._neg_lml_and_grad_device if dev else m._neg_lml_and_grad
            th = m._get_free()
            f(th)
            torch.cuda.synchronize()
            reps = 20 if dev else (5 if n <= 512 else 2)
            t0 = time.perf_counter()
            for _ in range(reps):
                f(th)
            torch.cuda.synchronize()
            row[f"{'device' if dev else 'host'}_eval_ms"] = (time.perf_counter() - t0) / reps * 1e3
            m2 = GPRegression(X, y, Matern52(6, ARD=True), device_fit=dev)
            m2.Gaussian_noise.variance.fix(0)
            t0 = time.perf_counter()
            res = m2.optimize(max_f_eval=1000 if (dev or n <= 512) else 100)
            row[f"{'device' if dev else 'host'}_fit_s"] = time.perf_counter() - t0
            row[f"{'device' if dev else 'host'}_fit_evals"] = int(res.nfev)
            row[f"{'device' if dev else 'host'}_fit_nlml"] = float(res.fun)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
