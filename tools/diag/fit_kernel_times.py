"""Diagnostic (GPU box): one-launch GP-fit evaluations (omb_gp_lml_grad_batch, 2 problems) at fixed n, 60 calls
each, wall time per call.  Run under rocprofv3 --kernel-trace to get the kernel's own durations per n
(dispatches come in blocks of 60 in the order of NS)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from optimobo_amd.device import AcqContext  # noqa: E402

NS = (20, 40, 60, 80, 96, 119, 128)
ctx = AcqContext(0)
for n in NS:
    rng = np.random.default_rng(n)
    X = torch.as_tensor(rng.uniform(-2, 2, (n, 2)), device="cuda:0")
    ys = [torch.as_tensor(rng.standard_normal(n), device="cuda:0") for _ in range(2)]
    ls = np.array([[0.8, 1.1], [1.3, 0.7]])
    ctx.gp_lml_grad_batch(X, ys, ls, [1.0, 2.0])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(60):
        ctx.gp_lml_grad_batch(X, ys, ls, [1.0, 2.0])
    dt = (time.perf_counter() - t) / 60
    print(f"n={n}: {dt * 1e6:.1f} us per call (wall, incl. launch + sync)", flush=True)
ctx.close()
