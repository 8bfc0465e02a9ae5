"""Probe: do two host threads' omb_gp_lml_grad calls (own context and stream each) overlap?  Times a
loop of bare C calls (no scipy) on 1 and 2 threads.  Run on the GPU box."""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from optimobo_amd.device import AcqContext  # noqa: E402


def worker(n, reps, out, i):
    torch.cuda.set_device(0)
    ctx = AcqContext(0)
    s = torch.cuda.Stream(0)
    rng = np.random.default_rng(i)
    with torch.cuda.stream(s):
        X = torch.as_tensor(rng.uniform(-2, 2, (n, 2)), device="cuda:0")
        y = torch.as_tensor(rng.uniform(0, 1, n), device="cuda:0")
        ctx.gp_lml_grad(X, y, [0.7, 1.1], 1.3)
        t = time.perf_counter()
        for _ in range(reps):
            ctx.gp_lml_grad(X, y, [0.7, 1.1], 1.3)
        out[i] = time.perf_counter() - t
    ctx.close()


for n in (20, 60, 96):
    reps = 400
    for nt in (1, 2, 4):
        out = [0.0] * nt
        th = [threading.Thread(target=worker, args=(n, reps, out, i)) for i in range(nt)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        print(f"n={n} threads={nt}: {max(out) / reps * 1e3:.3f} ms per call per thread, "
              f"{nt * reps / max(out):.0f} calls/s total", flush=True)
