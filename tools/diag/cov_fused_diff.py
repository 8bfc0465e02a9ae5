"""Where the fused-epilogue covariance differs from the two-launch build (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from optimobo_amd.device import AcqContext  # noqa: E402
from optimobo_amd.gp import GPState  # noqa: E402

ctx = AcqContext(0)
for n, d, N in [(20, 2, 77), (300, 6, 700)]:
    rng = np.random.default_rng(n + d)
    X = rng.uniform(0, 1, (n, d))
    y = np.sin(3 * X).sum(1) + X[:, 0] ** 2
    ls = rng.uniform(0.3, 1.5, d)
    ctx.set_gp_state(0, GPState(X, y, ls, float(np.var(y))))
    Xc = torch.as_tensor(np.clip(X[0] + 0.4 * (rng.uniform(0, 1, (N, d)) - 0.5), 0, 1), device="cuda:0")
    _, c1 = ctx.posterior_cov(0, Xc)
    ctx.debug_set("cov_fused", 0)
    _, c0 = ctx.posterior_cov(0, Xc)
    ctx.debug_set("cov_fused", 1)
    c1, c0 = c1.cpu().numpy(), c0.cpu().numpy()
    diff = c1 != c0
    idx = np.argwhere(diff)
    print(n, d, N, "differ:", diff.sum(), "of", diff.size, "max abs", np.abs(c1 - c0).max(),
          "diag differ", np.sum(np.diag(diff)))
    for i, j in idx[:8]:
        print("  ", i, j, repr(c1[i, j]), repr(c0[i, j]))
ctx.close()
