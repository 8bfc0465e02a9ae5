"""Ablation (tools only): the EHVI-2D chain with the candidate batch cut into C chunks, chunk c's EHVI on a second
stream overlapping chunk c+1's posterior, against the one-batch chain and against the same chunks on one stream.
Configs 2 and 3 of bench.py (their training sets, cache seed 1); prints ms per step and checks the arg-max pair.

Usage: python tools/ablate/overlap_chain.py [config] [steps] [chunks,...]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import bench  # noqa: E402
from optimobo_amd import pareto  # noqa: E402
from optimobo_amd.device import AcqContext  # noqa: E402
from optimobo_amd.gp import GPState  # noqa: E402


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    chunk_list = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [2, 4, 8]
    cfg = bench.CONFIGS[config]
    n, d, N = cfg["n"], cfg["d"], 1 << cfg["log2"]
    dev = torch.device("cuda:0")
    X, Y, ls, variances = bench.setup_problem(n, d, problem=cfg["problem"], tail_hi=cfg.get("tail_hi", 1.0))
    pf = pareto.calc_pf(Y)
    r = Y.max(axis=0) + 0.1 * (Y.max(axis=0) - Y.min(axis=0))
    s00, s01 = pareto.cache_stats(pareto.cached_samples(2, 5, seed=1))
    stripes = torch.as_tensor(pareto.stripes_2d(pf), device=dev)
    ctxP, ctxA = AcqContext(0), AcqContext(0)
    for o in range(2):
        ctxP.set_gp_state(o, GPState(X, Y[:, o], ls, variances[o]))
    Xc = torch.as_tensor(bench.candidates(d, 0, N), device=dev)
    acq = torch.empty(N, dtype=torch.float64, device=dev)
    pair = torch.empty(2, dtype=torch.float64, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run(C, overlap):
        Nc = N // C
        mus = [torch.empty((2, Nc), dtype=torch.float64, device=dev) for _ in range(C)]
        vrs = [torch.empty_like(mus[0]) for _ in range(C)]
        evs = [torch.cuda.Event() for _ in range(C)]
        done = torch.cuda.Event()

        def step():
            with torch.cuda.stream(s1):
                for c in range(C):
                    ctxP.posterior(Xc[c * Nc:(c + 1) * Nc], 2, out=(mus[c], vrs[c]))
                    if overlap:
                        evs[c].record(s1)
                        with torch.cuda.stream(s2):
                            s2.wait_event(evs[c])
                            ctxA.ehvi2d(mus[c], vrs[c], stripes, r, s00, s01, out=acq[c * Nc:(c + 1) * Nc])
                    else:
                        ctxA.ehvi2d(mus[c], vrs[c], stripes, r, s00, s01, out=acq[c * Nc:(c + 1) * Nc])
                if overlap:
                    done.record(s2)
                    s1.wait_event(done)
                ctxA.argmax_dev(acq, offset=0, out=pair)

        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3, pair.cpu().numpy().copy()

    base_ms, base_pair = run(1, False)
    print(f"config {config} N={N}: one batch {base_ms:.4f} ms/step pair {base_pair}", flush=True)
    for C in chunk_list:
        for overlap in (False, True):
            ms, p = run(C, overlap)
            print(f"  C={C} {'two streams' if overlap else 'one stream '} {ms:.4f} ms/step "
                  f"({ms - base_ms:+.4f}) pair {'same' if np.array_equal(p, base_pair) else p}", flush=True)
    base_ms2, _ = run(1, False)
    print(f"  one batch again {base_ms2:.4f} ms/step", flush=True)
    ctxP.close()
    ctxA.close()


if __name__ == "__main__":
    main()
