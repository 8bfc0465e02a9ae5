"""GPU: the multi-rank arg-max on the device pairs that omb_eval_argmax produces.

Two ranks share cuda:0 over gloo (the 1-GPU box rehearsal of the RCCL path): each
rank scores its own contiguous Sobol shard with the fused chain, the ranks exchange their
{value, index} pairs with ``global_argmax``, and the result must equal the single-process
arg-max over the whole batch.  The drop-in maximiser with ``seed=None`` must return the same
point on every rank (ranks agree on the seed and the numpy stream).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import torch.multiprocessing as mp  # noqa: E402


def _problem():
    rng = np.random.default_rng(11)
    X = rng.uniform(0, 1, (96, 5))
    f1 = X[:, 0]
    g = 1 + 9.0 / 4 * X[:, 1:].sum(1)
    Y = np.column_stack([f1, g * (1 - np.sqrt(f1 / g))])
    ls = np.array([0.4, 0.9, 1.3, 0.7, 1.1])
    return X, Y, ls


def _setup(ctx):
    from optimobo_amd import pareto
    from optimobo_amd.gp import GPState
    X, Y, ls = _problem()
    states = [GPState(X, Y[:, o], ls, float(np.var(Y[:, o]))) for o in range(2)]
    for o, st in enumerate(states):
        ctx.set_gp_state(o, st)
    pf = pareto.calc_pf(Y)
    r = Y.max(0) + 0.1 * (Y.max(0) - Y.min(0))
    s00, s01 = pareto.cache_stats(pareto.cached_samples(2, 5, seed=1))
    ctx.plan_ehvi2d(pareto.stripes_2d(pf), r, s00, s01, mode="reference")
    ctx.set_sobol(5, np.zeros(5), np.ones(5), seed=3)
    return states, pf, r


N_TOTAL = (1 << 18) + 37          # not a multiple of the world size: ragged shards


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from optimobo_amd.device import AcqContext
        from optimobo_amd.parallel import global_argmax, shard_range
        ctx = AcqContext(0)
        _setup(ctx)
        start, count = shard_range(N_TOTAL, world, rank)
        local = ctx.eval_argmax_sobol(start, count)
        g = global_argmax(local).cpu().numpy()
        # the drop-in maximiser with seed=None, same on every rank
        from optimobo_amd.algorithms.optimisers import MultiSurrogateOptimiser
        from optimobo_amd.problem import Problem

        class P(Problem):
            def __init__(self):
                super().__init__(n_var=5, n_obj=2, xl=np.zeros(5), xu=np.ones(5))

        np.random.seed(500 + rank)                      # ranks start out of step
        opt = MultiSurrogateOptimiser(P(), n_candidates=1 << 14, seed=None, device=0)
        states, pf, r = _setup(ctx)
        x, v = opt._get_proposed_EHVI("EHVI", states, None, r, pf, opt._get_cached_samples(2, 5))
        q.put((rank, [float(g[0]), float(g[1])], local.cpu().numpy().tolist(), x.tolist(), float(v)))
        ctx.close()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_device_pairs_equal_single_process():
    from optimobo_amd.device import AcqContext
    world = 2
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ctx = AcqContext(0)
    _setup(ctx)
    whole = ctx.eval_argmax_sobol(0, N_TOTAL).cpu().numpy()
    ctx.close()
    assert whole[0] > 0 and whole[1] >= 0
    for _, g, _, _, _ in got:
        assert (g[0], int(g[1])) == (whole[0], int(whole[1]))
    # the shards really were different: each rank's local winner lies in its own shard
    from optimobo_amd.parallel import shard_range
    for rank, _, local, _, _ in got:
        s, c = shard_range(N_TOTAL, world, rank)
        assert local[1] < 0 or s <= local[1] < s + c
    # the maximiser with seed=None: same point and value on both ranks
    assert got[0][3] == got[1][3] and got[0][4] == got[1][4]
