"""GPU: the arg-max exchange through RCCL on real hardware (VERDICT r03 missing #1).

A one-rank ``nccl`` (= RCCL on ROCm) process group on cuda:0: ``global_argmax(force=True)`` runs
the device all-gather of the 16-B {value, index} pair and the reduction, which is what every
rank of the multi-GPU bench does.  The gathered pair must equal the local one, for a real
device pair from the fused chain, an invalid pair and a tie.  ``torch.cuda.nccl.version()`` is
printed (``-s`` / ``-v`` output) so the GPU test log records which RCCL ran.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rccl_group():
    import torch.distributed as dist
    assert torch.cuda.is_available()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_rccl_version_and_backend(rccl_group):
    dist = rccl_group
    ver = torch.cuda.nccl.version()
    print(f"RCCL version {ver}, backend {dist.get_backend()}, torch {torch.__version__}, hip {torch.version.hip}")
    assert dist.get_backend() == "nccl"
    assert torch.version.hip is not None        # nccl here is RCCL


def test_rccl_all_gather_of_device_pair(rccl_group):
    from optimobo_amd import pareto
    from optimobo_amd.device import AcqContext
    from optimobo_amd.gp import GPState
    from optimobo_amd.parallel import global_argmax
    rng = np.random.default_rng(5)
    X = rng.uniform(0, 1, (64, 4))
    f1 = X[:, 0]
    g = 1 + 3.0 * X[:, 1:].sum(1)
    Y = np.column_stack([f1, g * (1 - np.sqrt(f1 / g))])
    ctx = AcqContext(0)
    try:
        for o in range(2):
            ctx.set_gp_state(o, GPState(X, Y[:, o], np.array([0.5, 0.8, 1.1, 0.7]), float(np.var(Y[:, o]))))
        pf = pareto.calc_pf(Y)
        r = Y.max(0) + 0.1 * (Y.max(0) - Y.min(0))
        s00, s01 = pareto.cache_stats(pareto.cached_samples(2, 5, seed=1))
        ctx.plan_ehvi2d(pareto.stripes_2d(pf), r, s00, s01, mode="reference")
        ctx.set_sobol(4, np.zeros(4), np.ones(4), seed=2)
        local = ctx.eval_argmax_sobol(0, 1 << 14)
        assert local.is_cuda
        got = global_argmax(local, force=True)
        torch.cuda.synchronize()
        assert got.is_cuda
        assert torch.equal(got.cpu(), local.cpu())
        assert float(local[1]) >= 0
    finally:
        ctx.close()


def test_rccl_all_gather_invalid_and_ties(rccl_group):
    from optimobo_amd.parallel import global_argmax
    dev = torch.device("cuda:0")
    none = torch.tensor([float("-inf"), -1.0], dtype=torch.float64, device=dev)
    assert global_argmax(none, force=True).cpu().tolist() == [float("-inf"), -1.0]
    pair = torch.tensor([0.25, 12345.0], dtype=torch.float64, device=dev)
    assert global_argmax(pair, force=True).cpu().tolist() == [0.25, 12345.0]
    # the raw collective: a multi-element all_gather_into_tensor over RCCL
    import torch.distributed as dist
    src = torch.arange(16, dtype=torch.float64, device=dev)
    out = torch.empty(16, dtype=torch.float64, device=dev)
    dist.all_gather_into_tensor(out, src)
    assert torch.equal(out, src)
