"""Multi-GPU candidate sharding: one process per GPU, torch.distributed (RCCL over xGMI).

The candidate batch is embarrassingly parallel: every rank holds a replica
of the per-iteration model state (X/ℓ, α, L⁻¹, σ_f², PF/cells, cache statistics) and scores
its own contiguous shard of candidate indices.  The only exchange is the arg-max: each rank
contributes {best value, best global index} (16 bytes) to one all-gather, and every rank
reduces the gathered pairs with the same rule as the device kernel (highest value, lowest
index on ties, index −1 = no valid candidate).  The result is identical to the single-GPU
arg-max over the concatenated batch.

The pair travels as two float64s, so the global index is exact up to 2^53 candidates (one step
scores at most 2^20-2^22 per rank; a maximiser sweep 2^16 per round).
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_range(n_total, world_size, rank):
    """Contiguous shard [start, start+count) of rank ``rank``; sizes differ by at most one."""
    base, extra = divmod(int(n_total), int(world_size))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def reduce_pairs(pairs):
    """pairs (W, 2) float64 {value, index}: best value, lowest index; invalid index < 0.

    Pure device arithmetic (no host synchronisation), so a multi-rank step loop never waits on the host.
    """
    vals = pairs[:, 0]
    idx = pairs[:, 1]
    valid = idx >= 0
    v = torch.where(valid, vals, torch.full_like(vals, float("-inf")))
    best = v.max()
    cand = valid & (v == best)
    i = torch.where(cand, idx, torch.full_like(idx, float("inf"))).min()
    none = ~valid.any()
    best = torch.where(none, torch.full_like(best, float("-inf")), best)
    i = torch.where(none, torch.full_like(i, -1.0), i)
    return torch.stack([best, i])


def agree_host_rng(seed=None):
    """Make every rank draw the same host randomness; returns the seed every rank uses.

    The drivers draw from numpy's global generator (LHS initial design, reference directions,
    ``np.random.randint`` in the reference's loops) and from Python's ``random`` (ParEGO's and KEEP's
    evolutionary search: ``random.sample`` for the temporary population and the tournaments,
    parego.py:91,228, keep.py:246), and derive the Sobol candidate seed and the MC sample cache from
    ``seed``.  With several ranks each of those must agree, or the ranks would score different
    candidate sets (or run different searches) and propose different points.  Rank 0's numpy state,
    ``random`` state and seed (drawn there when ``seed`` is None) are broadcast; with one rank nothing
    changes.
    """
    import random

    import numpy as np
    w, rank = world()
    if w == 1:
        return seed
    if rank == 0 and seed is None:
        seed = int(np.random.randint(0, 2 ** 31 - 1))
    box = [seed, np.random.get_state(), random.getstate()] if rank == 0 else [None, None, None]
    dist.broadcast_object_list(box, src=0)
    np.random.set_state(box[1])
    random.setstate(box[2])
    return box[0]


def global_argmax(local_pair, group=None, force=False):
    """All-gather each rank's {value, global index} pair and reduce it identically everywhere.

    At world size 1 the pair is returned as is, unless ``force``: then the all-gather and the
    reduction run anyway (a one-rank RCCL communicator exercises the same library load,
    communicator init and device all-gather that a multi-GPU run uses).
    """
    if not (dist.is_available() and dist.is_initialized()):
        return local_pair
    w = dist.get_world_size(group)
    if w == 1 and not force:
        return local_pair
    pair = local_pair.contiguous()
    if dist.get_backend(group) == "gloo" and pair.is_cuda:
        pair = pair.cpu()            # gloo rehearsal of the multi-rank path (tests, 1-GPU boxes)
    gathered = [torch.empty_like(pair) for _ in range(w)]
    dist.all_gather(gathered, pair, group=group)
    return reduce_pairs(torch.stack(gathered)).to(local_pair.device)
