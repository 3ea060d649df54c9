"""Problem sharding over ranks.

Problems are independent, so N GPUs take disjoint slices of the global problem
stream with no collective on the data path: rank r owns global problem
indices ``[r*B, (r+1)*B)`` ("weak" scaling: per-rank work is fixed).  Inputs
are generated from the global index, so a problem's data and result do not
depend on the number of ranks.  The only collectives are a barrier and a
max-reduction of the timed interval (and optional gathers for checking).
"""
from __future__ import annotations

from .batch import make_batch


def global_range(per_rank, rank):
    return rank * per_rank, (rank + 1) * per_rank


def shard_batch(scenario, per_rank, rank, base_seed=0, **kw):
    """The batch rank ``rank`` owns (global indices rank*per_rank ...)."""
    lo, _ = global_range(per_rank, rank)
    return make_batch(scenario, per_rank, base_seed=base_seed, offset=lo, **kw)


def max_over_ranks(value, dist=None, device=None):
    """Max of a scalar over all ranks (the timed region's wall time)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
