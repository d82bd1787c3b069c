"""Batch sharding across GPUs.

One process per GPU; chunk k of the global batch belongs to exactly one rank and
is compressed there with no data-path communication.  The only exchange is one
all-gather of the per-chunk compressed sizes, which gives every rank the global
output offsets (exclusive prefix sum) of the concatenated frames.  Over RCCL
(backend "nccl") on MI355X this is B x 8 bytes on xGMI; the same code runs over
gloo on CPU for the multi-process tests.
"""
from __future__ import annotations


def shard_range(rank: int, world: int, n_total: int):
    """Contiguous split of n_total chunks: rank r gets [r*q, min(n, (r+1)*q)), q = ceil(n/world)."""
    q = (n_total + world - 1) // world
    lo = min(n_total, rank * q)
    return lo, min(n_total, lo + q)


def weak_range(rank: int, n_per_rank: int):
    """Weak scaling (bench.py): every rank compresses n_per_rank chunks of its own slice."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


def gather_offsets(local_sizes, world: int, group=None):
    """All-gather equal-length int64 size vectors and return (all_sizes, exclusive offsets).

    local_sizes: 1-D int64 torch tensor on the rank's device (RCCL) or CPU (gloo).
    """
    import torch
    import torch.distributed as dist

    n = local_sizes.numel()
    all_sizes = torch.empty(world * n, dtype=local_sizes.dtype, device=local_sizes.device)
    if world > 1:
        dist.all_gather_into_tensor(all_sizes, local_sizes.contiguous(), group=group)
    else:
        all_sizes.copy_(local_sizes)
    offsets = torch.cumsum(all_sizes, 0) - all_sizes
    return all_sizes, offsets
