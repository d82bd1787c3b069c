"""Batch sharding across GPUs.

One process per GPU; chunk k of the global batch belongs to exactly one rank and
is compressed there with no data-path communication.  The only exchange is one
all-gather of the per-chunk compressed sizes, which gives every rank the global
output offsets (exclusive prefix sum) of the concatenated frames.  Over RCCL
(backend "nccl") on MI355X this is B x 8 bytes on xGMI; the same code runs over
gloo on CPU for the multi-process tests.

Strong scaling (C4, the default of bench.py --gpus N): the same B-chunk batch is split
into contiguous ranges of q = ceil(B / world) chunks (shard_range), so the last ranks may
hold fewer chunks or none.  The all-gather needs equal-length vectors: every rank pads its
sizes to q, and the padding is dropped again by rank bounds before the prefix sum.
"""
from __future__ import annotations


def shard_range(rank: int, world: int, n_total: int):
    """Contiguous split of n_total chunks: rank r gets [r*q, min(n, (r+1)*q)), q = ceil(n/world)."""
    q = (n_total + world - 1) // world
    lo = min(n_total, rank * q)
    return lo, min(n_total, lo + q)


def weak_range(rank: int, n_per_rank: int):
    """Weak scaling (bench.py --weak): every rank compresses n_per_rank chunks of its own slice."""
    return rank * n_per_rank, (rank + 1) * n_per_rank


class ShardPlan:
    """Strong-scaling plan for n_total chunks over `world` ranks; caches the index that
    removes the all-gather padding (one gather kernel, no host work per step)."""

    def __init__(self, world: int, n_total: int):
        self.world, self.n_total = world, n_total
        self.q = (n_total + world - 1) // world if world else 0
        self._keep = {}

    def range(self, rank: int):
        return shard_range(rank, self.world, self.n_total)

    def _keep_index(self, device):
        import torch

        k = self._keep.get(device)
        if k is None:
            parts = []
            for r in range(self.world):
                lo, hi = self.range(r)
                parts.append(torch.arange(r * self.q, r * self.q + (hi - lo), dtype=torch.int64))
            k = torch.cat(parts).to(device)
            self._keep[device] = k
        return k

    def gather_offsets(self, local_sizes, group=None, force_collective=False):
        """All-gather this rank's per-chunk sizes (padded to q) -> (all_sizes[n_total],
        exclusive offsets[n_total]) in global chunk order.  A one-rank plan skips the
        collective unless force_collective (the RCCL test drives the gather at world 1)."""
        import torch
        import torch.distributed as dist

        if self.world == 1 and not force_collective:
            all_sizes = local_sizes.clone()
        else:
            n = local_sizes.numel()
            if n > self.q:
                raise ValueError(f"rank holds {n} chunks, more than the shard size {self.q}")
            pad = torch.zeros(self.q, dtype=local_sizes.dtype, device=local_sizes.device)
            pad[:n] = local_sizes
            gathered = torch.empty(self.world * self.q, dtype=local_sizes.dtype, device=local_sizes.device)
            dist.all_gather_into_tensor(gathered, pad, group=group)
            all_sizes = gathered.index_select(0, self._keep_index(local_sizes.device))
        offsets = torch.cumsum(all_sizes, 0) - all_sizes
        return all_sizes, offsets


def gather_offsets(local_sizes, world: int, group=None, n_total: int | None = None):
    """All-gather per-chunk size vectors and return (all_sizes, exclusive offsets).

    local_sizes: 1-D int64 torch tensor on the rank's device (RCCL) or CPU (gloo).
    n_total: the global chunk count of a shard_range split (ranks may hold unequal
    slices); None means every rank holds the same number of chunks (weak_range).
    """
    if n_total is None:
        n_total = local_sizes.numel() * world
    return ShardPlan(world, n_total).gather_offsets(local_sizes, group=group)
