"""Batch sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Robots are independent: rank g owns the contiguous range [g B/G, (g+1) B/G) and
keeps its history resident; the only exchange is an all-gather of the torque block (and, if
wanted, statuses) so every rank holds B x 12 torques.
"""
from __future__ import annotations


def shard_bounds(total: int, world: int, rank: int):
    """Contiguous, balanced [lo, hi) robot range of `rank` (first total % world ranks get one more)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def all_gather_rows(local, world: int, group=None):
    """Concatenate every rank's equal-length 1-D block (RCCL all_gather_into_tensor on GPU tensors;
    the list form on gloo/CPU)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    if local.is_cuda:
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous(), group=group)
    return torch.cat(parts)
