"""Batch sharding and descriptor exchange across GPUs (one process per GPU).

Every hot-path kernel is per cloud, so clouds shard with no
data-path collective.  Registration pairs keep src and tgt of a pair on the
same rank (per-point matching needs no exchange).  The only collective is the
all-gather of per-cloud descriptors [B_local, C] for registration matching
(RCCL over xGMI under the "nccl" backend; gloo on CPU for tests).
"""
import torch
import torch.distributed as dist


def shard_range(total, world, rank, unit=1):
    """Contiguous [start, stop) of `total` items for `rank`, in multiples of
    `unit` (unit=2 keeps a (src, tgt) registration pair together)."""
    if total % unit:
        raise ValueError("total %d is not a multiple of unit %d" % (total, unit))
    groups = total // unit
    base, rem = divmod(groups, world)
    start = rank * base + min(rank, rem)
    stop = start + base + (1 if rank < rem else 0)
    return start * unit, stop * unit


def gather_descriptors(desc, group=None):
    """All-gather [B_local, C] descriptors -> [world * B_local, C] in rank
    order (equal B_local on every rank)."""
    world = dist.get_world_size(group)
    out = torch.empty((world * desc.shape[0],) + tuple(desc.shape[1:]), dtype=desc.dtype,
                      device=desc.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, desc.contiguous(), group=group)
        return torch.cat(parts, dim=0)
    dist.all_gather_into_tensor(out, desc.contiguous(), group=group)
    return out
