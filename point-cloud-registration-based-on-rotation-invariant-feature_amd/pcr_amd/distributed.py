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


def shard_counts(total, world, unit=1):
    """Items per rank under shard_range, in rank order."""
    return [e - s for s, e in (shard_range(total, world, r, unit) for r in range(world))]


def gather_descriptors(desc, group=None, counts=None):
    """All-gather [B_local, C] descriptors -> [sum B_local, C] in rank order.

    Shards may be uneven (shard_range of a total not divisible by the world
    size): every rank pads its block to the largest shard, one
    all_gather_into_tensor moves the padded blocks, and the padding is
    dropped.  `counts` (B_local per rank, e.g. shard_counts(...)) saves the
    size exchange; without it the sizes are all-gathered first."""
    world = dist.get_world_size(group)
    rows = desc.shape[0]
    if counts is None:
        mine = torch.tensor([rows], dtype=torch.int64, device=desc.device)
        sizes = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(sizes, mine, group=group)
        counts = [int(s.item()) for s in sizes]
    counts = [int(c) for c in counts]
    if len(counts) != world or counts[dist.get_rank(group)] != rows:
        raise ValueError("counts %s do not match this rank's %d rows" % (counts, rows))
    mx = max(counts)
    block = desc.contiguous()
    if rows < mx:
        block = torch.cat((block, block.new_zeros((mx - rows,) + tuple(desc.shape[1:]))), 0)
    out = torch.empty((world * mx,) + tuple(desc.shape[1:]), dtype=desc.dtype,
                      device=desc.device)
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, block, group=group)
    else:
        dist.all_gather_into_tensor(out, block, group=group)
    if all(c == mx for c in counts):
        return out
    return torch.cat([out[r * mx:r * mx + counts[r]] for r in range(world)], 0)
