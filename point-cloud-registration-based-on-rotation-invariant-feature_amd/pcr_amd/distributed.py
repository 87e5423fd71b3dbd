"""Batch sharding and descriptor exchange across GPUs (one process per GPU).

Every hot-path kernel is per cloud, so clouds shard with no
data-path collective.  Registration pairs keep src and tgt of a pair on the
same rank (per-point matching needs no exchange).  The only collective is the
all-gather of per-cloud descriptors [B_local, C] for registration matching
(RCCL over xGMI under the "nccl" backend; gloo on CPU for tests).

The reference has no collective of its own: it runs single-process
nn.DataParallel (train.py:114-117), and its registration evaluation extracts
both clouds of a pair on that one process (datasets/deepgmr_mn40.py:71-97).
Here a rank owns whole pairs and only the [B, C] descriptors cross xGMI.
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


def check_counts(counts, group=None, device=None):
    """Raise unless every rank passed the same `counts` list.

    all_gather_into_tensor needs the same block size on every rank; with
    different lists, max(counts) differs between ranks and the collective
    hangs or mixes rows instead of failing.  One small all-reduce (MIN and
    MAX of every entry), so call it once at setup, not per step."""
    world = dist.get_world_size(group)
    counts = [int(c) for c in counts]
    if len(counts) != world:
        raise ValueError("counts %s: %d entries for world size %d" % (counts, len(counts), world))
    if device is None:
        device = torch.device("cpu") if dist.get_backend(group) == "gloo" else \
            torch.device("cuda", torch.cuda.current_device())
    lo = torch.tensor(counts, dtype=torch.int64, device=device)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if not torch.equal(lo, hi):
        raise ValueError("ranks passed different counts (entry-wise min %s, max %s)"
                         % (lo.tolist(), hi.tolist()))
    return counts


def _all_gather_block(out, block, group, async_op):
    """out [world * rows, ...] <- every rank's block [rows, ...] in rank order."""
    if dist.get_backend(group) == "gloo":
        parts = list(out.chunk(dist.get_world_size(group), dim=0))
        return dist.all_gather(parts, block, group=group, async_op=async_op)
    return dist.all_gather_into_tensor(out, block, group=group, async_op=async_op)


def gather_descriptors(desc, group=None, counts=None):
    """All-gather [B_local, C] descriptors -> [sum B_local, C] in rank order.

    Shards may be uneven (shard_range of a total not divisible by the world
    size): every rank pads its block to the largest shard, one
    all_gather_into_tensor moves the padded blocks, and the padding is
    dropped.  `counts` (B_local per rank, e.g. shard_counts(...)) saves the
    size exchange; it must be the SAME list on every rank (check_counts
    verifies that; only this rank's own entry is checked here).  Without it
    the sizes are all-gathered first."""
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
    _all_gather_block(out, block, group, async_op=False)
    if all(c == mx for c in counts):
        return out
    return torch.cat([out[r * mx:r * mx + counts[r]] for r in range(world)], 0)


class DescriptorPipeline:
    """The per-call descriptor all-gather of a pipelined step loop.

    A rank's loop enqueues m steps at a time (the native runner,
    pcr_extractor_run) whose descriptors land in desc_steps [m, B_local, C];
    submit() all-gathers them across ranks while the next call's steps run:

      * the copy into the padded send block runs on the caller's (current)
        stream, right after the steps that wrote desc_steps;
      * the collective runs on a side stream that waited for that copy, so
        it overlaps the next call's kernels (GPU); on gloo it is async_op;
      * two send/receive buffer pairs alternate; a submit waits for the
        gather that last used its pair before overwriting it.

    `counts` = clouds per step of every rank, identical on all ranks
    (checked once here).  Uneven counts are padded to the largest; result()
    drops the padding.  This is the code bench.py times at --gpus N."""

    def __init__(self, counts, channels, max_steps, device, group=None, check=True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = torch.device(device)
        self.counts = check_counts(counts, group, self.device) if check else \
            [int(c) for c in counts]
        if len(self.counts) != self.world:
            raise ValueError("counts %s for world size %d" % (self.counts, self.world))
        self.rows = self.counts[self.rank]
        self.mx = max(self.counts)
        self.c = int(channels)
        self.max_steps = int(max_steps)
        z = dict(dtype=torch.float32, device=self.device)
        # padding rows of the send blocks stay zero forever
        self.send = [torch.zeros((self.max_steps, self.mx, self.c), **z) for _ in range(2)]
        # flat receive buffers: a call of m steps uses the first world * m *
        # mx * C floats as [world, m, mx, C] (contiguous for any m)
        self.recv = [torch.empty((self.world * self.max_steps * self.mx * self.c,), **z)
                     for _ in range(2)]
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" \
            else None
        self.pending = []   # (work, slot, m) in submission order
        self.done = []      # (slot, m) of completed gathers, newest last
        self.calls = 0

    def _retire_oldest(self):
        work, slot, m = self.pending.pop(0)
        work.wait()
        self.done.append((slot, m))
        del self.done[:-2]

    def submit(self, desc_steps):
        """All-gather desc_steps [m, B_local, C] (m <= max_steps)."""
        m = int(desc_steps.shape[0])
        if m < 1 or m > self.max_steps or tuple(desc_steps.shape[1:]) != (self.rows, self.c):
            raise ValueError("desc_steps %s: expected [1..%d, %d, %d]"
                             % (tuple(desc_steps.shape), self.max_steps, self.rows, self.c))
        slot = self.calls & 1
        self.calls += 1
        # the gather that last read / wrote this slot's buffers is done
        # (its wait orders the current stream after it)
        while any(s == slot for _, s, _ in self.pending):
            self._retire_oldest()
        send = self.send[slot][:m]
        send[:, :self.rows].copy_(desc_steps)
        out = self.recv[slot][:self.world * m * self.mx * self.c].view(-1, self.c)
        if self.stream is None:
            work = _all_gather_block(out, send.view(-1, self.c), self.group, True)
        else:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                work = _all_gather_block(out, send.view(-1, self.c), self.group, True)
        self.pending.append((work, slot, m))

    def wait_all(self):
        """Wait for every submitted gather (orders the current stream after
        them on GPU)."""
        while self.pending:
            self._retire_oldest()

    def result(self):
        """Descriptors of the most recently completed gather as
        [m, sum(counts), C]: step-major, ranks in order inside a step,
        padding dropped.  Call wait_all() first."""
        if not self.done:
            raise RuntimeError("no completed gather")
        slot, m = self.done[-1]
        out = self.recv[slot][:self.world * m * self.mx * self.c].view(self.world, m, self.mx,
                                                                        self.c)
        return torch.cat([out[r, :, :self.counts[r]] for r in range(self.world)], dim=1)


def step_chunks(total, per_call):
    """A run of `total` steps as calls of at most `per_call` steps."""
    per_call = max(1, int(per_call))
    return [min(per_call, total - i) for i in range(0, int(total), per_call)]


def run_pipelined(total, per_call, launch, pipe=None):
    """The step loop of a rank: `total` steps as calls of at most `per_call`
    steps.  launch(i, m) enqueues call i (m steps) and returns its
    descriptors [m, B_local, C]; with a DescriptorPipeline they are
    all-gathered while the next call runs, and every gather is waited for
    before returning.  Returns the number of calls."""
    calls = step_chunks(total, per_call)
    for i, m in enumerate(calls):
        desc = launch(i, m)
        if pipe is not None:
            pipe.submit(desc)
    if pipe is not None:
        pipe.wait_all()
    return len(calls)
