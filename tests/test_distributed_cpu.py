"""CPU, world_size 2 over gloo: the registration-pair sharding and the
descriptor all-gather of the product path (pcr_amd.distributed) reproduce
the single-process descriptor table -- even and uneven shards, with and
without precomputed counts.  The descriptors are a fixed table made in the
parent (the per-cloud [C] descriptors a step produces); the workers run only
the product's sharding + gather code, as the GPU ranks do over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, table, with_counts, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "point-cloud-registration-based-on-rotation-"
                                             "invariant-feature_amd"), here]
    import torch.distributed as dist
    from pcr_amd.distributed import gather_descriptors, shard_counts, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total = table.shape[0]
    s, e = shard_range(total, world, rank, unit=2)
    local = torch.from_numpy(table[s:e])
    counts = shard_counts(total, world, unit=2) if with_counts else None
    allv = gather_descriptors(local, counts=counts)
    q.put((rank, (s, e), allv.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_keeps_pairs():
    from pcr_amd.distributed import shard_counts, shard_range
    spans = [shard_range(20, 3, r, unit=2) for r in range(3)]
    assert spans == [(0, 8), (8, 14), (14, 20)]
    assert all((e - s) % 2 == 0 for s, e in spans)
    assert shard_counts(20, 3, unit=2) == [8, 6, 6]
    with pytest.raises(ValueError):
        shard_range(7, 2, 0, unit=2)


@pytest.mark.parametrize("clouds,with_counts", [(8, True), (10, True), (10, False)])
def test_two_rank_pair_shards_and_gather(clouds, with_counts):
    table = np.random.default_rng(clouds).standard_normal((clouds, 16)).astype(np.float32)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, 2, port, table, with_counts, q))
             for rk in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rk, span, got = q.get(timeout=120)
        res[rk] = (span, got)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the two shards tile the clouds, pairs (2i, 2i+1) never split
    (s0, e0), (s1, e1) = res[0][0], res[1][0]
    assert s0 == 0 and e0 == s1 and e1 == clouds and e0 % 2 == 0
    for rk in range(2):
        assert np.array_equal(res[rk][1], table)
