"""CPU, world_size 2 over gloo: cloud sharding + descriptor all-gather give
the same descriptors as a single process (descriptors computed by the CPU
oracle here; on the GPU box the same code path runs over RCCL)."""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def descriptors(xyz, feat, r):
    import oracle
    nc = oracle.normalize_sph(xyz)
    grid, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
    dv, _, _ = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
    return dv.max(axis=2)


def _worker(rank, world, port, xyz, feat, r, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "point-cloud-registration-based-on-rotation-"
                                             "invariant-feature_amd"), here]
    import torch.distributed as dist
    from pcr_amd.distributed import shard_range, gather_descriptors
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e = shard_range(xyz.shape[0], world, rank, unit=2)
    local = torch.from_numpy(descriptors(xyz[s:e], feat[s:e], r))
    allv = gather_descriptors(local)
    q.put((rank, allv.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_keeps_pairs():
    from pcr_amd.distributed import shard_range
    spans = [shard_range(20, 3, r, unit=2) for r in range(3)]
    assert spans == [(0, 8), (8, 14), (14, 20)]
    assert all((e - s) % 2 == 0 for s, e in spans)


def test_two_rank_descriptor_gather():
    from clouds import gaussian_clouds
    b, n, c, r = 8, 256, 8, 16
    xyz, _, feat = gaussian_clouds(b, n, seed=3, c=c)
    expected = descriptors(xyz, feat, r)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(rk, 2, port, xyz, feat, r, q)) for rk in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rk in range(2):
        assert np.array_equal(res[rk], expected)
