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


def _pipe_worker(rank, world, port, counts, per_call, total, channels, bad_counts, q):
    """One rank of the bench's step loop (pcr_amd.distributed.run_pipelined +
    DescriptorPipeline) with a stub launch: call i of m steps 'produces'
    descriptors whose values encode (rank, global step, cloud, channel)."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    sys.path[:0] = [root, os.path.join(root, "point-cloud-registration-based-on-rotation-"
                                             "invariant-feature_amd"), here]
    import torch.distributed as dist
    from pcr_amd.distributed import DescriptorPipeline, run_pipelined, step_chunks
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if bad_counts:
            mine = list(counts)
            mine[0] += rank  # rank 1 disagrees
            try:
                DescriptorPipeline(mine, channels, per_call, "cpu")
                q.put((rank, "no error"))
            except ValueError as e:
                q.put((rank, "ValueError: %s" % e))
            return
        rows = counts[rank]
        pipe = DescriptorPipeline(counts, channels, per_call, "cpu")
        buf = torch.empty((per_call, rows, channels))
        seen = []
        start = [0]

        def launch(i, m):
            s0 = start[0]
            start[0] += m
            d = buf[:m]
            for s in range(m):
                for j in range(rows):
                    d[s, j] = torch.arange(channels, dtype=torch.float32) + \
                        1000.0 * j + 1e5 * (s0 + s) + 1e7 * rank
            # the previous call's gather is complete once this launch returns
            # (at most one pair in flight beyond it): record finished results
            if pipe.done:
                seen.append(pipe.result().clone())
            return d

        ncalls = run_pipelined(total, per_call, launch, pipe)
        seen.append(pipe.result().clone())
        q.put((rank, (ncalls, step_chunks(total, per_call), [t.numpy() for t in seen])))
    finally:
        dist.barrier()
        dist.destroy_process_group()


def _expected(counts, s, channels):
    rows = []
    for r, cnt in enumerate(counts):
        for j in range(cnt):
            rows.append(np.arange(channels, dtype=np.float32) + 1000.0 * j + 1e5 * s + 1e7 * r)
    return np.stack(rows)


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(rk, world, port) + args + (q,))
             for rk in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rk, val = q.get(timeout=120)
        res[rk] = val
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("counts,per_call,total", [([4, 4], 5, 12), ([3, 2], 4, 9)])
def test_two_rank_step_loop_gathers_every_call(counts, per_call, total):
    """The bench's per-call loop at world size 2: calls of <= per_call steps,
    double-buffered gathers, uneven shards padded and unpadded; every
    completed gather holds [m, sum(counts), C] in step-major, rank order."""
    channels = 8
    res = _spawn(_pipe_worker, 2, counts, per_call, total, channels, False)
    for rk in range(2):
        ncalls, chunks, seen = res[rk]
        assert ncalls == len(chunks) and sum(chunks) == total
        # the last result is the last call's steps
        last = seen[-1]
        m = chunks[-1]
        assert last.shape == (m, sum(counts), channels)
        for s in range(m):
            assert np.array_equal(last[s], _expected(counts, total - m + s, channels))
        # every earlier result is a whole earlier call, in order
        starts = np.cumsum([0] + chunks)
        for got in seen[:-1]:
            m0 = got.shape[0]
            s0 = int(got[0, 0, 0] // 1e5) % 100
            assert s0 in starts and chunks[list(starts).index(s0)] == m0
            for s in range(m0):
                assert np.array_equal(got[s], _expected(counts, s0 + s, channels))


def test_two_rank_mismatched_counts_raise():
    res = _spawn(_pipe_worker, 2, [4, 4], 3, 3, 4, True)
    for rk in range(2):
        assert res[rk].startswith("ValueError"), res[rk]


def test_bench_gpus_beyond_visible_fails_loudly():
    """bench.py --gpus N with fewer visible GPUs exits non-zero with a clear
    message and prints no JSON line (no GPU in this container; on a one-GPU
    box the same holds for N = 2)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    want = max(2, torch.cuda.device_count() + 1)
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload", "pairs",
                        "--gpus", str(want), "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "--gpus %d needs %d GPUs" % (want, want) in p.stderr
    assert p.stdout.strip() == ""
