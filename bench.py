#!/usr/bin/env python3
"""bench.py -- north-star metric of BASELINE.json:
point-clouds/sec (1024 pts, k=32) PPF + sph-vox forward at 1/2/4/8 MI355X.

One step = one sph-dg extractor forward pass (pcr_amd.extractor.SphExtractor)
over one batch of synthetic clouds already resident in HBM: self-KNN (k) +
local PPF, spherical normalisation + voxelisation (dense [B,C,r^3] grid, ind,
cnt), spherical devoxelisation of that grid and the per-cloud descriptor.
Workload = BASELINE config 2: batch 32 x 1024 points, k=32, 32^3 spherical
grid, C=64 channels (PVConv-1 width), per GPU.  Multi-GPU: one process per
GPU (torch.distributed, RCCL), the batch is sharded by cloud (weak scaling:
32 clouds per rank) and the per-cloud descriptors are all-gathered every step
(registration matching), overlapped on a side stream.

Prints ONE JSON line (rank 0).  `roofline` is step level: SURVEY 8d's
algorithmic bytes of the whole step over ms_per_step against the 8 TB/s HBM
peak; its `kernel` entry prices the dominant kernel (vox_stream_kernel, the
dense [B,C,r^3] grid + cnt) from its in-step duration, HIP events on its own
stream around its launches in the last 10 steps of the timed region.
`cpu_baseline` times the CPU restatement (oracle/, the "port") on a bounded
sample of the same workload on this box's host cores, single-thread and on
every usable core.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--workload", choices=("extract", "pairs"), default="extract",
                    help="extract: BASELINE c2, the sph-dg extractor forward over 32 clouds "
                         "per GPU; pairs: BASELINE c4, 256 clouds (128 registration pairs) "
                         "per GPU, extractor forward over sources + targets, on-rank mutual-NN "
                         "matching of their devoxelised features, descriptor all-gather")
    ap.add_argument("--batch", type=int, default=None,
                    help="clouds per GPU (default 32 for extract, 256 for pairs)")
    ap.add_argument("--points", type=int, default=1024)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--schedule", type=int, choices=(0, 1, 2), default=1,
                    help="pcr_extractor_run schedule (include/pcr_amd.h): 1 = three streams "
                         "(sort+select+PPF / prep+means+devox / dense-grid stream), 2 = as 1 "
                         "with the Morton sort on the prep stream, 0 = two streams")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="diagnostic: no timing events around the grid kernel (no in-step "
                         "kernel duration; checks the events' own cost)")
    ap.add_argument("--no-verify", action="store_true",
                    help="diagnostic: skip the after-run output check (runs that drop launches)")
    ap.add_argument("--steps-per-launch", type=int, default=40,
                    help="most pipelined steps per native runner call; --steps and --warmup "
                         "are split into calls of at most this many steps")
    args = ap.parse_args()
    if args.batch is None:
        args.batch = 256 if args.workload == "pairs" else 32
    if args.workload == "pairs" and args.batch % 2:
        ap.error("--workload pairs needs an even --batch (source + target clouds)")
    return args


def synthetic_inputs(b, n, c, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    xyz = torch.randn((b, 3, n), generator=g, device=device)
    xyz = (xyz - xyz.mean(dim=2, keepdim=True)).contiguous()
    nrm = torch.randn((b, 3, n), generator=g, device=device)
    nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
    feat = (torch.rand((b, c, n), generator=g, device=device) * 2 - 1).contiguous()
    return xyz, nrm, feat


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def usable_cores():
    """Threads this process can really run: its CPU affinity, capped by the
    cgroup CPU quota when one is set (a container's share of the host)."""
    aff = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(p))))
            if quota < aff:
                return quota, "affinity %d CPUs, cgroup quota %d" % (aff, quota)
    except (OSError, ValueError):
        pass
    return aff, "affinity %d CPUs" % aff


def cpu_baseline(args):
    """Time the CPU restatement (oracle/pcr_oracle.c, OpenMP across clouds)
    on repeated batches of the same workload: once on one thread and once on
    every core this process may run on (len(os.sched_getaffinity(0))), each
    for about args.cpu_seconds.  The all-core figure is `value`."""
    import numpy as np
    import oracle
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from clouds import gaussian_clouds
    # the same workload on a sample batch of at most 32 clouds (16 pairs)
    b, n, c, k, r = min(args.batch, 32), args.points, args.channels, args.k, args.res
    xyz, nrm, feat = gaussian_clouds(b, n, seed=0, c=c)
    pairs = args.workload == "pairs"

    def one_batch():
        _, ki = oracle.knn_dir(xyz, xyz, k)
        oracle.local_ppf(xyz, nrm, xyz, nrm, ki, kmajor=True, relative=True)
        nc = oracle.normalize_sph(xyz)
        grid, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
        dv, _, _ = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
        dv.max(axis=2)
        if pairs:
            f = dv.transpose(0, 2, 1)
            oracle.mutual_nn(np.ascontiguousarray(f[:b // 2]), np.ascontiguousarray(f[b // 2:]))

    def rate(threads, seconds):
        oracle.set_num_threads(threads)
        one_batch()  # warm (page-in, thread pool)
        done, t0 = 0, time.perf_counter()
        while True:
            one_batch()
            done += b
            el = time.perf_counter() - t0
            if el >= seconds:
                return done / el, done, el

    cores, why = usable_cores()
    r1, d1, e1 = rate(1, args.cpu_seconds / 2)
    rn, dn, en = rate(cores, args.cpu_seconds)
    return {"value": rn, "unit": "point-clouds/sec", "cores": cores, "kind": "port",
            "single_thread": {"value": r1, "cores": 1},
            "sample": "batches of %d clouds (N=%d, k=%d, r=%d, C=%d): %d clouds in %.1f s on "
                      "1 thread, %d clouds in %.1f s on %d threads; oracle/pcr_oracle.c, "
                      "OpenMP over clouds, %s; %s" % (b, n, k, r, c, d1, e1, dn, en, cores,
                                                       cpu_model(), why)}


def verify_runner(ex, xyz, nrm, feat, args, dev):
    """Two native-runner steps with the bench's schedule vs one forward():
    knn_idx, local_ppf, ind, cnt, grid and devox must be identical."""
    sx = ex.ex if args.workload == "pairs" else ex
    ref = {k: v.clone() for k, v in sx.forward(xyz, nrm, feat).items()}
    for t in list(sx.outputs(0).values()) + list(sx.outputs(1).values()):
        t.view(-1).view(torch.uint8).fill_(0xFF)
    out = sx.run_native(xyz, nrm, feat, 2, None, schedule=args.schedule)
    torch.cuda.synchronize(dev)
    for key in ("knn_idx", "local_ppf", "ind", "cnt", "grid", "devox"):
        if not torch.equal(out[key], ref[key]) and not torch.allclose(out[key], ref[key],
                                                                      equal_nan=True):
            raise SystemExit("bench: runner output %s differs from the single-step path" % key)
    return True


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from pcr_amd.extractor import (SphExtractor, algorithmic_bytes_per_cloud,
                                   stream_kernel_bytes_per_cloud)
    b, n, c, k, r = args.batch, args.points, args.channels, args.k, args.res
    xyz, nrm, feat = synthetic_inputs(b, n, c, dev, seed=1234 + rank)
    if args.workload == "pairs":
        # targets = sources rotated by a fixed rotation and permuted
        rot = torch.linalg.qr(torch.randn(3, 3, generator=torch.Generator().manual_seed(7)))[0]
        rot = rot.to(dev)
        perm = torch.randperm(n, generator=torch.Generator().manual_seed(8)).to(dev)
        p = b // 2
        xyz[p:] = torch.einsum("ij,bjn->bin", rot, xyz[:p])[:, :, perm]
        nrm[p:] = torch.einsum("ij,bjn->bin", rot, nrm[:p])[:, :, perm]
        feat[p:] = feat[:p][:, :, perm]
    if args.workload == "pairs":
        from pcr_amd.registration import PairExtractor
        ex = PairExtractor(b // 2, n, c, k, r, device=dev)
    else:
        ex = SphExtractor(b, n, c, k, r, device=dev)

    # the native runner enqueues up to S pipelined steps per call; the step
    # counts are split into calls of at most S steps (the last call shorter)
    S = max(1, args.steps_per_launch)

    def chunks(total):
        return [min(S, total - i) for i in range(0, total, S)]

    comm = torch.cuda.Stream(device=dev) if world > 1 else None
    desc_out = [torch.empty((world * S * b, c), device=dev) for _ in range(2)]
    desc_in = [torch.empty((S * b, c), device=dev) for _ in range(2)]
    pending = []
    desc_steps = {m: torch.empty((m, b, c), device=dev) for m in set(chunks(args.steps)) |
                  set(chunks(args.warmup))}

    def launch(i, m, timed=False):
        """One native runner call of m steps (call i of a sequence)."""
        ex.run_native(xyz, nrm, feat, m, desc_steps[m], schedule=args.schedule, timed=timed)
        src = desc_steps[m].view(m * b, c)
        if world > 1:
            # descriptor all-gather of the m batches (registration matching),
            # overlapped with the next launch on a side stream; double-buffered:
            # the gather that last read this slot is waited for before the copy
            slot = i & 1
            if len(pending) == 2:
                pending.pop(0).wait()
            desc_in[slot][:m * b].copy_(src)
            comm.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(comm):
                pending.append(dist.all_gather_into_tensor(
                    desc_out[slot][:world * m * b], desc_in[slot][:m * b], async_op=True))

    # the runner's timing events exist before the timed region (creating them
    # synchronises the device)
    # (the grid kernel of the last KTIMED steps of the timed region is timed:
    # each timing pair costs the step ~1.5%, so not every step carries one)
    KTIMED = 10
    if not args.no_kernel_timing:
        ex.reserve_timing(KTIMED)
    # before the warm-up, outside the timed region: the runner's outputs are
    # checked against the single-step (one call per stage) path on the same
    # inputs, with every runner output poisoned first, so the timed number is
    # for complete work (the check also brings the GPU up to clock)
    verified = False if args.no_verify else verify_runner(ex, xyz, nrm, feat, args, dev)
    for i, m in enumerate(chunks(args.warmup)):
        launch(i, m)
    for w in pending:
        w.wait()
    pending.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    timed_chunks = chunks(args.steps)
    for i, m in enumerate(timed_chunks):
        # the last call of the timed region also brackets the grid kernel of
        # its last KTIMED steps with timing events on its stream (in-step
        # durations)
        launch(i, m, timed=KTIMED if (i == len(timed_chunks) - 1 and not args.no_kernel_timing)
               else False)
    for w in pending:
        w.wait()
    pending.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # dominant kernel (the dense-grid stream kernel), in step: HIP events on
    # the stream it is launched on (ex.s_vox) around each of its launches in
    # the last runner call of the timed region
    grid_ms = ex.grid_kernel_times()
    grid_avg_ms = sum(grid_ms) / len(grid_ms) if grid_ms else float("nan")
    grid_bytes = stream_kernel_bytes_per_cloud(r, c) * b
    grid_gbs = grid_bytes / (grid_avg_ms * 1e-3) / 1e9
    kname = "vox_stream_kernel (sph-vox dense grid + cnt from the voxel means)"


    total_clouds = b * world * args.steps
    value = total_clouds / elapsed
    step_bytes = algorithmic_bytes_per_cloud(n, k, r, c)["total"] * b
    if args.workload == "pairs":
        # matching: both clouds' [C, N] features read, corr12 / corr21 /
        # idx1 / idx2 written (4 x 4N), per pair
        step_bytes += (2 * 4 * c * n + 16 * n) * (b // 2)
    step_gbs = step_bytes * args.steps / elapsed / 1e9
    traffic = step_traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("config") == [b, n, k, r, c]:
                traffic = pm.get("grid_kernel_hbm_bytes_per_launch")
                step_traffic = pm.get("step_hbm_bytes")
        except (OSError, ValueError):
            traffic = None

    result = {
        "metric": "point-clouds/sec (1024 pts, k=32) PPF+sph-vox forward",
        "value": round(value, 1),
        "unit": "point-clouds/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded gaussian clouds, unit normals, U(-1,1) features)",
        "outputs_verified": verified,
        "config": {"workload": ("sph-dg extractor forward: self-KNN k=%d + local PPF + "
                                "sph-vox r=%d^3 + sph-devox + descriptor" % (k, r))
                   if args.workload == "extract" else
                   ("registration pairs (BASELINE c4): extractor forward over %d source + %d "
                    "target clouds (self-KNN k=%d + local PPF + sph-vox r=%d^3 + sph-devox + "
                    "descriptor), mutual-NN matching of each pair's devox features on-rank, "
                    "descriptor all-gather" % (b // 2, b // 2, k, r)),
                   "clouds_per_gpu": b, "pairs_per_gpu": b // 2 if args.workload == "pairs"
                   else None, "points": n, "k": k, "resolution": r, "channels": c,
                   "global_batch": b * world, "parallelism": "dp%d (clouds sharded, "
                   "descriptor all-gather)" % world, "schedule": args.schedule,
                   "runner_calls": [len(chunks(args.warmup)), len(timed_chunks)],
                   "steps_per_launch": S},
        # step level (the north-star quantity): SURVEY 8d algorithmic bytes of
        # the whole step / ms_per_step; per rank, since every rank moves its
        # own HBM
        "roofline": {"bound": "hbm", "achieved": round(step_gbs, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(step_gbs / HBM_PEAK_GBS, 4),
                     "traffic": step_traffic,
                     "level": "step: %d B/cloud x %d clouds per rank / ms_per_step"
                              % (step_bytes // b, b),
                     "kernel": {"name": kname, "avg_ms_in_step": round(grid_avg_ms, 5),
                                "launches_timed": len(grid_ms),
                                "bytes_per_launch": grid_bytes,
                                "achieved": round(grid_gbs, 1),
                                "frac": round(grid_gbs / HBM_PEAK_GBS, 4),
                                "traffic": traffic}},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
