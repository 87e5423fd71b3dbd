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

Prints ONE JSON line (rank 0).  `roofline` prices the dominant kernel (the
voxel kernel of the step, vox_grid_kernel<3>: dense [B,C,r^3] grid + cnt, devox + descriptor) from its HIP-event-timed average duration;
`cpu_baseline` times the CPU restatement (oracle/, the "port") on a bounded
sample of the same workload on this box's host cores.
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
    ap.add_argument("--batch", type=int, default=32, help="clouds per GPU")
    ap.add_argument("--points", type=int, default=1024)
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--res", type=int, default=32)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=("native", "native2", "pipelined", "pipelined_split",
                                       "pipelined3", "pipelined4",
                                       "pipelined_sv", "pipelined_fs", "pipelined_3s", "pipelined_2s", "graph",
                                       "eager"),
                    default="native",
                    help="native: S steps enqueued by the library (pcr_extractor_run) on three "
                         "streams -- KNN, prep + means/devox, grid stream; native2: the same "
                         "runner, two streams with the fused grid kernel; "
                         "pipelined: S steps on two independent streams (KNN / voxel, fused "
                         "grid+devox kernel) from Python with no join between them; pipelined_split: "
                         "separate grid and devox launches; pipelined3/4/_sv: schedules with cross-stream "
                         "events; graph: one hipGraph replay per step; eager: fork/join per step")
    ap.add_argument("--steps-per-launch", type=int, default=40,
                    help="pipelined steps per launch group (must divide --steps and --warmup)")
    return ap.parse_args()


def synthetic_inputs(b, n, c, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    xyz = torch.randn((b, 3, n), generator=g, device=device)
    xyz = (xyz - xyz.mean(dim=2, keepdim=True)).contiguous()
    nrm = torch.randn((b, 3, n), generator=g, device=device)
    nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
    feat = (torch.rand((b, c, n), generator=g, device=device) * 2 - 1).contiguous()
    return xyz, nrm, feat


def cpu_baseline(args):
    """Time the CPU restatement (oracle, OpenMP across clouds) on repeated
    batches of the same workload for ~args.cpu_seconds."""
    import numpy as np
    import oracle
    threads = min(len(os.sched_getaffinity(0)), 16)
    oracle.set_num_threads(threads)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from clouds import gaussian_clouds
    b, n, c, k, r = args.batch, args.points, args.channels, args.k, args.res
    xyz, nrm, feat = gaussian_clouds(b, n, seed=0, c=c)

    def one_batch():
        _, ki = oracle.knn_dir(xyz, xyz, k)
        oracle.local_ppf(xyz, nrm, xyz, nrm, ki, kmajor=True, relative=True)
        nc = oracle.normalize_sph(xyz)
        grid, ind, _ = oracle.spherical_avg_voxelize_forward(feat, nc, r)
        dv, _, _ = oracle.spherical_trilinear_devoxelize_forward(r, nc, grid, ind)
        dv.max(axis=2)

    one_batch()  # warm (page-in, thread pool)
    done, t0 = 0, time.perf_counter()
    while True:
        one_batch()
        done += b
        el = time.perf_counter() - t0
        if el >= args.cpu_seconds:
            break
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    del np
    return {"value": done / el, "unit": "point-clouds/sec", "cores": threads, "kind": "port",
            "sample": "%d clouds (%d x batch %d, N=%d, k=%d, r=%d, C=%d) in %.1f s, "
                      "oracle/pcr_oracle.c OpenMP over clouds, %d threads, %s"
                      % (done, done // b, b, n, k, r, c, el, threads, model)}


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
                                   fused_grid_kernel_bytes_per_cloud,
                                   stream_kernel_bytes_per_cloud)
    b, n, c, k, r = args.batch, args.points, args.channels, args.k, args.res
    xyz, nrm, feat = synthetic_inputs(b, n, c, dev, seed=1234 + rank)
    ex = SphExtractor(b, n, c, k, r, device=dev)

    # S pipelined steps per graph launch (one launch = S batches); S must
    # divide the step counts so exactly --steps steps are timed
    S = max(1, args.steps_per_launch) if args.mode.startswith(("pipelined", "native")) else 1
    if args.steps % S or (args.warmup and args.warmup % S):
        S = 1
    comm = torch.cuda.Stream(device=dev) if world > 1 else None
    desc_out = [torch.empty((world * S * b, c), device=dev) for _ in range(2)]
    desc_in = [torch.empty((S * b, c), device=dev) for _ in range(2)]
    pending = []

    desc_steps = torch.empty((S, b, c), device=dev)
    if args.mode == "graph":
        ex.capture(xyz, nrm, feat)

    def launch(i):
        """Steps i*S .. i*S+S-1."""
        if args.mode.startswith("native"):
            ex.run_native(xyz, nrm, feat, S, desc_steps, schedule=0 if args.mode == "native2" else 1)
            src = desc_steps.view(S * b, c)
        elif args.mode.startswith("pipelined"):
            ex.run_pipelined(xyz, nrm, feat, S, desc_steps,
                             mode={"pipelined": "two_fused", "pipelined_split": "two",
                                   "pipelined3": "three",
                                   "pipelined4": "four", "pipelined_sv": "sortvox",
                                   "pipelined_fs": "four_split", "pipelined_3s": "three_stream",
                                   "pipelined_2s": "two_stream"}[args.mode])
            src = desc_steps.view(S * b, c)
        elif args.mode == "graph":
            ex.replay()
            src = ex.desc
        else:
            ex.forward(xyz, nrm, feat)
            src = ex.desc
        if world > 1:
            # descriptor all-gather of the S batches (registration matching),
            # overlapped with the next launch on a side stream; double-buffered:
            # the gather that last read this slot is waited for before the copy
            slot = i & 1
            if len(pending) == 2:
                pending.pop(0).wait()
            desc_in[slot].copy_(src)
            comm.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(comm):
                pending.append(dist.all_gather_into_tensor(desc_out[slot], desc_in[slot],
                                                           async_op=True))

    for i in range(args.warmup // S):
        launch(i)
    for w in pending:
        w.wait()
    pending.clear()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps // S):
        launch(i)
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

    # dominant kernel, HIP events on the stream it is launched on: the grid
    # stream kernel of the split voxel stage (native) or the fused grid /
    # devox kernel (the other schedules)
    split = args.mode == "native"
    s_k = ex.s_vox
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.kernel_iters)]
    with torch.cuda.stream(s_k):
        for e0, e1 in ev:
            ex.voxel_prep(xyz, s_k.cuda_stream)
            if split:
                ex.voxel_means_devox(feat, s_k.cuda_stream)
                e0.record(s_k)
                ex.voxel_stream(s_k.cuda_stream)
            else:
                e0.record(s_k)
                ex.voxel_grid_devox(feat, s_k.cuda_stream)
            e1.record(s_k)
    torch.cuda.synchronize(dev)
    grid_ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    grid_avg_ms = sum(grid_ms) / len(grid_ms)
    grid_bytes = (stream_kernel_bytes_per_cloud(r, c) if split
                  else fused_grid_kernel_bytes_per_cloud(n, r, c)) * b
    achieved = grid_bytes / (grid_avg_ms * 1e-3) / 1e9
    kname = ("vox_stream_kernel (sph-vox dense grid + cnt from the voxel means, write-through "
             "stores)" if split else
             "vox_grid_kernel<3> (sph-vox dense grid + cnt, sph-devox + descriptor)")

    total_clouds = b * world * args.steps
    value = total_clouds / elapsed
    step_bytes = algorithmic_bytes_per_cloud(n, k, r, c)["total"] * b
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("config") == [b, n, k, r, c] and pm.get("kernel", "") in kname:
                traffic = pm.get("grid_kernel_hbm_bytes_per_launch")
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
        "config": {"workload": "sph-dg extractor forward: self-KNN k=%d + local PPF + "
                               "sph-vox r=%d^3 + sph-devox + descriptor" % (k, r),
                   "clouds_per_gpu": b, "points": n, "k": k, "resolution": r, "channels": c,
                   "global_batch": b * world, "parallelism": "dp%d (clouds sharded, "
                   "descriptor all-gather)" % world, "launch": args.mode,
                   "steps_per_launch": S},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "kernel": kname,
                     "kernel_avg_ms": round(grid_avg_ms, 5),
                     "kernel_bytes_per_launch": grid_bytes},
        "step_algorithmic_GBps": round(step_bytes * world * args.steps / elapsed / 1e9, 1),
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
