"""Is the c2 runner call host-enqueue bound at its start?  For a runner call
of S steps (bench's ExtractWorkload, driver flags: 20 steps):
  host    wall time of the pcr_extractor_run call itself (enqueue only)
  wall    wall time of the call + synchronize (what bench.py times)
  gated   GPU time of the same call when every launch is enqueued before the
          GPU starts (a spin kernel holds the origin stream; HIP events after
          it and after the join)
usage: [STEPS=20[,S2,...]] [REPS=8] python scripts/host_enqueue_probe.py [bench args]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from pcr_amd import _lib as bench_lib  # noqa: E402

SS = [int(x) for x in os.environ.get("STEPS", "20").split(",")]
REPS = int(os.environ.get("REPS", "8"))
args = bench.parse(sys.argv[1:] + ["--no-verify", "--no-cpu-baseline", "--no-kernel-timing"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
wl = bench.WORKLOADS[args.workload](args, dev, 0, 1)
wl.run(40, timed=False)
torch.cuda.synchronize()
cur = torch.cuda.current_stream()
for S in SS:
    host, wall, gated, wall_cold = [], [], [], []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wl.run(S, timed=False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
        # the batches re-checked and re-keyed (run_ring's cache dropped)
        wl.ex._ring_seen = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wl.run(S, timed=False)
        torch.cuda.synchronize()
        wall_cold.append((time.perf_counter() - t0) * 1e3)
        # gated: a spin kernel on the origin stream, then the whole call enqueued
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(40_000_000)
        e0.record(cur)
        wl.run(S, timed=False)
        e1.record(cur)
        torch.cuda.synchronize()
        gated.append(e0.elapsed_time(e1))
    for name, v in (("host", host), ("wall", wall), ("wcold", wall_cold), ("gated", gated)):
        v = sorted(v)
        print("S %3d %-6s ms per call: median %.3f  min %.3f  (%.1f us per step median)" % (
            S, name, v[len(v) // 2], v[0], v[len(v) // 2] * 1e3 / S), flush=True)

# the host prologue of one call, piece by piece (us, median of 200)
ex = wl.ex


def med(fn, n=200):
    v = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        v.append((time.perf_counter() - t0) * 1e6)
    return sorted(v)[n // 2]


print("check_inputs x R   %.1f us" % med(lambda: [ex._check_inputs(*t) for t in wl.batches]))
print("ring_outputs       %.1f us" % med(lambda: ex.ring_outputs(wl.R, 0)))
print("args key           %.1f us" % med(
    lambda: ("ring", tuple(tuple(x.data_ptr() for x in t) for t in wl.batches), None)))
print("current_stream     %.1f us" % med(lambda: torch.cuda.current_stream(dev).cuda_stream))
print("lib.load           %.1f us" % med(lambda: bench_lib.load()))

# the same call captured once into a hipGraph (torch.cuda.graph), replayed
for S in SS:
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        wl.run(S, timed=False)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    host, wall = [], []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    for name, v in (("ghost", host), ("gwall", wall)):
        v = sorted(v)
        print("S %3d %-6s ms per call: median %.3f  min %.3f  (%.1f us per step median)" % (
            S, name, v[len(v) // 2], v[0], v[len(v) // 2] * 1e3 / S), flush=True)

# a short spin on the origin stream in front of the call (the host enqueues
# during it): wall minus the spin's own duration, against the spin length
for S in SS:
    for cyc in (0, 50_000, 100_000, 200_000, 400_000, 800_000):
        spin = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            if cyc:
                torch.cuda._sleep(cyc)
            e1.record(cur)
            torch.cuda.synchronize()
            spin.append(e0.elapsed_time(e1))
        sp = sorted(spin)[2]
        walls = []
        for _ in range(REPS):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if cyc:
                torch.cuda._sleep(cyc)
            wl.run(S, timed=False)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e3)
        w = sorted(walls)[len(walls) // 2]
        print("S %3d spin %7d cycles = %.3f ms: wall %.3f, wall - spin %.3f ms" % (
            S, cyc, sp, w, w - sp), flush=True)

# bench.py's timed call: a 5-step call, synchronize, then the S-step call
# with its grid launches of KT steps bracketed by timing events (KT = 0:
# untimed), interleaved
ex.reserve_timing(4)
wl.args.no_kernel_timing = False
res = {0: [], 2: [], 4: []}
for _ in range(REPS):
    for kt in (0, 2, 4):
        wl.KTIMED = kt
        wl.run(5, timed=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        wl.run(S, timed=kt > 0)
        torch.cuda.synchronize()
        res[kt].append((time.perf_counter() - t0) * 1e3)
for kt, v in res.items():
    v = sorted(v)
    print("S %3d timed grid launches %d: wall median %.3f  min %.3f ms" % (
        S, kt, v[len(v) // 2], v[0]), flush=True)
