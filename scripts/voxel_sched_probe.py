"""Probe of the c2 voxel chain alone (no KNN chain): how fast can the voxel
side go, and how do two grid streams share HBM?  At BASELINE c2 (32 x 1024,
C = 64, r = 32), HIP events on the caller's stream around S steps:
  one     one grid stream launch (pcr_extractor_voxel_stream_devox) at a time,
          NB output sets in turn (no Infinity-Cache reuse of the grid lines)
  onenodv the same without the devox role (pcr_extractor_voxel_stream; the
          devox then comes from the means launch, not timed here)
  same    one grid stream launch at a time into the SAME output set
  two     two grid stream launches at once, on two streams
  sched6  the runner's voxel chains only: prep -> means -> stream of step s on
          queue s % 2 with workspace s % 2 (schedule 6 without the KNN chain)
  split   every grid stream on queue 0 in order, the heads (prep -> means) of
          step s + 1 on queue 1 ahead of step s's stream (two workspaces)
usage: [STEPS=40] python scripts/voxel_sched_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
S = int(os.environ.get("STEPS", "40"))
b, n, c, r = 32, 1024, 64, 32
r3 = r ** 3
lib = _lib.load()
g = torch.Generator(device=dev).manual_seed(0)
NB = 4  # distinct batches / output sets
xyz = [torch.randn((b, 3, n), generator=g, device=dev) for _ in range(NB)]
feat = [torch.randn((b, c, n), generator=g, device=dev) for _ in range(NB)]
e = torch.empty
wsb = lib.pcr_extractor_workspace_size(b, n, c, r)
ws = [e((wsb,), dtype=torch.uint8, device=dev) for _ in range(2)]
nc = [e((b, 3, n), device=dev) for _ in range(NB)]
ind = [e((b, n), dtype=torch.int32, device=dev) for _ in range(NB)]
dinds = [e((b, 8, n), dtype=torch.int32, device=dev) for _ in range(NB)]
dwgts = [e((b, 8, n), device=dev) for _ in range(NB)]
cnt = [e((b, r3), dtype=torch.int32, device=dev) for _ in range(NB)]
grid = [e((b, c, r3), device=dev) for _ in range(NB)]
devox = [e((b, c, n), device=dev) for _ in range(NB)]
desc = [e((b, c), device=dev) for _ in range(NB)]
q = [torch.cuda.Stream(device=dev) for _ in range(2)]
cur = torch.cuda.current_stream()


def prep(s, w, st):
    _lib.check(lib.pcr_extractor_voxel_prep(_ptr(xyz[s % NB]), b, n, r, _ptr(nc[s % NB]),
                                            _ptr(ind[s % NB]), _ptr(dinds[s % NB]),
                                            _ptr(dwgts[s % NB]), _ptr(ws[w]), wsb, st), "prep")


def means(s, w, st):
    _lib.check(lib.pcr_extractor_voxel_means(_ptr(feat[s % NB]), b, c, n, r, _ptr(ws[w]), wsb,
                                             st), "means")


def stream(s, w, st):
    i = s % NB
    _lib.check(lib.pcr_extractor_voxel_stream_devox(b, c, n, r, _ptr(cnt[i]), _ptr(grid[i]),
                                                    _ptr(devox[i]), _ptr(dwgts[i]), _ptr(desc[i]),
                                                    _ptr(ws[w]), wsb, st), "stream")


def timed(fn, reps=3):
    best = None
    for _ in range(reps):
        for st in q:
            st.wait_stream(cur)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        for st in q:
            st.wait_event(e0)
        fn()
        for st in q:
            cur.wait_stream(st)
        e1.record(cur)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1000.0 / S
        best = t if best is None else min(best, t)
    return best


# every workspace / set prepared once (the stream-only probes reuse them)
for s in range(2):
    prep(s, s, cur.cuda_stream)
    means(s, s, cur.cuda_stream)
torch.cuda.synchronize()


def one():
    for s in range(S):
        stream(s % NB, s % 2, q[0].cuda_stream)


def onenodv():
    for s in range(S):
        i = s % NB
        _lib.check(lib.pcr_extractor_voxel_stream(b, c, n, r, _ptr(cnt[i]), _ptr(grid[i]),
                                                  _ptr(ws[s % 2]), wsb, q[0].cuda_stream),
                   "stream")


def same():
    for s in range(S):
        stream(0, 0, q[0].cuda_stream)


def two():
    for s in range(S):
        stream(s % 2, s % 2, q[s % 2].cuda_stream)


def sched6():
    for s in range(S):
        st = q[s % 2].cuda_stream
        prep(s, s % 2, st)
        means(s, s % 2, st)
        stream(s, s % 2, st)


def split():
    # heads on q[1], streams on q[0]; head s + 2 reuses workspace s % 2 only
    # after stream s is done with it
    done = [None, None]
    ready = []
    for s in range(S + 1):
        if s < S:
            if done[s % 2] is not None:
                q[1].wait_event(done[s % 2])
            prep(s, s % 2, q[1].cuda_stream)
            means(s, s % 2, q[1].cuda_stream)
            ev = torch.cuda.Event()
            ev.record(q[1])
            ready.append(ev)
        if s >= 1:
            t = s - 1
            q[0].wait_event(ready[t])
            stream(t, t % 2, q[0].cuda_stream)
            ev = torch.cuda.Event()
            ev.record(q[0])
            done[t % 2] = ev


for name, fn in (("one", one), ("onenodv", onenodv), ("same", same), ("two", two),
                 ("sched6", sched6)):
    fn()  # warm-up
    t = timed(fn)
    print("%-7s %7.1f us per step  (%.2f TB/s of grid + cnt + devox stream bytes)" % (
        name, t, (b * (4 * c * r3 + 4 * r3 + 4 * c * n + 64 * n + 4 * c)) / (t * 1e-6) / 1e12),
        flush=True)
