"""Per-phase s_memtime stamps of the c2 grid stream (vox_stream_kernel with
the devox role, pcr_extractor_voxel_stream_devox) from the diagnostic
library (`make -C <pkg>/csrc diag`; DIAGLIB names the copy to load), with the
launches rotating over 4 output sets as in the bench's batch ring.  Per
workgroup (256 of them, four items each): the prologue (the loader's first
loads + the word prefix, until the first barrier), then per item the grid
stream, the devox + descriptor role and the wait at the item's barrier.
Not part of the product."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ["PCR_AMD_LIB"] = os.path.join(PKG, "lib", os.environ.get("DIAGLIB", "libpcr_amd_diag.so"))
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
b, n, c, r = 32, 1024, 64, 32
r3 = r ** 3
NB = 4
lib = _lib.load()
g = torch.Generator(device=dev).manual_seed(0)
e = torch.empty
wsb = lib.pcr_extractor_workspace_size(b, n, c, r)
sets = []
st = torch.cuda.current_stream().cuda_stream
for i in range(NB):
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    feat = torch.randn((b, c, n), generator=g, device=dev)
    ws = e((wsb,), dtype=torch.uint8, device=dev)
    nc, ind = e((b, 3, n), device=dev), e((b, n), dtype=torch.int32, device=dev)
    dinds, dwgts = e((b, 8, n), dtype=torch.int32, device=dev), e((b, 8, n), device=dev)
    out = (e((b, r3), dtype=torch.int32, device=dev), e((b, c, r3), device=dev),
           e((b, c, n), device=dev), e((b, c), device=dev))
    _lib.check(lib.pcr_extractor_voxel_prep(_ptr(xyz), b, n, r, _ptr(nc), _ptr(ind), _ptr(dinds),
                                            _ptr(dwgts), _ptr(ws), wsb, st), "prep")
    _lib.check(lib.pcr_extractor_voxel_means(_ptr(feat), b, c, n, r, _ptr(ws), wsb, st), "means")
    sets.append((ws, dwgts, out))


def stream(i):
    ws, dwgts, (cnt, grid, devox, desc) = sets[i % NB]
    _lib.check(lib.pcr_extractor_voxel_stream_devox(b, c, n, r, _ptr(cnt), _ptr(grid), _ptr(devox),
                                                    _ptr(dwgts), _ptr(desc), _ptr(ws), wsb, st),
               "stream")


for i in range(12):
    stream(i)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(20):
    stream(i)
e1.record()
torch.cuda.synchronize()
print("grid stream, 4 sets in turn: %.1f us per launch" % (e0.elapsed_time(e1) / 20 * 1e3))
buf = (ctypes.c_ulonglong * (1024 * 16))()
lib.pcr_diag_read_vox.restype = ctypes.c_int
lib.pcr_diag_read_vox(buf)
s = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:256].astype(np.int64)
clk = 2400.0  # cycles per us (nominal)


def show(name, d):
    print("%-22s median %6.2f us  p10 %6.2f  p90 %6.2f" % (
        name, np.median(d) / clk, np.percentile(d, 10) / clk, np.percentile(d, 90) / clk))


show("prologue", s[:, 1] - s[:, 0])
show("  loader start", s[:, 6] - s[:, 0])
show("  loader loads landed", s[:, 7] - s[:, 6])
show("  prefix + barrier", s[:, 1] - s[:, 7])
prev = s[:, 1]
for it in range(4):
    show("item %d stream" % it, s[:, 12 + it] - prev)
    show("item %d devox" % it, s[:, 2 + it] - s[:, 12 + it])
    show("item %d barrier wait" % it, s[:, 8 + it] - s[:, 2 + it])
    prev = s[:, 8 + it]
show("workgroup total", s[:, 11] - s[:, 0])
