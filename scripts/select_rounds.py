"""Diagnostic: start / end times of the KNN selection's workgroups (diag
build stamps) -- how many run at once per CU.  Not part of the product."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ.setdefault("PCR_AMD_LIB", os.path.join(PKG, "lib", "libpcr_amd_diag.so"))
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
ex.knn_sort(xyz, s)
for _ in range(3):
    lib.pcr_knn_local_ppf_prepared(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(ex.knn_idx), None, None,
                                   _ptr(ex.knn_ws), ex.knn_ws.numel(), s)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (1024 * 16))()
lib.pcr_diag_read_knn(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:512].astype(np.int64)
t0 = a[:, 0].min()
st = a[:, 0] - t0
en = a[:, 5] - t0
print("WG durations (0->5) median %d cycles" % np.median(a[:, 5] - a[:, 0]))
print("start times (cycles): percentiles 0/25/50/75/90/100:", np.percentile(st, [0, 25, 50, 75, 90, 100]).astype(int))
print("end times:", np.percentile(en, [0, 25, 50, 75, 90, 100]).astype(int))
hist, edges = np.histogram(st, bins=10)
print("start histogram:", list(hist), "bin width", int(edges[1] - edges[0]))
for p in range(1, 6):
    d = a[:, p] - a[:, p - 1]
    print("phase %d->%d median %d" % (p - 1, p, np.median(d)))
# per XCD (workgroup i runs on XCD i % 8; each XCD has its own counter)
for x in range(8):
    sel = np.arange(x, a.shape[0], 8)
    s0 = a[sel, 0] - a[sel, 0].min()
    e0 = a[sel, 5] - a[sel, 0].min()
    print("xcd %d: start pct 0/50/90/100 %s  end max %d" % (
        x, np.percentile(s0, [0, 50, 90, 100]).astype(int), e0.max()))
