"""Diagnostic: phase cycles and work counters (wave 0 of each workgroup:
flushes, processed candidate blocks) of the KNN block kernel on one c5 cloud
(65,536 points, k = 64).  Uses lib/libpcr_amd_diag.so (make diag)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ.setdefault("PCR_AMD_LIB", os.path.join(PKG, "lib", "libpcr_amd_diag.so"))
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pcr_amd import _lib, ops  # noqa: E402

dev = torch.device("cuda:0")
n, k = int(os.environ.get("N", 65536)), int(os.environ.get("K", 64))
g = torch.Generator(device=dev).manual_seed(0)
B = int(os.environ.get("B", 1))
xyz = torch.randn((B, 3, n), generator=g, device=dev)
nrm = torch.randn((B, 3, n), generator=g, device=dev)
lib = _lib.load()
buf = (ctypes.c_ulonglong * (1024 * 16))()
ops.knn_local_ppf(xyz, nrm, k)
torch.cuda.synchronize()
ops.knn_local_ppf(xyz, nrm, k)
torch.cuda.synchronize()
lib.pcr_diag_read_knn(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.int64)
ok = a[:, 1] > 0
d = a[ok, 1] - a[ok, 0]
for p in range(1, 7):
    okp = (a[:, p] > 0) & (a[:, p - 1] > 0)
    if okp.any():
        print("phase %d->%d: median %d cycles" % (p - 1, p, np.median(a[okp, p] - a[okp, p - 1])))
print("workgroups with stamps", ok.sum())
print("scan cycles: median %d  p90 %d  max %d" % (np.median(d), np.percentile(d, 90), d.max()))
names = (("flushes", 8), ("blocks processed", 9)) if os.environ.get("IMPL") == "block" else \
    (("fallback (select)", 8), ("collected keys (select)", 9),
     ("blocks visited by wave 0 in the count pass (select)", 10))
for name, col in names:
    v = a[ok, col]
    print("%s per wave: median %d  p90 %d  max %d  (of %d blocks)" %
          (name, np.median(v), np.percentile(v, 90), v.max(), (n + 63) // 64))
