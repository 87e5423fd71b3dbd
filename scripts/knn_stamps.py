"""Per-phase s_memtime stamps of the KNN selection at BASELINE c2, or c5 with
C5=1 (diagnostic library lib/libpcr_amd_diag.so, `make -C <pkg>/csrc diag`).
Phases: 0->1 bound, 1->2 count, 2->3 cut + collect, 3->4 rank, 4->5 scatter.
Only the first 1024 workgroups are stamped (c5: cloud 0).  Not part of the
product."""
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
from pcr_amd.extractor import SphExtractor  # noqa: E402

C5 = os.environ.get("C5") == "1"
b, n, k = (8, 65536, 64) if C5 else (int(os.environ.get("B", 32)), int(os.environ.get("N", 1024)), 32)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
nrm = torch.randn((b, 3, n), generator=g, device=dev)
if C5:
    from pcr_amd import ops  # noqa: E402
    for _ in range(2):
        ops.knn_local_ppf(xyz, nrm, k)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        ops.knn_local_ppf(xyz, nrm, k)
    e1.record()
    torch.cuda.synchronize()
    print("c5 knn_local_ppf: %.3f ms per call (incl. sort)" % (e0.elapsed_time(e1) / 5))
else:
    ex = SphExtractor(b, n, 8, k, 8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ok = ex.knn_sort(xyz, s)
    for _ in range(3):
        ex.knn_select(xyz, nrm, s, sorted_ok=ok, ppf=False)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (1024 * 16))()
_lib.load().pcr_diag_read_knn(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16).astype(np.int64)
nwg = min(1024, b * ((n + 63) // 64))
a = a[:nwg]
for p in range(1, 7):
    d = a[:, p] - a[:, p - 1]
    okp = (a[:, p] > 0) & (a[:, p - 1] > 0)
    if okp.any():
        print("phase %d->%d: median %d max %d cycles" % (p - 1, p, np.median(d[okp]), d[okp].max()))
t0 = a[:, 0][a[:, 0] > 0]
t5 = a[:, 6][a[:, 6] > 0] if (a[:, 6] > 0).any() else a[:, 5][a[:, 5] > 0]
fb = a[:, 8]
for code in sorted(set(int(v) for v in fb if v)):
    w = np.where(fb == code)[0]
    print("cut flags %d (1 no bound, 2 cut below range, 4 over capacity, 8 refined): "
          "%d workgroups, first %s" % (code, len(w), [int(v) for v in w[:6]]))
nv = a[:, 10]
print("wave-0 visited blocks (all passes): median %d p90 %d max %d" % (
    np.median(nv), np.percentile(nv, 90), nv.max()))
print("span %d cycles over %d workgroups" % (t5.max() - t0.min(), nwg))
rt = (a[:, 15] - a[:, 14]).astype(np.float64)
cy = (a[:, 6] - a[:, 0]).astype(np.float64)
okr = (a[:, 15] > 0) & (a[:, 14] > 0) & (a[:, 6] > 0)
if not okr.any():  # sorted-key emission ends at stamp 5
    cy = (a[:, 5] - a[:, 0]).astype(np.float64)
    okr = (a[:, 15] > 0) & (a[:, 14] > 0) & (a[:, 5] > 0)
if okr.any():
    print("shader clock (s_memtime / s_memrealtime at 100 MHz): median %.0f MHz; "
          "phase 0->6 median %.1f us" % (np.median(cy[okr] / rt[okr]) * 100,
                                         np.median(rt[okr]) / 100.0))
    t14, t15 = a[:, 14][okr], a[:, 15][okr]
    print("realtime span of stamped phases over workgroups: %.1f us" % ((t15.max() - t14.min()) / 100.0))

# per-wave count / collect times and visits (diagnostic library only)
try:
    wbuf = (ctypes.c_ulonglong * (1024 * 8 * 8))()
    _lib.load().pcr_diag_read_knn_wave(wbuf)
    w = np.frombuffer(wbuf, dtype=np.uint64).reshape(1024, 8, 8).astype(np.int64)[:nwg]
    ok = (w[:, :, 0] > 0).all(1) & (a[:, 1] > 0)
    if ok.any():
        cnt_t = w[ok, :, 0] - a[ok, 1][:, None]
        col_t = w[ok, :, 2] - w[ok, :, 4]
        for name, t, v in (("count", cnt_t, w[ok, :, 1]), ("collect", col_t, w[ok, :, 3])):
            print("%s: wave time median %d, max/mean over a workgroup's waves median %.2f; "
                  "visits per wave mean %.1f max %.1f; cycles per visit (sum t / sum v) %.0f" % (
                      name, np.median(t), np.median(t.max(1) / np.maximum(t.mean(1), 1)),
                      v.mean(), v.max(1).mean(), t.sum() / max(v.sum(), 1)))
except AttributeError:
    pass
