"""Diagnostic: per-phase s_memtime stamps of the prep and KNN kernels
(lib/libpcr_amd_diag.so, built with `make -C <pkg>/csrc diag`).  Not part of
the product; prints median cycles per phase over workgroups."""
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
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
lib = _lib.load()
buf = (ctypes.c_ulonglong * (1024 * 16))()
for _ in range(3):
    ex.forward(xyz, nrm, feat)
torch.cuda.synchronize()
s = torch.cuda.current_stream().cuda_stream
for name, fn, reader, nwg in (("vox_prep", lambda: ex.voxel_prep(xyz, s), lib.pcr_diag_read_vox, b),
                              ("vox_grid", lambda: ex.voxel_grid(feat, s), lib.pcr_diag_read_vox, 512),
                              ("vox_devox", lambda: ex.voxel_devox(feat, s), lib.pcr_diag_read_vox, 512),
                              ("vox_fused", lambda: ex.voxel_grid_devox(feat, s), lib.pcr_diag_read_vox, 1024),
                              ("knn", lambda: ex.neighbor_stage(xyz, nrm, s), lib.pcr_diag_read_knn,
                               b * n // 64)):
    fn()
    torch.cuda.synchronize()
    reader(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:min(nwg, 1024)].astype(np.int64)
    print(name, "workgroups", a.shape[0])
    for p in list(range(1, 8)) + list(range(9, 13)):
        d = a[:, p] - a[:, p - 1]
        ok = (a[:, p] > 0) & (a[:, p - 1] > 0)
        if ok.any():
            print("  phase %d->%d: median %d  max %d cycles" % (p - 1, p, np.median(d[ok]), d[ok].max()))
    if name in ("vox_grid", "vox_devox", "vox_fused"):
        t0 = a[:, 8][a[:, 8] > 0]
        t1 = a[:, 12][a[:, 12] > 0]
        print("  kernel span %d cycles; WG durations median %d" % (t1.max() - t0.min(), np.median(t1 - t0)))
    if name == "knn":
        print("  fallback blocks %d of %d; collected keys (lane 0) median %d max %d"
              % (a[:, 8].sum(), a.shape[0], np.median(a[:, 9]), a[:, 9].max()))
