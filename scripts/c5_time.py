"""Diagnostic: wall time of the c5-shaped path (8 x 65,536 points, k = 64,
r = 64, C = 64): KNN + local PPF, normalisation, voxelisation,
devoxelisation.  Not part of the product."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402

b, n, k, r, c = int(os.environ.get("B", 8)), 65536, 64, 64, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
feat = torch.rand((b, c, n), generator=g, device=dev)


def t(label, fn, reps=3):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    print("%-28s %.2f ms" % (label, (time.perf_counter() - t0) / reps * 1e3), flush=True)
    return out


t("knn + local ppf (k=64)", lambda: ops.knn_local_ppf(xyz, nrm, k))
nc = t("normalize", lambda: ops.spherical_normalize(xyz))
out, ind, cnt = t("sph voxelize r=64", lambda: ops.spherical_avg_voxelize_forward(feat, nc, r))
t("sph devoxelize", lambda: ops.spherical_trilinear_devoxelize_forward(r, False, nc, out, ind))
