"""Timing of the path's share of the BASELINE c3 train step (256 clouds x
2048 points, k = 32, r = 32, C = 64, forward + backward): the fused
extractor forward (KNN + local PPF + sph vox + devox + descriptor, native
runner) and the backward of the devoxelisation and voxelisation (the
gradient the reference computes with atomics).  Conv3d / MLP layers are
outside the path.  HIP events on the launch stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, k, r, c = 256, 2048, 32, 32, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()


def timeit(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


ex = SphExtractor(b, n, c, k, r, device=dev)
t = timeit(lambda: ex.forward(xyz, nrm, feat), it=5)
print("extractor forward                  %.3f ms/step  %.0f clouds/s" % (t, b / t * 1e3), flush=True)
out = ex.outputs()
t = timeit(lambda: ops.knn_local_ppf(xyz, nrm, k))
print("knn + local ppf alone              %.3f ms" % t, flush=True)
nc = ops.spherical_normalize(xyz)
grid, ind, cnt = ops.spherical_avg_voxelize_forward(feat, nc, r)
_, dinds, dwgts = ops.spherical_trilinear_devoxelize_forward(r, True, nc, grid, ind)
gy = torch.randn((b, c, n), generator=g, device=dev)
t = timeit(lambda: ops.spherical_trilinear_devoxelize_backward(gy, dinds, dwgts, r))
print("sph devoxelize backward            %.3f ms  (grad grid %.0f MB written)"
      % (t, b * c * r ** 3 * 4 / 1e6), flush=True)
gg = torch.randn((b, c, r ** 3), generator=g, device=dev)
t = timeit(lambda: ops.spherical_avg_voxelize_backward(gg, ind, cnt))
print("sph voxelize backward              %.3f ms" % t, flush=True)
del out
