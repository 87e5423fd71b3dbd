"""Diagnostic: the spherical devoxelize backward at the c3 shape (256 x 2048
points, C = 64, r = 32) with and without the per-cloud corner-set order
(pcr_devoxelize_backward_ws vs pcr_devoxelize_backward), HIP events."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from clouds import gaussian_clouds  # noqa: E402
from pcr_amd import _lib, ops  # noqa: E402
from pcr_amd.ops import _ptr, _stream  # noqa: E402

dev = torch.device("cuda:0")
b, n, c, r = 256, 2048, 64, 32
xyz, _, feat = [torch.from_numpy(a).to(dev) for a in gaussian_clouds(b, n, seed=3, c=c)]
nc = ops.spherical_normalize(xyz)
grid, ind, cnt = ops.spherical_avg_voxelize_forward(feat, nc, r)
_, dinds, dwgts = ops.spherical_trilinear_devoxelize_forward(r, False, nc, grid, ind)
gy = torch.randn((b, c, n), device=dev)
lib = _lib.load()
gx_old = torch.empty((b, c, r ** 3), device=dev)


def old():
    _lib.check(lib.pcr_devoxelize_backward(_ptr(gy), _ptr(dinds), _ptr(dwgts), b, c, n, r, 1,
                                           _ptr(gx_old), _stream()), "old")


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t_old = timeit(old)
t_new = timeit(lambda: ops.spherical_trilinear_devoxelize_backward(gy, dinds, dwgts, r))
gx_new = ops.spherical_trilinear_devoxelize_backward(gy, dinds, dwgts, r)
old()
torch.cuda.synchronize()
d = (gx_new - gx_old).abs().max().item()
print("sph devox backward c3: per-wave sort %.3f ms, per-cloud order %.3f ms, max |diff| %.2e"
      % (t_old, t_new, d))
