"""Timing of the cube (cu-dg) voxelize / devoxelize path at the c3 shape
(256 clouds x 2048 points, r = 32, C = 64), forward and backward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402

b, n, r, c = 256, 2048, 32, 64
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
feat = torch.rand((b, c, n), generator=g, device=dev)
nc = (xyz - xyz.mean(2, keepdim=True) + 1) / 2
nc = torch.clamp(nc * r, 0, r - 1).contiguous()
vox = torch.round(nc).int().contiguous()


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


print("cube voxelize fwd      %.3f ms" % timeit(lambda: ops.avg_voxelize_forward(feat, vox, r)))
grid, ind, cnt = ops.avg_voxelize_forward(feat, vox, r)
print("cube devoxelize fwd    %.3f ms" % timeit(lambda: ops.trilinear_devoxelize_forward(r, True, nc, grid)))
_, inds, wgts = ops.trilinear_devoxelize_forward(r, True, nc, grid)
gy = torch.randn((b, c, n), generator=g, device=dev)
print("cube devoxelize bwd    %.3f ms" % timeit(lambda: ops.trilinear_devoxelize_backward(gy, inds, wgts, r)))
gg = torch.randn((b, c, r ** 3), generator=g, device=dev)
print("cube voxelize bwd      %.3f ms" % timeit(lambda: ops.avg_voxelize_backward(gg, ind, cnt)))
