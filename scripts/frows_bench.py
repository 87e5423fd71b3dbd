"""Timings of the SURVEY.md 8f kernels on one MI355X (diagnostic, not the
bench): LRF change_coords, FPS, 3-NN interpolate, gather, normal estimation,
each at a c2-like shape (32 clouds x 1024 points) and a larger one, with the
bound each is measured against.  HIP-event timing on the launch stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
HBM = 8.0e12


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e-3


def report(name, t, nbytes=None, extra=""):
    s = "%-44s %9.1f us" % (name, t * 1e6)
    if nbytes:
        s += "  %7.1f GB/s (%.0f%% of HBM)" % (nbytes / t / 1e9, 100 * nbytes / t / HBM)
    print(s + ("  " + extra if extra else ""), flush=True)


g = torch.Generator(device=dev).manual_seed(0)
for b, n in ((32, 1024), (256, 2048), (8, 65536)):
    x = torch.randn((b, 3, n), device=dev, generator=g)
    t = timeit(lambda: ops.lrf_change_coords(x, check=False))
    report("lrf_change_coords b=%d n=%d" % (b, n), t, 24 * b * n,
           "%.0f clouds/s" % (b / t))
for b, n, m in ((32, 1024, 512), (32, 2048, 512), (8, 16384, 1024)):
    x = torch.randn((b, 3, n), device=dev, generator=g)
    t = timeit(lambda: ops.furthest_point_sampling(x, m), it=10)
    report("furthest_point_sampling b=%d n=%d m=%d" % (b, n, m), t, None,
           "%.2f us/sample step" % (t / m * 1e6))
for b, c, m, n in ((32, 64, 256, 1024), (32, 128, 512, 2048)):
    pts = torch.randn((b, 3, n), device=dev, generator=g)
    ctr = torch.randn((b, 3, m), device=dev, generator=g)
    cf = torch.randn((b, c, m), device=dev, generator=g)
    t = timeit(lambda: ops.three_nearest_neighbors_interpolate_forward(pts, ctr, cf))
    report("three_nn_interpolate b=%d c=%d m=%d n=%d" % (b, c, m, n), t,
           4 * b * (3 * n + 3 * m + c * m + c * n + 6 * n),
           "%.1f Gpairs/s" % (b * n * m / t / 1e9))
    f = torch.randn((b, c, n), device=dev, generator=g)
    idx = torch.randint(0, n, (b, m), device=dev, dtype=torch.int32, generator=g)
    t = timeit(lambda: ops.gather_features_forward(f, idx))
    report("gather_features b=%d c=%d n=%d m=%d" % (b, c, n, m), t, 4 * b * (m + 2 * c * m))
for b, n, r in ((32, 1024, 0.1), (32, 2048, 0.1), (8, 16384, 0.05)):
    v = torch.randn((b, 3, n), device=dev, generator=g)
    v = 0.5 * v / v.norm(dim=1, keepdim=True)
    t = timeit(lambda: ops.estimate_normals(v, r), it=20)
    report("estimate_normals b=%d n=%d r=%.2f" % (b, n, r), t, None,
           "%.0f clouds/s, %.1f G candidate tests/s" % (b / t, b * n * n / t / 1e9))
