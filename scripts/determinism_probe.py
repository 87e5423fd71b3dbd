"""Diagnostic: runs the extractor forward (c2 shape and the c3 per-cloud shape),
the one-call KNN + local PPF, ball query, the voxelize forwards and the
devoxelize / voxelize backwards (spherical and cube) many times on the same
inputs and reports any output that is not bit-identical to the first run
(every output here has a fixed summation order, so any difference is a
race).  usage: python scripts/determinism_probe.py [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from clouds import gaussian_clouds  # noqa: E402
from pcr_amd import ops  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")


def probe(name, fn):
    ref = [t.clone() for t in fn() if t is not None]
    bad = 0
    for _ in range(reps):
        out = [t for t in fn() if t is not None]
        if any(not torch.equal(a, b) and not (torch.isnan(a).any() and
               torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))) for a, b in zip(out, ref)):
            bad += 1
    print("%-34s %d of %d runs differ" % (name, bad, reps), flush=True)
    return bad


total = 0
for b, n in ((32, 1024), (8, 2048)):
    xyz, nrm, feat = [torch.from_numpy(a).to(dev) for a in gaussian_clouds(b, n, seed=5, c=64)]
    ex = SphExtractor(b, n, 64, 32, 32, device=dev)
    total += probe("extractor forward %dx%d" % (b, n),
                   lambda: list(ex.forward(xyz, nrm, feat).values()))
    total += probe("knn + local ppf %dx%d" % (b, n),
                   lambda: list(ops.knn_local_ppf(xyz, nrm, 32)))
    total += probe("ball query %dx%d" % (b, n),
                   lambda: [ops.ball_query(xyz, xyz, 0.3, 128)])
    nc = ops.spherical_normalize(xyz)
    total += probe("sph voxelize %dx%d" % (b, n),
                   lambda: list(ops.spherical_avg_voxelize_forward(feat, nc, 32)))
    grid, ind, cnt = ops.spherical_avg_voxelize_forward(feat, nc, 32)
    _, dinds, dwgts = ops.spherical_trilinear_devoxelize_forward(32, True, nc, grid, ind)
    gy = torch.randn(feat.shape, generator=torch.Generator(device=dev).manual_seed(3), device=dev)
    total += probe("sph devox backward %dx%d" % (b, n),
                   lambda: [ops.spherical_trilinear_devoxelize_backward(gy, dinds, dwgts, 32)])
    total += probe("sph vox backward %dx%d" % (b, n),
                   lambda: [ops.spherical_avg_voxelize_backward(grid, ind, cnt)])
    cc = ((xyz - xyz.mean(2, keepdim=True) + 1) / 2 * 32).clamp(0, 31).contiguous()
    _, cinds, cwgts = ops.trilinear_devoxelize_forward(32, True, cc, grid)
    total += probe("cube devox backward %dx%d" % (b, n),
                   lambda: [ops.trilinear_devoxelize_backward(gy, cinds, cwgts, 32)])
print("total differing runs:", total)
sys.exit(1 if total else 0)
