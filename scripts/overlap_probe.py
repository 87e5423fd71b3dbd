"""Diagnostic: how well the extractor's kernels overlap.  Times R launches of
each kernel alone (one stream, back to back), then pairs of kernels on two
streams concurrently (R launches each), and prints the pair time next to the
sum / max of the solo times.  Not part of the product."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
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
sa, sb = ex.s_nbr, ex.s_vox
ok = ex.knn_sort(xyz, sa.cuda_stream)
ex.voxel_prep(xyz, sb.cuda_stream)
torch.cuda.synchronize()
big = torch.empty(b * c * r ** 3, device=dev)


def fill(s):
    with torch.cuda.stream(s):
        big.fill_(0.5)


K = {
    "fill": fill,
    "sort": lambda s: ex.knn_sort(xyz, s.cuda_stream),
    "select": lambda s: ex.knn_select(xyz, nrm, s.cuda_stream, 0, ok),  # + ppf launch
    "prep": lambda s: ex.voxel_prep(xyz, s.cuda_stream),
    "grid": lambda s: ex.voxel_grid_devox(feat, s.cuda_stream),
}
R = 50


def run(fns):
    for f, s in fns:
        for _ in range(3):
            f(s)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(R):
            for f, s in fns:
                f(s)
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / R * 1e6)
    return best


solo = {name: run([(f, sa)]) for name, f in K.items()}
for name, t in solo.items():
    print("solo %-8s %7.1f us" % (name, t), flush=True)
for a, bb in [("select", "fill"), ("fill", "fill"), ("select", "grid"), ("select", "prep"), ("sort", "grid"), ("sort", "prep"),
              ("grid", "grid"), ("select", "select")]:
    t = run([(K[a], sa), (K[bb], sb)])
    print("pair %-7s + %-7s %7.1f us   (sum %6.1f, max %6.1f)" % (
        a, bb, t, solo[a] + solo[bb], max(solo[a], solo[bb])), flush=True)
