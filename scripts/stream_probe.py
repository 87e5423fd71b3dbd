"""Diagnostic: step throughput of each half of the two-stream schedule on its
own (KNN side: sort + select + PPF; voxel side: prep + fused grid/devox) and
of individual kernels back to back, to see how much the halves slow each
other down.  Not part of the product."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402
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
sn, sv = ex.s_nbr, ex.s_vox


def ppf(st):
    _lib.check(lib.pcr_local_ppf_forward(_ptr(xyz), _ptr(nrm), _ptr(xyz), _ptr(nrm),
                                         _ptr(ex.knn_idx), b, n, n, k, 1, 1,
                                         _ptr(ex.local_ppf), st), "ppf")


def sel(st):
    lib.pcr_knn_local_ppf_prepared(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(ex.knn_idx), None,
                                   None, _ptr(ex.knn_ws), ex.knn_ws.numel(), st)


steps = {
    "nbr": lambda: (ex.knn_sort(xyz, sn.cuda_stream), ex.knn_select(xyz, nrm, sn.cuda_stream)),
    "vox": lambda: ex.voxel_stage(xyz, feat, sv.cuda_stream),
    "both": lambda: (ex.knn_sort(xyz, sn.cuda_stream), ex.knn_select(xyz, nrm, sn.cuda_stream),
                     ex.voxel_stage(xyz, feat, sv.cuda_stream)),
    "sort": lambda: ex.knn_sort(xyz, sn.cuda_stream),
    "select": lambda: sel(sn.cuda_stream),
    "ppf": lambda: ppf(sn.cuda_stream),
    "prep": lambda: ex.voxel_prep(xyz, sv.cuda_stream),
    "grid": lambda: ex.voxel_grid_devox(feat, sv.cuda_stream),
    "sel+grid": lambda: (sel(sn.cuda_stream), ex.voxel_grid_devox(feat, sv.cuda_stream)),
    "ppf+grid": lambda: (ppf(sn.cuda_stream), ex.voxel_grid_devox(feat, sv.cuda_stream)),
    "stream": lambda: ex.voxel_stream(sv.cuda_stream),
    "stream+sel": lambda: (ex.voxel_stream(sv.cuda_stream), sel(sn.cuda_stream)),
    "ppf+stream": lambda: (ppf(sn.cuda_stream), ex.voxel_stream(sv.cuda_stream)),
    "means": lambda: ex.voxel_means_devox(feat, sv.cuda_stream),
    "sel+stream": lambda: (sel(sn.cuda_stream), ex.voxel_stream(sv.cuda_stream)),
    "vox2": lambda: (ex.voxel_prep(xyz, sv.cuda_stream), ex.voxel_means_devox(feat, sv.cuda_stream),
                     ex.voxel_stream(sv.cuda_stream)),
    "both2": lambda: (ex.knn_sort(xyz, sn.cuda_stream), ex.knn_select(xyz, nrm, sn.cuda_stream),
                      ex.voxel_prep(xyz, sv.cuda_stream), ex.voxel_means_devox(feat, sv.cuda_stream),
                      ex.voxel_stream(sv.cuda_stream)),
    "sel+prep": lambda: (sel(sn.cuda_stream), ex.voxel_prep(xyz, sv.cuda_stream)),
}
names = sys.argv[1:] or list(steps)
ex.forward(xyz, nrm, feat)
torch.cuda.synchronize()
for name in names:
    f = steps[name]
    for _ in range(20):
        f()
    torch.cuda.synchronize()
    best = 1e9
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(200):
            f()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / 200)
    print("%-10s %7.1f us/step  %7.0f clouds/s" % (name, best * 1e6, b / best), flush=True)
