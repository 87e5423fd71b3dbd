"""Diagnostic: KNN selection time vs batch (workgroups per CU) -- do two
selection workgroups really share a CU?  Not part of the product."""
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

dev = torch.device("cuda:0")
lib = _lib.load()
for b in (8, 16, 24, 32, 48, 64):
    n, c, k, r = 1024, 64, 32, 32
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = torch.randn((b, 3, n), generator=g, device=dev)
    ex = SphExtractor(b, n, c, k, r, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ex.knn_sort(xyz, s)

    def sel():
        lib.pcr_knn_local_ppf_prepared(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(ex.knn_idx), None,
                                       None, _ptr(ex.knn_ws), ex.knn_ws.numel(), s)
    for _ in range(10):
        sel()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(100):
        sel()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 100
    print("b=%d (%d WGs): %.1f us" % (b, b * 16, dt * 1e6), flush=True)
