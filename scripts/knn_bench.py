"""Diagnostic: time the fused self-KNN + local PPF launch (neighbour stage of
the extractor) alone, c2 shape, with HIP events; with the diag library
(PCR_AMD_LIB=.../libpcr_amd_diag.so) PCR_KNN_IMPL=1 selects the older
list-merge kernel for comparison.  Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402

b, n, k = int(os.environ.get("B", 32)), int(os.environ.get("N", 1024)), int(os.environ.get("K", 32))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
for want_ppf in (True, False):
    fn = (lambda: ops.knn_local_ppf(xyz, nrm, k)) if want_ppf else (lambda: ops.knn_forward_cuda(xyz, xyz, k))
    ref = fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(30)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    print("impl %s %s: median %.1f us  min %.1f us" % (os.environ.get("PCR_KNN_IMPL", "0"),
          "knn_local_ppf" if want_ppf else "knn_forward(both dirs)", t[len(t) // 2] * 1e3, t[0] * 1e3))
