"""Times the KNN selection launch alone (the Morton sort done once before),
HIP events on the launching stream, at BASELINE c2 (32 x 1024, k=32) and the
c3 per-cloud shape (256 x 2048, k=32), and checks the result against the
one-call path.  usage: [CFG=BxNxK,...] python scripts/knn_select_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

from pcr_amd import ops  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

dev = torch.device("cuda:0")
CFG = os.environ.get("CFG")
cfgs = [tuple(int(v) for v in c.split("x")) for c in CFG.split(",")] if CFG else \
    [(32, 1024, 32), (256, 2048, 32), (32, 1024, 16)]
for b, n, k in cfgs:
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
    nrm = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
    ex = SphExtractor(b, n, 8, k, 8, device=dev)
    s = torch.cuda.current_stream()
    ok = ex.knn_sort(xyz, s.cuda_stream)
    ex.knn_select(xyz, nrm, s.cuda_stream, sorted_ok=ok, ppf=False)
    ref, _, _ = ops.knn_local_ppf(xyz, nrm, k)
    torch.cuda.synchronize()
    same = torch.equal(ex.knn_idx, ref)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(20)]
    for e0, e1 in ev:
        e0.record(s)
        ex.knn_select(xyz, nrm, s.cuda_stream, sorted_ok=ok, ppf=False)
        e1.record(s)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    print("select b=%d n=%d k=%d: median %.1f us, min %.1f us, equal to one-call path: %s"
          % (b, n, k, t[len(t) // 2] * 1e3, t[0] * 1e3, same), flush=True)
