"""Diagnostic: host time to enqueue the pipelined schedules vs the GPU time
of the same steps (is the step host-bound?).  Not part of the product."""
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
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
for mode in sys.argv[1:] or ["two_fused", "three_stream"]:
    def go(mode=mode):
        if mode.startswith("native"):
            ex.run_native(xyz, nrm, feat, 50, schedule=int(mode[6:] or 1))
        else:
            ex.run_pipelined(xyz, nrm, feat, 50, mode=mode)
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    go()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%-14s host enqueue %.1f us/step, total %.1f us/step" % (mode, (t1 - t0) / 50 * 1e6,
                                                                   (t2 - t0) / 50 * 1e6), flush=True)
