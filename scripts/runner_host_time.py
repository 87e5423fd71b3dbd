"""Diagnostic: host time of one pcr_extractor_run call (the enqueue of S
steps from C++) against the GPU time of those steps, c2 ring of 20 batches,
schedule 6.  If the enqueue of the first steps is slower than their
execution, the start of every call waits on the host.  Not part of the
product.  usage: python scripts/runner_host_time.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 40
b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
batches = []
for i in range(20):
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = torch.nn.functional.normalize(torch.randn((b, 3, n), generator=g, device=dev), dim=1)
    feat = torch.rand((b, c, n), generator=g, device=dev) * 2 - 1
    batches.append((xyz.contiguous(), nrm.contiguous(), feat.contiguous()))
ex = SphExtractor(b, n, c, k, r, device=dev)
for _ in range(3):
    ex.run_ring(batches, S, 0, None, schedule=6)
torch.cuda.synchronize()
for rep in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    t0 = time.perf_counter()
    ex.run_ring(batches, S, 0, None, schedule=6)
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    print("steps %d: host enqueue %.3f ms (%.1f us/step), GPU %.3f ms (%.1f us/step)" % (
        S, (t1 - t0) * 1e3, (t1 - t0) * 1e6 / S, e0.elapsed_time(e1), e0.elapsed_time(e1) * 1e3 / S))
