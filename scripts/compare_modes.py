"""Diagnostic: step throughput of the extractor's schedules, interleaved in
one process (three rounds each, medians), so box-to-box variation does not
decide between them.  Not part of the product."""
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
modes = sys.argv[1:] or ["three", "two", "four", "sortvox"]
print("stream priority range", torch.cuda.Stream.priority_range(), flush=True)
plain = (ex.s_nbr, ex.s_vox)
prio = {"hi_knn": (torch.cuda.Stream(device=dev, priority=-1), plain[1]),
        "hi_vox": (plain[0], torch.cuda.Stream(device=dev, priority=-1))}
res = {m: [] for m in modes}
for rnd in range(3):
    for m in modes:
        mm, S = (m.split(":") + ["10"])[:2]
        S = int(S)
        ex.s_nbr, ex.s_vox = plain
        if m in prio:
            ex.s_nbr, ex.s_vox = prio[m]
            mm = "two_fused"
        def go(mm=mm, S=S):
            if mm.startswith("native"):
                ex.run_native(xyz, nrm, feat, S, schedule=int(mm[6:] or 1))
            else:
                ex.run_pipelined(xyz, nrm, feat, S, mode=mm)
        for _ in range(2):
            go()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200 // S):
            go()
        torch.cuda.synchronize()
        res[m].append(b * (200 // S) * S / (time.perf_counter() - t0))
for m, v in res.items():
    v = sorted(v)
    print("%-16s median %.0f clouds/s  (min %.0f max %.0f)" % (m, v[1], v[0], v[2]), flush=True)
