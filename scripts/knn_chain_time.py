"""Times the extractor's KNN chain launch by launch, alone on the GPU (HIP
events on the launching stream): the Morton sort (pcr_knn_prepare), the
selection in sorted query order (pcr_knn_select_sorted) and the local PPF
that un-permutes it (pcr_knn_ppf_sorted), at BASELINE c2 (32 x 1024, k=32)
and the c3 per-cloud shape (256 x 2048, k=32); checks the chain's idx / PPF
against the one-call knn_local_ppf path.
usage: [CFG=BxNxK,...] python scripts/knn_chain_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

from pcr_amd import _lib, ops  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
CFG = os.environ.get("CFG")
cfgs = [tuple(int(v) for v in c.split("x")) for c in CFG.split(",")] if CFG else \
    [(32, 1024, 32), (256, 2048, 32), (32, 1024, 16)]
lib = _lib.load()
for b, n, k in cfgs:
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
    nrm = torch.randn((b, 3, n), generator=g, device=dev)
    nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
    ws = torch.zeros((lib.pcr_knn_workspace_size(b, n, n),), dtype=torch.uint8, device=dev)
    idx = torch.zeros((b, k, n), dtype=torch.int32, device=dev)
    ppf = torch.zeros((b, 4, k, n), device=dev)
    s = torch.cuda.current_stream()
    st = s.cuda_stream

    def sort():
        _lib.check(lib.pcr_knn_prepare(_ptr(xyz), b, n, _ptr(ws), ws.numel(), st), "prepare")

    def select():
        _lib.check(lib.pcr_knn_select_sorted(_ptr(xyz), b, n, k, _ptr(ws), ws.numel(), st),
                   "select_sorted")

    def ppf_launch():
        _lib.check(lib.pcr_knn_ppf_sorted(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(idx), _ptr(ppf),
                                          _ptr(ws), ws.numel(), st), "ppf_sorted")

    sort()
    select()
    ppf_launch()
    ref_i, ref_p, _ = ops.knn_local_ppf(xyz, nrm, k)
    torch.cuda.synchronize()
    same = torch.equal(idx, ref_i) and torch.equal(torch.nan_to_num(ppf, 7.0),
                                                   torch.nan_to_num(ref_p, 7.0))
    res = {}
    for name, f in (("sort", sort), ("select", select), ("ppf", ppf_launch)):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(30)]
        for e0, e1 in ev:
            e0.record(s)
            f()
            e1.record(s)
        torch.cuda.synchronize()
        t = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
        res[name] = (t[len(t) // 2] * 1e3, t[0] * 1e3)
    # the three back to back, as in a step
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        sort()
        select()
        ppf_launch()
    e1.record(s)
    torch.cuda.synchronize()
    chain = e0.elapsed_time(e1) * 1e3 / 20
    print("b=%d n=%d k=%d: " % (b, n, k) +
          "  ".join("%s median %.1f us (min %.1f)" % (nm, v[0], v[1]) for nm, v in res.items()) +
          "  chain %.1f us/step  matches one-call path: %s" % (chain, same), flush=True)
