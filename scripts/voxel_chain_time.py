"""Times the extractor's voxel chain launch by launch, alone on the GPU (HIP
events on the launching stream) at BASELINE c2 (32 x 1024, C = 64, r = 32):
prep (pcr_extractor_voxel_prep), the means launch (pcr_extractor_voxel_means)
and the grid stream from those means (pcr_extractor_voxel_stream_devox); the
round-6 grid stream that formed the means itself was timed with it
(profiles/r06_ab_stream_means.log).
Clouds past the stream's devox role (c3) time prep, the means + devox launch
and the grid stream without devox.
usage: [CFG=BxNxCxR,...] python scripts/voxel_chain_time.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
CFG = os.environ.get("CFG")
cfgs = [tuple(int(v) for v in c.split("x")) for c in CFG.split(",")] if CFG else \
    [(32, 1024, 64, 32)]
lib = _lib.load()
for b, n, c, r in cfgs:
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev).contiguous()
    feat = torch.randn((b, c, n), generator=g, device=dev).contiguous()
    r3 = r ** 3
    ws = torch.zeros((lib.pcr_extractor_workspace_size(b, n, c, r),), dtype=torch.uint8,
                     device=dev)
    e = torch.empty
    nc, ind = e((b, 3, n), device=dev), e((b, n), dtype=torch.int32, device=dev)
    dinds, dwgts = e((b, 8, n), dtype=torch.int32, device=dev), e((b, 8, n), device=dev)
    outs = [(e((b, r3), dtype=torch.int32, device=dev), e((b, c, r3), device=dev),
             e((b, c, n), device=dev), e((b, c), device=dev)) for _ in range(1)]
    s = torch.cuda.current_stream()
    st = s.cuda_stream

    def prep():
        _lib.check(lib.pcr_extractor_voxel_prep(_ptr(xyz), b, n, r, _ptr(nc), _ptr(ind),
                                                _ptr(dinds), _ptr(dwgts), _ptr(ws), ws.numel(),
                                                st), "prep")

    def means():
        _lib.check(lib.pcr_extractor_voxel_means(_ptr(feat), b, c, n, r, _ptr(ws), ws.numel(),
                                                 st), "means")

    def stream_devox():
        cnt, grid, devox, desc = outs[0]
        _lib.check(lib.pcr_extractor_voxel_stream_devox(
            b, c, n, r, _ptr(cnt), _ptr(grid), _ptr(devox), _ptr(dwgts), _ptr(desc), _ptr(ws),
            ws.numel(), st), "stream_devox")

    def means_devox():
        cnt, grid, devox, desc = outs[0]
        _lib.check(lib.pcr_extractor_voxel_means_devox(
            _ptr(feat), b, c, n, r, _ptr(devox), _ptr(dinds), _ptr(dwgts), _ptr(desc), _ptr(ws),
            ws.numel(), st), "means_devox")

    def stream():
        cnt, grid, devox, desc = outs[0]
        _lib.check(lib.pcr_extractor_voxel_stream(b, c, n, r, _ptr(cnt), _ptr(grid), _ptr(ws),
                                                  ws.numel(), st), "stream")

    # clouds past the stream's devox role (c3: 2048 points): the means launch
    # evaluates the devox, the grid stream writes grid + cnt only
    dv = bool(lib.pcr_extractor_stream_devox_ok(n, c, r))
    launches = (("prep", prep), ("means", means), ("stream_devox", stream_devox)) if dv else \
        (("prep", prep), ("means_devox", means_devox), ("stream", stream))
    for _, f in launches:
        f()
    torch.cuda.synchronize()
    res = {}
    for name, f in launches:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(30)]
        for e0, e1 in ev:
            e0.record(s)
            f()
            e1.record(s)
        torch.cuda.synchronize()
        ts = sorted(e0.elapsed_time(e1) * 1000.0 for e0, e1 in ev)
        res[name] = (ts[len(ts) // 2], ts[0])
    print("b=%d n=%d c=%d r=%d  " % (b, n, c, r) +
          "  ".join("%s %.1f us (min %.1f)" % (k, v[0], v[1]) for k, v in res.items()),
          flush=True)
