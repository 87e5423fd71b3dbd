"""Diagnostic: a small-footprint streaming kernel (scripts/micro/stream_exp.hip)
alone and beside the KNN selection.  Not part of the product."""
import ctypes
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

ex_lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "micro", "libstream_exp.so"))
ex_lib.exp_stream.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
lib = _lib.load()
sn, sv = ex.s_nbr, ex.s_vox
grid = torch.empty((b, c, r ** 3), device=dev)
n4 = grid.numel() // 4
ex.forward(xyz, nrm, feat)
torch.cuda.synchronize()


def sel():
    lib.pcr_knn_local_ppf_prepared(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(ex.knn_idx), None,
                                   None, _ptr(ex.knn_ws), ex.knn_ws.numel(), sn.cuda_stream)


def run(name, f):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(100):
            f()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / 100)
    print("%-34s %7.1f us  (%.2f TB/s of grid)" % (name, best * 1e6, grid.numel() * 4 / best / 1e12),
          flush=True)


ex_lib.exp_stream_fat.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
run("select alone", sel)
for nt, vr, lds in ((256, 4, 0), (320, 4, 0), (256, 48, 0), (256, 4, 36000), (320, 48, 36000)):
    def stf(nt=nt, vr=vr, lds=lds):
        ex_lib.exp_stream_fat(_ptr(grid), n4, 256, nt, vr, lds, sv.cuda_stream)

    tag = "fat nt=%d vregs=%d lds=%d" % (nt, vr, lds)
    run("stream " + tag, stf)
    run("sel+stream " + tag, lambda: (sel(), stf()))
sys.exit(0)
run("select alone", sel)
for wgs, nt, mode, lds in ((256, 256, 65536, 0), (256, 256, 16384, 0), (1024, 256, 16384, 0),
                           (256, 256, 0, 0), (256, 512, 0, 0), (256, 1024, 0, 0), (512, 256, 0, 0),
                           (1024, 256, 0, 0), (2048, 256, 0, 0), (256, 256, 4096, 0),
                           (256, 512, 8192, 0), (512, 256, 4096, 0), (256, 256, 0, 20000)):
    def st(wgs=wgs, nt=nt, mode=mode, lds=lds):
        ex_lib.exp_stream(_ptr(grid), n4, wgs, nt, mode, lds, sv.cuda_stream)

    tag = "wgs=%d nt=%d mode=%d lds=%d" % (wgs, nt, mode, lds)
    run("stream " + tag, st)
    run("stream+sel " + tag, lambda: (st(), sel()))
