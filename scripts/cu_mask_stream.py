"""Diagnostic: the grid-streaming kernel confined to a CU subset (several
workgroups per CU) and the KNN selection on the rest
(hipExtStreamCreateWithCUMask).  Not part of the product."""
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

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
dev = torch.device("cuda:0")
ncu = torch.cuda.get_device_properties(0).multi_processor_count


def masked_stream(cus):
    words = (ncu + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for c in cus:
        m[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, m) == 0
    return torch.cuda.ExternalStream(s.value, device=dev)


b, n, c, k, r = 32, 1024, 64, 32, 32
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
lib = _lib.load()
ex.forward(xyz, nrm, feat)
ex.voxel_means_devox(feat, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()


def run(label, f):
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
    print("%-44s %7.1f us" % (label, best * 1e6), flush=True)


for nv in (64, 96, 128):
    step = ncu // nv
    vox = list(range(0, ncu, step))[:nv]
    knn = [cc for cc in range(ncu) if cc not in set(vox)]
    sk, sv = masked_stream(knn), masked_stream(vox)

    def sel(sk=sk):
        lib.pcr_knn_local_ppf_prepared(_ptr(xyz), _ptr(nrm), b, n, k, 1, _ptr(ex.knn_idx), None,
                                       None, _ptr(ex.knn_ws), ex.knn_ws.numel(), sk.cuda_stream)

    def st(sv=sv):
        ex.voxel_stream(sv.cuda_stream)

    run("select on %d CUs" % len(knn), sel)
    run("stream on %d CUs (%s WGs)" % (nv, os.environ.get("PCR_STREAM_WGS")), st)
    run("both", lambda: (sel(), st()))
