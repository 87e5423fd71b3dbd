"""Diagnostic: pipelined extractor throughput when the KNN stream and the
voxel stream are confined to disjoint CU sets (hipExtStreamCreateWithCUMask).
Not part of the product."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(ctypes.c_uint32)]
dev = torch.device("cuda:0")
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs", ncu)


def masked_stream(cus):
    words = (ncu + 31) // 32
    m = (ctypes.c_uint32 * words)()
    for c in cus:
        m[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), words, m)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


b, n, c, k, r = 32, 1024, 64, 32, 32
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
ref = {kk: v.clone() for kk, v in ex.forward(xyz, nrm, feat).items()}


def run(label, s_nbr, s_vox, steps=100):
    ex.s_nbr, ex.s_vox = s_nbr, s_vox
    for _ in range(2):
        ex.run_pipelined(xyz, nrm, feat, 10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps // 10):
        out = ex.run_pipelined(xyz, nrm, feat, 10)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    ok = all(torch.equal(out[kk], v) or torch.allclose(out[kk], v, equal_nan=True)
             for kk, v in ref.items())
    print("%-28s %.1f us/step  %.0f clouds/s  ok=%s" % (label, dt * 1e6, b / dt, ok), flush=True)


plain_n, plain_v = ex.s_nbr, ex.s_vox
run("unmasked", plain_n, plain_v)
for nv in (32, 48, 64, 96):
    # contiguous split and an interleaved split (every (ncu/nv)-th CU to voxels)
    vox = list(range(ncu - nv, ncu))
    knn = list(range(0, ncu - nv))
    run("contig knn %d / vox %d" % (len(knn), nv), masked_stream(knn), masked_stream(vox))
    step = ncu // nv
    vox = list(range(0, ncu, step))[:nv]
    knn = [cc for cc in range(ncu) if cc not in set(vox)]
    run("strided knn %d / vox %d" % (len(knn), nv), masked_stream(knn), masked_stream(vox))
