"""Diagnostic: s_memtime stamps of vox_stream_kernel (diag build) -- per item
streaming time and barrier waits -- and step times under the PCR_STREAM_DBG
switches.  Not part of the product."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ.setdefault("PCR_AMD_LIB", os.path.join(PKG, "lib", "libpcr_amd_diag.so"))
sys.path[:0] = [ROOT, PKG]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pcr_amd import _lib  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
nrm = (nrm / nrm.norm(dim=1, keepdim=True)).contiguous()
feat = (torch.rand((b, c, n), generator=g, device=dev) * 2 - 1).contiguous()
ex = SphExtractor(b, n, c, k, r, device=dev)
lib = _lib.load()
s = torch.cuda.current_stream().cuda_stream
ex.voxel_prep(xyz, s)
ex.voxel_means_devox(feat, s)
for _ in range(5):
    ex.voxel_stream(s)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100):
    ex.voxel_stream(s)
torch.cuda.synchronize()
print("stream alone %.1f us  (PCR_STREAM_DBG=%s NS=%s)" % ((time.perf_counter() - t0) * 1e4,
      os.environ.get("PCR_STREAM_DBG", "0"), os.environ.get("PCR_STREAM_NS", "4")))
buf = (ctypes.c_ulonglong * (1024 * 16))()
ex.voxel_stream(s)
torch.cuda.synchronize()
lib.pcr_diag_read_vox(buf)
a = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:256].astype(np.int64)
t0 = a[:, 0].min()
print("WG start spread %d cycles; end spread %d" % (a[:, 0].max() - t0, a[:, 11].max() - a[:, 11].min()))
print("load0 (0->1) median %d" % np.median(a[:, 1] - a[:, 0]))
prev = a[:, 1]
for it in range(4):
    st = a[:, 2 + it] - prev
    bw = a[:, 8 + it] - a[:, 2 + it]
    print("item %d: stream median %d max %d; barrier wait median %d max %d"
          % (it, np.median(st), st.max(), np.median(bw), bw.max()))
    prev = a[:, 8 + it]
print("kernel span %d cycles" % (a[:, 11].max() - t0))
