"""Per-phase s_memtime stamps of the extractor's prep kernel
(vox_prep_kernel<kSphNormalize, 256>) at BASELINE c2 (diagnostic library
lib/libpcr_amd_diag.so, `make -C <pkg>/csrc diag`), plus its duration alone
with HIP events.  Phases: 0->1 load + fp64 mean, 1->2 max-norm +
normalise, 2->3 voxel index + devox corners (+ stores), 3->4 bitmap + word
scan + corner segments, 4->5 counts + segment scan, 5->6 point placement.
Not part of the product."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ["PCR_AMD_LIB"] = os.path.join(PKG, "lib", os.environ.get("DIAGLIB", "libpcr_amd_diag.so"))
sys.path[:0] = [ROOT, PKG]
import ctypes  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from pcr_amd import _lib  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, c, k, r = 32, 1024, 64, 32, 32
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz = (xyz - xyz.mean(2, keepdim=True)).contiguous()
feat = torch.rand((b, c, n), generator=g, device=dev)
ex = SphExtractor(b, n, c, k, r, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    ex.voxel_prep(xyz, s)
torch.cuda.synchronize()
for name, fn in (("prep", lambda: ex.voxel_prep(xyz, s)),
                 ("means+devox", lambda: ex.voxel_means_devox(feat, s))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print("%s alone: %.2f us per launch" % (name, e0.elapsed_time(e1) / 20 * 1e3))
ex.voxel_prep(xyz, s)
torch.cuda.synchronize()
lib = _lib.load()
buf = (ctypes.c_ulonglong * (1024 * 16))()
lib.pcr_diag_read_vox.restype = ctypes.c_int
lib.pcr_diag_read_vox(buf)
st = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[:b].astype(np.int64)
for p in range(6):
    d = st[:, p + 1] - st[:, p]
    print("phase %d->%d: median %6d cycles, max %6d" % (p, p + 1, int(np.median(d)), int(d.max())))
tot = st[:, 6] - st[:, 0]
print("total: median %d cycles (%.2f us at 2.4 GHz)" % (int(np.median(tot)), np.median(tot) / 2400.0))
