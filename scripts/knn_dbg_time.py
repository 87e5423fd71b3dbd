"""Diagnostic: time the KNN selection (plain knn_forward, no PPF) of the
diagnostic library under the experiment bits of knn_select_kernel
(PCR_KNN_DBG: 1 count without LDS atomics, 2 candidates from registers,
4 stop after the count, 8 stop after the collect, 16 collect without
stores).  Outputs are garbage under any bit; timing only.  Not part of the
product.  usage: python scripts/knn_dbg_time.py B N K"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
os.environ["PCR_AMD_LIB"] = os.path.join(PKG, "lib", "libpcr_amd_diag.so")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import ops  # noqa: E402

b, n, k = (int(x) for x in sys.argv[1:4])
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
for bits in (0, 4, 4 | 1, 4 | 2, 4 | 3, 8, 8 | 16, 8 | 2 | 16, 0):
    os.environ["PCR_KNN_DBG"] = str(bits)
    for _ in range(3):
        ops.knn_forward_cuda(xyz, xyz, k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.knn_forward_cuda(xyz, xyz, k)
    e1.record()
    torch.cuda.synchronize()
    print("bits %2d: %.4f ms per call (incl. sort)" % (bits, e0.elapsed_time(e1) / 20), flush=True)
