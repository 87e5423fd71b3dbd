"""Diagnostic (PCR_AMD_LIB=<diag lib>, PCR_KNN_PSEL=3): counters and phase
cycles of knn_psel_kernel over one selection launch per shape (first 1023
workgroups): registers per prune, prunes / passes per query, exact-path
queries, wave-clock cycles per query in prune + threshold, compaction,
sort + output."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402

from pcr_amd import _lib  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
raw = ctypes.CDLL(_lib.LIB_PATH)
for b, n, k in ((32, 1024, 32), (256, 2048, 32)):
    g = torch.Generator(device=dev).manual_seed(0)
    xyz = torch.randn((b, 3, n), generator=g, device=dev)
    ws = torch.zeros((lib.pcr_knn_workspace_size(b, n, n),), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    _lib.check(lib.pcr_knn_prepare(_ptr(xyz), b, n, _ptr(ws), ws.numel(), st), "prepare")
    _lib.check(lib.pcr_knn_select_sorted(_ptr(xyz), b, n, k, _ptr(ws), ws.numel(), st), "sel")
    torch.cuda.synchronize()
    hw = np.zeros((1024, 8, 8), dtype=np.uint64)
    raw.pcr_diag_read_knn_wave(hw.ctypes.data_as(ctypes.c_void_p))
    nwg = min(1023, (n // 64) * b)
    v = hw[:nwg].astype(np.float64).sum(axis=(0, 1))
    nq = nwg * 64.0
    print("b=%d n=%d k=%d: S/prune %.2f  prunes/query %.3f  passes/query %.3f  exact %d  "
          "cycles/query: prune+threshold %.0f compaction %.0f sort+output %.0f" %
          (b, n, k, v[0] / max(v[1], 1), v[1] / nq, v[2] / nq, v[3], v[4] / nq, v[5] / nq,
           v[6] / nq), flush=True)
