"""Diagnostic (PCR_AMD_LIB=<diag lib>): path counters of knn_wsel_kernel over
one c2 selection launch: queries, exact-path queries, 64-bit-sort queries,
mean keys collected, extra threshold passes."""
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
# per-workgroup timeline of the last launch (c2 k=16 above; rerun c2 k=32)
b, n, k = 32, 1024, 32
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
ws = torch.zeros((lib.pcr_knn_workspace_size(b, n, n),), dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
_lib.check(lib.pcr_knn_prepare(_ptr(xyz), b, n, _ptr(ws), ws.numel(), st), "prepare")
_lib.check(lib.pcr_knn_select_sorted(_ptr(xyz), b, n, k, _ptr(ws), ws.numel(), st), "sel")
torch.cuda.synchronize()
h = np.zeros((1024, 16), dtype=np.uint64)
raw.pcr_diag_read_knn(h.ctypes.data_as(ctypes.c_void_p))
nwg = 16 * b
t0 = h[:nwg, 12].astype(np.int64)
t1 = h[:nwg, 13].astype(np.int64)
base = t0.min()
st_us = (t0 - base) / 100.0
en_us = (t1 - base) / 100.0
print("WG start us: min %.2f p25 %.2f p50 %.2f p75 %.2f max %.2f" % tuple(np.percentile(st_us, [0, 25, 50, 75, 100])))
print("WG end   us: min %.2f p25 %.2f p50 %.2f p75 %.2f max %.2f" % tuple(np.percentile(en_us, [0, 25, 50, 75, 100])))
dur = en_us - st_us
print("WG dur   us: min %.2f p50 %.2f max %.2f" % (dur.min(), np.median(dur), dur.max()))
load = (h[:nwg, 1].astype(np.int64) - h[:nwg, 0].astype(np.int64))
print("load cycles: p50 %d max %d" % (np.median(load), load.max()))
wv = h[:nwg, 4:12].astype(np.int64) - h[:nwg, 1:2].astype(np.int64)
print("wave loop cycles: p50 %d min %d max %d" % (np.median(wv), wv.min(), wv.max()))
hist = np.histogram(st_us, bins=10)
print("start histogram:", hist[0].tolist(), np.round(hist[1], 1).tolist())

hw = np.zeros((1024, 8, 8), dtype=np.uint64)
raw.pcr_diag_read_knn_wave(hw.ctypes.data_as(ctypes.c_void_p))
v = hw[:nwg, :, 0].astype(np.int64)
ex, sl, ps = v >> 48, (v >> 32) & 0xFFFF, (v >> 16) & 0xFFFF
print("queries: exact %d slow %d extra passes %.3f/query" %
      (ex.sum(), sl.sum(), ps.sum() / (nwg * 64.0)))
ph = hw[:nwg, :, 1:6].astype(np.float64).reshape(-1, 5)
names = ["distances", "threshold passes", "compaction", "sort", "tie/payload/tile"]
tot = ph.sum(1)
nq = nwg * 64.0
print("per-query phase cycles (wave clock, summed over waves / queries): " +
      ", ".join("%s %.0f" % (nm, ph[:, i].sum() / nq) for i, nm in enumerate(names)) +
      "; total %.0f" % (tot.sum() / nq))
