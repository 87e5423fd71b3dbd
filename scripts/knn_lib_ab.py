"""Diagnostic: time pcr_knn_local_ppf (self KNN + local PPF) of several
library builds on the same inputs, interleaved (A/B of KNN kernel changes;
binds only the two entry points it calls, so older builds load too).
usage: python scripts/knn_lib_ab.py <B> <N> <k> <lib.so> [<lib.so> ...]"""
import ctypes
import sys

import torch

b, n, k = (int(x) for x in sys.argv[1:4])
libs = sys.argv[4:]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
P = ctypes.c_void_p
handles = []
for path in libs:
    L = ctypes.CDLL(path)
    L.pcr_knn_workspace_size.restype = ctypes.c_size_t
    L.pcr_knn_workspace_size.argtypes = [ctypes.c_int] * 3
    L.pcr_knn_local_ppf.restype = ctypes.c_int
    L.pcr_knn_local_ppf.argtypes = [P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    P, P, P, P, ctypes.c_size_t, P]
    handles.append(L)
idx = torch.empty((b, k, n), dtype=torch.int32, device=dev)
ppf = torch.empty((b, 4, k, n), device=dev)
res = {p: [] for p in libs}
ref = None
for rnd in range(3):
    for path, L in zip(libs, handles):
        ws = torch.empty(L.pcr_knn_workspace_size(b, n, n), dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream

        def run():
            rc = L.pcr_knn_local_ppf(xyz.data_ptr(), nrm.data_ptr(), b, n, k, 1, idx.data_ptr(),
                                     None, ppf.data_ptr(), ws.data_ptr(), ws.numel(), st)
            assert rc == 0, rc
        run()
        torch.cuda.synchronize()
        if ref is None:
            ref = idx.clone()
        same = torch.equal(idx, ref)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run()
        e1.record()
        torch.cuda.synchronize()
        res[path].append(e0.elapsed_time(e1) / 3)
        print("%-60s %8.3f ms  idx==first lib: %s" % (path.split("/")[-1], res[path][-1], same),
              flush=True)
