"""Diagnostic: time the KNN op entry points (pcr_knn_forward both directions,
pcr_knn_local_ppf) of several library builds, interleaved, and check that
their outputs agree.  Not part of the product.
usage: python scripts/knn_api_ab.py B N K lib.so [lib.so ...]"""
import ctypes
import sys

import torch

b, n, k = (int(x) for x in sys.argv[1:4])
libs = sys.argv[4:]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
xyz2 = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
P, I, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
hs = []
for path in libs:
    L = ctypes.CDLL(path)
    L.pcr_knn_workspace_size.restype = SZ
    L.pcr_knn_workspace_size.argtypes = [I, I, I]
    L.pcr_knn_forward.restype = I
    L.pcr_knn_forward.argtypes = [P, P, I, I, I, I, I, P, P, P, P, P, SZ, P]
    L.pcr_knn_local_ppf.restype = I
    L.pcr_knn_local_ppf.argtypes = [P, P, I, I, I, I, P, P, P, P, SZ, P]
    hs.append(L)
d1 = torch.empty((b, k, n), device=dev)
i1 = torch.empty((b, k, n), dtype=torch.int32, device=dev)
d2 = torch.empty((b, k, n), device=dev)
i2 = torch.empty((b, k, n), dtype=torch.int32, device=dev)
ppf = torch.empty((b, 4, k, n), device=dev)
st = torch.cuda.current_stream().cuda_stream
ref = {}
for rnd in range(3):
    for path, L in zip(libs, hs):
        ws = torch.empty(L.pcr_knn_workspace_size(b, n, n), dtype=torch.uint8, device=dev)
        def fwd():
            assert L.pcr_knn_forward(xyz.data_ptr(), xyz2.data_ptr(), b, 3, n, n, k, d1.data_ptr(),
                                     d2.data_ptr(), i1.data_ptr(), i2.data_ptr(), ws.data_ptr(),
                                     ws.numel(), st) == 0
        def lppf():
            assert L.pcr_knn_local_ppf(xyz.data_ptr(), nrm.data_ptr(), b, n, k, 0, i1.data_ptr(),
                                       None, ppf.data_ptr(), ws.data_ptr(), ws.numel(), st) == 0
        out = []
        for name, fn in (("knn_forward", fwd), ("knn_local_ppf", lppf)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res = (i1.clone(), d1.clone(), i2.clone()) if name == "knn_forward" else (i1.clone(), ppf.clone())
            same = ""
            if name in ref:
                # bitwise (the self-neighbour's PPF angles are NaN, as the reference's)
                same = all(torch.equal(a.view(torch.int32), c.view(torch.int32))
                           for a, c in zip(ref[name], res))
            else:
                ref[name] = res
            out.append("%s %.4f ms %s" % (name, e0.elapsed_time(e1) / 10, same))
        print("%-40s %s" % (path.split("/")[-1], "  |  ".join(out)), flush=True)
