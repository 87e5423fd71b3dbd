"""Throughput of the MFMA mutual-NN matching at the c4
shape: 128 registration pairs per GPU x 1024 points, C channels; FLOP/s of
the cross term against the fp32 MFMA peak.  Diagnostic, not the bench."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd import _lib, ops  # noqa: E402
from pcr_amd.ops import _ptr  # noqa: E402

dev = torch.device("cuda:0")
PEAK = 157.3e12  # MI355X fp32 MFMA dense (MI355X_MICROARCH.md)
for p, n, c in ((128, 1024, 64), (128, 1024, 512), (32, 1024, 512)):
    f1 = torch.randn((p, n, c), device=dev)
    f2 = torch.randn((p, n, c), device=dev)
    lib = _lib.load()
    i32 = dict(dtype=torch.int32, device=dev)
    outs = [torch.empty((p, n), **i32) for _ in range(4)] + [torch.empty((p,), **i32)]
    ws = torch.empty(lib.pcr_mutual_nn_workspace_size(p, n, n), dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    cm = os.environ.get("CM") == "1"  # channel-major [p][c][n] (the runner's matching)

    def run():
        fn = lib.pcr_mutual_nn_match_cm if cm else lib.pcr_mutual_nn_match
        _lib.check(fn(_ptr(f1), _ptr(f2), p, n, n, c, *[_ptr(o) for o in outs],
                      _ptr(ws), ws.numel(), s), "match")
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it = 20
    for _ in range(it):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / it
    fl = 2.0 * p * n * n * c
    print("%sp=%d n=%d c=%d: %.3f ms  %.0f pairs/s  %.1f TFLOP/s (%.0f%% of fp32 MFMA peak)"
          % ("cm " if cm else "", p, n, c, dt * 1e3, p / dt, fl / dt / 1e12, 100 * fl / dt / PEAK), flush=True)
