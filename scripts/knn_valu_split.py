"""Diagnostic: the KNN selection of the diagnostic library at c2 (or B / N
/ K from the environment; c5: B=8 N=65536 K=64) under PCR_KNN_DBG 0 (whole kernel), 4 (stop after the
count) and 8 (stop after the collect), two launches each, in that order --
run under `rocprofv3 --pmc SQ_INSTS_VALU ...` and split the counts with
--report <counter_collection.csv>.  Not part of the product."""
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "point-cloud-registration-based-on-rotation-invariant-feature_amd")
BITS = (0, 4, 8)

if len(sys.argv) > 2 and sys.argv[1] == "--report":
    per = defaultdict(lambda: defaultdict(float))
    for f in sys.argv[2:]:
        for r in csv.DictReader(open(f)):
            if "knn_select" in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(per)
    bits = BITS if len(ids) >= 2 * len(BITS) else (0,)
    ids = ids[-2 * len(bits):]
    for i, bv in enumerate(bits):
        cs = defaultdict(float)
        for d in ids[2 * i:2 * i + 2]:
            for c, v in per[d].items():
                cs[c] += v / 2
        print("dbg %d: " % bv + "  ".join("%s %.4g" % kv for kv in sorted(cs.items())))
    sys.exit(0)

# the diagnostic build (the PCR_KNN_DBG phase stops); PRODUCT=1: the product
# library, whole launches only
if os.environ.get("PRODUCT") == "1":
    BITS = (0,)
else:
    os.environ["PCR_AMD_LIB"] = os.path.join(PKG, "lib", "libpcr_amd_diag.so")
sys.path[:0] = [ROOT, PKG]
import torch  # noqa: E402
from pcr_amd.extractor import SphExtractor  # noqa: E402

b, n, k = int(os.environ.get("B", 32)), int(os.environ.get("N", 1024)), int(os.environ.get("K", 32))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
xyz = torch.randn((b, 3, n), generator=g, device=dev)
nrm = torch.randn((b, 3, n), generator=g, device=dev)
if n <= 2048:
    ex = SphExtractor(b, n, 8, k, 8, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    ok = ex.knn_sort(xyz, s)
    run = lambda: ex.knn_select(xyz, nrm, s, sorted_ok=ok, ppf=False)  # noqa: E731
else:  # large clouds: the whole KNN + PPF call (sort, selection, emit)
    from pcr_amd import ops  # noqa: E402
    run = lambda: ops.knn_local_ppf(xyz, nrm, k)  # noqa: E731
for bits in BITS:
    os.environ["PCR_KNN_DBG"] = str(bits)
    for _ in range(2):
        run()
    torch.cuda.synchronize()
print("done b=%d n=%d" % (b, n))
