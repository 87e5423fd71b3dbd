#!/usr/bin/env python3
"""Turn the rocprofv3 --pmc passes of scripts/pmc_c2.sh (FETCH_SIZE,
WRITE_SIZE; separate passes, TCC slots) into profiles/pmc_traffic.json, the
per-launch HBM bytes of the dominant kernel (bench.py roofline.kernel.traffic)
and of the whole step, summed over the step's kernels (roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane streaming stores (the grid kernel's float4 stores).
Both counters are in KiB.
  usage: scripts/pmc_traffic.py <fetch_dir> <write_dir> <out.json> B N K R C
                                [<rdreq_dir> <wrreq_dir>]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = os.environ.get("PCR_PMC_KERNEL", "vox_stream_kernel")


# the kernels of one bench step (schedule 1): one launch each per step
STEP_KERNELS = ("knn_sort_kernel", "knn_wsel_kernel", "local_ppf_quad_kernel",
                "vox_prep_kernel", "vox_means_kernel", "vox_stream_kernel")


def per_dispatch(d, counter, kernel=None, missing_ok=False):
    kernel = kernel or KERNEL
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(float)
    for fn in files:
        for row in csv.DictReader(open(fn)):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            acc[row["Dispatch_Id"]] += float(row["Counter_Value"])
    if not acc:
        if missing_ok:
            return None
        raise SystemExit(f"no {counter} rows for {kernel} under {d}")
    return list(acc.values())


def main():
    fd, wd, out = sys.argv[1:4]
    cfg = [int(x) for x in sys.argv[4:9]]
    f = per_dispatch(fd, "FETCH_SIZE")
    w = per_dispatch(wd, "WRITE_SIZE")
    fetch = 2.0 * sum(f) / len(f) * 1024.0
    write = sum(w) / len(w) * 1024.0
    res = {"kernel": KERNEL, "config": cfg,
           "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
           "grid_kernel_hbm_bytes_per_launch": fetch + write,
           "dispatches": [len(f), len(w)],
           "step_kernels": {}, "step_hbm_bytes": 0.0,
           "note": "FETCH_SIZE x2 (gfx950 half-count on wide streaming reads), WRITE_SIZE as is; KiB -> bytes"}
    # the whole step: every step kernel's average fetch + write per launch
    for kname in STEP_KERNELS:
        kf = per_dispatch(fd, "FETCH_SIZE", kname)
        kw = per_dispatch(wd, "WRITE_SIZE", kname)
        kb = 2.0 * sum(kf) / len(kf) * 1024.0 + sum(kw) / len(kw) * 1024.0
        res["step_kernels"][kname] = kb
        res["step_hbm_bytes"] += kb
    # optional request-count passes (TCC_EA0_RDREQ / _32B, TCC_EA0_WRREQ /
    # _64B): per kernel and launch, the raw fabric request counts, which do
    # not depend on the FETCH_SIZE width calibration
    if len(sys.argv) > 10:
        rd, wr = sys.argv[9], sys.argv[10]
        reqs = {}
        for kname in STEP_KERNELS:
            row = {}
            for d, cn in ((rd, "TCC_EA0_RDREQ_sum"), (rd, "TCC_EA0_RDREQ_32B_sum"),
                          (wr, "TCC_EA0_WRREQ_sum"), (wr, "TCC_EA0_WRREQ_64B_sum")):
                v = per_dispatch(d, cn, kname, missing_ok=True)
                row[cn] = (sum(v) / len(v)) if v else None
            reqs[kname] = row
        res["ea_requests_per_launch"] = reqs
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
