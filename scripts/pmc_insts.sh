#!/bin/bash
# Diagnostic: instruction mix per kernel (SQ_INSTS_* counters, one pass) for
# the bench step, summarised per kernel.  Not part of the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/pmc_insts -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --kernel-iters 5 --no-cpu-baseline --mode eager > gpurun_out/pmc_insts.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for fn in glob.glob("gpurun_out/pmc_insts/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"][:50]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
for k, d in acc.items():
    n = len(cnt[k])
    print("%-50s x%3d " % (k, n) + " ".join("%s=%.3g" % (c.replace("SQ_INSTS_", ""), v / n) for c, v in sorted(d.items())))
PY
