#!/bin/bash
# Diagnostic: instruction mix per kernel (SQ_INSTS_* counters, one pass) of the
# bench step (native runner), averaged per dispatch.  Not part of the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES -d gpurun_out/pmc_insts -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/pmc_insts.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for fn in glob.glob("gpurun_out/pmc_insts/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
tot = 0.0
for k, d in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU", 0) / len(cnt[kv[0]])):
    n = len(cnt[k])
    v = d.get("SQ_INSTS_VALU", 0) / n
    if not k.startswith("void pcr") and not k.startswith("pcr"):
        continue
    tot += v
    # wave64 VALU op = 4 SIMD cycles; 1024 SIMDs at ~2.1 GHz
    print("%-60s x%3d VALU-floor %.1f us " % (k, n, v * 4 / 1024 / 2.1e3) +
          " ".join("%s=%.3g" % (c.replace("SQ_INSTS_", ""), val / n) for c, val in sorted(d.items())))
print("sum of pcr kernels' VALU floor per step: %.1f us" % (tot * 4 / 1024 / 2.1e3))
PY
