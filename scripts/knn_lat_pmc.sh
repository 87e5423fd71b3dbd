#!/bin/bash
# Diagnostic: memory / LDS latency counters (Little's law: level / instructions)
# of the c5 KNN selection, and its L2 hit rate; one rocprofv3 --pmc pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for set in "SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  d=gpurun_out/latpmc$i
  B=8 N=65536 K=64 timeout -s KILL 120 rocprofv3 --pmc $set -d $d -o run --output-format csv -- python3 scripts/knn_bench.py > $d.log 2>&1 || { echo "pass $i failed"; tail -5 $d.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/latpmc*/**/*counter_collection.csv', recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if 'knn_select' not in r['Kernel_Name']:
            continue
        per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
    for (d, c), v in per.items():
        acc[c].append(v)
m = {c: sum(v) / len(v) for c, v in acc.items()}
for c in sorted(m):
    print("   %-22s %.4g" % (c, m[c]))
for lv, n in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"), ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM")):
    if lv in m and m.get(n):
        print("   latency %s / %s = %.0f" % (lv, n, m[lv] / m[n]))
if m.get("TCC_HIT_sum") is not None:
    print("   L2 hit rate %.3f" % (m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"])))
PY
