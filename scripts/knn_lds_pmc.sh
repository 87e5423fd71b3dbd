#!/bin/bash
# Diagnostic: LDS-pipe counters of the KNN kernels at c5 and c2 (one
# rocprofv3 --pmc pass each; summary via knn_pmc.sh's reducer).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
set="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_INSTS_LDS_ATOMIC SQ_INST_LEVEL_LDS SQ_CYCLES GRBM_GUI_ACTIVE"
for cfg in "8 65536 64" "32 1024 32"; do
  set -- $cfg
  d=gpurun_out/lpmc_$2
  B=$1 N=$2 K=$3 timeout -s KILL 120 rocprofv3 --pmc $set -d $d -o run --output-format csv -- python3 scripts/knn_bench.py > $d.log 2>&1 || { echo "pass $cfg failed"; tail -5 $d.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob('gpurun_out/lpmc_*/**/*counter_collection.csv', recursive=True)):
    per = collections.defaultdict(float); names = {}
    for r in csv.DictReader(open(f)):
        if 'knn_select' not in r['Kernel_Name']:
            continue
        per[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        names[r['Dispatch_Id']] = r['Kernel_Name'][:60]
    acc = collections.defaultdict(list)
    for (d, c), v in per.items():
        acc[c].append(v)
    print(f, set(names.values()))
    for c, vs in sorted(acc.items()):
        print("   %-24s %.4g" % (c, sum(vs) / len(vs)))
PY
