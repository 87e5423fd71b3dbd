#!/bin/bash
# Diagnostic: SQ counters of the KNN kernels (one rocprofv3 --pmc pass per set).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=${1:-libpcr_amd_diag}
export PCR_AMD_LIB=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib/$LIB.so
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/kpmc$i -o run --output-format csv -- python3 scripts/knn_bench.py > gpurun_out/kpmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/kpmc$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/kpmc*/**/*counter_collection.csv', recursive=True):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        if 'knn' not in r['Kernel_Name']:
            continue
        key = (r['Dispatch_Id'], r['Counter_Name'])
        per[key] += float(r['Counter_Value'])
        names[r['Dispatch_Id']] = r['Kernel_Name'][:40]
    for (d, c), v in per.items():
        acc[names[d]][c].append(v)
for kname, cs in acc.items():
    print(kname)
    for c, vs in sorted(cs.items()):
        print("   %-22s %.4g" % (c, sum(vs) / len(vs)))
PY
