#!/bin/bash
# diagnostic: packed fp32 issue rate and its SQ_INSTS_VALU accounting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/micro/pk_rate || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES -d gpurun_out/pkpmc -o run --output-format csv -- ./scripts/micro/pk_rate > gpurun_out/pkpmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pkpmc/**/*counter_collection.csv', recursive=True):
    acc = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        acc[(r['Dispatch_Id'], r['Counter_Name'])] += float(r['Counter_Value'])
        names[r['Dispatch_Id']] = r['Kernel_Name'].split('(')[0]
    for (d, c), v in acc.items():
        per[names[d]][c].append(v)
for k, cs in per.items():
    print(k, {c: "%.4g" % (sum(v) / len(v)) for c, v in cs.items()})
PY
