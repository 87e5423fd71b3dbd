#!/bin/bash
# round-4: VALU / LDS instruction split of the KNN selection by phase (c2 and
# c3 shapes) + the cut flags (refined / fallback workgroups)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for shape in "32 1024" "256 2048"; do
  set -- $shape
  tag=b$1n$2
  B=$1 N=$2 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM \
    -d gpurun_out/kvalu_$tag -o run --output-format csv -- python3 scripts/knn_valu_split.py > gpurun_out/kvalu_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 gpurun_out/kvalu_$tag.log; exit 1; }
  echo "== $tag"
  python3 scripts/knn_valu_split.py --report $(find gpurun_out/kvalu_$tag -name "*counter_collection.csv")
  B=$1 N=$2 timeout -k 10 120 python3 scripts/knn_stamps.py > gpurun_out/kstamps_$tag.log 2>&1 || exit $?
  cat gpurun_out/kstamps_$tag.log
done
