#!/bin/bash
# round-4: the c5 KNN selection in isolation (8 x 65,536 points, k = 64):
# SQ / TCC counters of the product library's selection launch (two passes),
# then per-phase stamps and visit counts of cloud 0 from the diagnostic
# build (which runs the c5 selection ~4x slower: its debug bits sit in the
# visit loops -- read its phase ratios, not its times)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export B=8 N=65536 K=64 PRODUCT=1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
  -d gpurun_out/c5p1 -o run --output-format csv -- python3 scripts/knn_valu_split.py > gpurun_out/c5p1.log 2>&1 || { echo "pmc 1 failed"; tail -5 gpurun_out/c5p1.log; exit 1; }
python3 scripts/knn_valu_split.py --report $(find gpurun_out/c5p1 -name "*counter_collection.csv")
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM TCC_HIT_sum TCC_MISS_sum \
  -d gpurun_out/c5p2 -o run --output-format csv -- python3 scripts/knn_valu_split.py > gpurun_out/c5p2.log 2>&1 || { echo "pmc 2 failed"; tail -5 gpurun_out/c5p2.log; exit 1; }
python3 scripts/knn_valu_split.py --report $(find gpurun_out/c5p2 -name "*counter_collection.csv")
unset PRODUCT
C5=1 timeout -k 10 120 python3 scripts/knn_stamps.py 2>&1 | grep -v amdgpu.ids
