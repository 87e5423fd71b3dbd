#!/bin/bash
# round-4: diagnostic-library knob sweep under runner schedule 6 (c2, 200 steps)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
BENCH_ARGS="--schedule 6" timeout -k 10 900 bash scripts/env_sweep.sh libpcr_amd_diag "" "PCR_PREP_NT=512" "PCR_PREP_NT=1024" \
  "PCR_PREP_PRIO=0" "PCR_STREAM_WGS=128" "PCR_STREAM_WGS=512" "PCR_MEANS_G=4" "PCR_STREAM_NS=2"
