#!/bin/bash
# round-4: diagnostic-library knob sweep 2 under runner schedule 6 (c2, 200
# steps): 1024-thread prep with issue-priority combinations
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export HSA_ENABLE_IPC_MODE_LEGACY=0
N=PCR_PREP_NT=1024
BENCH_ARGS="--schedule 6" timeout -k 10 900 bash scripts/env_sweep.sh libpcr_amd_diag "" "$N" "$N PCR_PREP_PRIO=0" \
  "$N PCR_PRIO_4=1 PCR_PRIO_5=1" "$N PCR_PRIO_4=2 PCR_PRIO_5=2" "$N PCR_PRIO_0=0" "$N PCR_PRIO_5=3" \
  "$N PCR_PRIO_1=1 PCR_PRIO_2=1" "$N PCR_PREP_PRIO=0 PCR_PRIO_0=0"
