#!/bin/bash
# round-4 A/B of the local PPF launch: base (product), oldppf (the per-256-point
# local_ppf_self_kernel), ppfhw (v_rsq / v_sqrt arithmetic), ppfsl2 (two slots
# per workgroup); 3 interleaved rounds of c2, 2 of c3; then prep stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/lib_ab.sh "extract" 3 base oldppf ppfhw || exit $?
bash scripts/lib_ab.sh "c3" 2 base oldppf ppfsl2 || exit $?
timeout -k 10 120 python scripts/prep_stamps.py > gpurun_out/prep_stamps.log 2>&1; tail -12 gpurun_out/prep_stamps.log
