#!/bin/bash
# round-4 A/B of the local PPF launch: base (product), oldppf (the per-256-point
# local_ppf_self_kernel), ppfhw (v_rsq / v_sqrt arithmetic), ppfsl2 (two slots
# per workgroup); 3 interleaved rounds of c2, 2 of c3; then prep stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/lib_ab.sh "extract" 3 base oldppf ppfhw || exit $?
bash scripts/lib_ab.sh "c3" 2 base oldppf ppfsl2 || exit $?
timeout -k 10 120 python scripts/prep_stamps.py > gpurun_out/prep_stamps.log 2>&1; tail -12 gpurun_out/prep_stamps.log
for f in 0.5 0.375 0.625; do
  timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --c3-cu-split $f > gpurun_out/c3_cusplit_$f.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print('c3 cu-split', sys.argv[2], d['ms_per_step'], 'ms', d['value'], 'clouds/s')" gpurun_out/c3_cusplit_$f.log $f
done
