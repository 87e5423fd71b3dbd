#!/bin/bash
# One GPU call: the bench's rocprofv3 kernel stats and PMC traffic passes, the
# bench line, and kernel stats of the c3 / c5 timing scripts.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_steps.sh prof pmc bench || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for s in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${s}prof -o run --output-format csv \
    -- python3 scripts/${s}_time.py > gpurun_out/${s}p.log 2>&1 || exit $?
done
echo profiles done
