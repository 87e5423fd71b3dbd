#!/bin/bash
# first half of scripts/final_runs.sh (smoke, GPU suite, bench lines), for a
# gpurun call of its own
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?; tail -n 1 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_c2 200 python bench.py
run bench_c2_driver 200 python bench.py --steps 20 --warmup 5
run bench_pairs 300 python bench.py --workload pairs
run bench_c3 300 python bench.py --workload c3
run bench_c5 300 python bench.py --workload c5
