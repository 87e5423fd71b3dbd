#!/bin/bash
# round-4 GPU session: smoke, the whole GPU suite, the c2 / c3 / c5 bench
# lines, the local-PPF A/B and the prep stamps.  Each step has its own time
# limit; a crash / abort / timeout stops the script (a test failure does not).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n "${TAILN:-3}" "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
step bench_drv 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
step bench 300 python bench.py --no-cpu-baseline
step bench_c3 400 python bench.py --workload c3 --no-cpu-baseline
step bench_c5 300 python bench.py --workload c5 --no-cpu-baseline
[ "${SKIP_AB:-0}" = 1 ] && exit 0
step ab 600 bash scripts/r04_gpu_c.sh
