#!/bin/bash
# second half of scripts/final_runs.sh: rocprofv3 kernel traces + stats of
# the c2 / c3 / pairs / c5 bench commands, then the c2 PMC passes
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
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run prof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 80 --warmup 40 --no-cpu-baseline --no-verify
run prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 10 --no-cpu-baseline --no-verify
run prof_pairs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pairs -o run --output-format csv -- python3 bench.py --workload pairs --steps 40 --warmup 20 --no-cpu-baseline --no-verify
run prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --no-cpu-baseline --no-verify
bash scripts/pmc_c2.sh
