#!/bin/bash
# Runs GPU steps in order on the gpurun box.  Each step has its own time
# limit; a test failure (exit 1) lets the next step run, but a crash, abort,
# signal or timeout (anything else non-zero) stops the script: nothing more
# touches the GPU after a fault.
#   usage: scripts/gpu_steps.sh <step> [<step> ...]
#   steps: smoke tests tests_all large c5 bench bench_drv bench_c3 bench_c5 bench_pairs
#          prof prof_c3 prof_c5 pmc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 25 "gpurun_out/$name.log"
  echo "=== $name exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1200 python -m pytest tests -x -q -m gpu -p no:cacheprovider ;;
    tests_all) run pytest_gpu 1200 python -m pytest tests -q -m gpu -p no:cacheprovider ;;
    bench) run bench 600 python bench.py ;;
    bench_drv) run bench_drv 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    bench_c3) run bench_c3 600 python bench.py --workload c3 ;;
    bench_c5) run bench_c5 600 python bench.py --workload c5 ;;
    bench_pairs) run bench_pairs 300 python bench.py --workload pairs --no-cpu-baseline ;;
    prof_c3) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof_c3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 10 --no-cpu-baseline ;;
    prof_c5) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof_c5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --steps 5 --no-cpu-baseline ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
          run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 80 --warmup 40 --no-cpu-baseline ;;
    pmc)  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 5 --steps-per-launch 5 --kernel-iters 5 --no-cpu-baseline
          run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 5 --steps-per-launch 5 --kernel-iters 5 --no-cpu-baseline
          run pmc_json 60 python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json 32 1024 32 32 64 ;;
    large) run pytest_large 600 python -m pytest tests/test_gpu_large.py -q -m gpu -p no:cacheprovider ;;
    c5) run c5_time 300 python scripts/c5_time.py ;;
    cube) run cube_time 300 python scripts/cube_time.py ;;
    cubebwd) run cube_bwd 300 python scripts/cube_bwd_time.py
             cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
             run cube_bwd_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cubeprof -o run --output-format csv -- python3 scripts/cube_bwd_time.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
