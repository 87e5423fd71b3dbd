#!/bin/bash
# round-4 final c2 state (schedule 6 default): GPU suite, bench lines (default
# and driver flags), rocprofv3 stats of the default bench, PMC traffic passes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c2_driver.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c2_driver.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 80 --warmup 40 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || exit $?
tail -1 gpurun_out/prof_c2.log
bash scripts/r04_pmc.sh
