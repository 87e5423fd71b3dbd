#!/bin/bash
# round-4 check b: the large-cloud tests (c5 sorted voxelize), then the c5 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_large.py > gpurun_out/pt_b.log 2>&1
rc=$?; tail -4 gpurun_out/pt_b.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c5.log
timeout -k 10 400 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c3.log
