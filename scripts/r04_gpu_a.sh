#!/bin/bash
# round-4 check: smoke, the extractor / registration / backward / ops GPU
# tests, then the driver-flag and default c2 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_extractor.py tests/test_gpu_registration.py tests/test_gpu_backward.py tests/test_gpu_ops.py > gpurun_out/pt_a.log 2>&1
rc=$?; tail -4 gpurun_out/pt_a.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_drv.log 2>&1 || exit $?
tail -1 gpurun_out/bench_drv.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
