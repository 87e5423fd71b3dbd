#!/bin/bash
# round-4: fused grid kernel under schedule 6 (A/B), then the c5 bench with
# its output check and the c3 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ -n "$AB" ] && { bash scripts/lib_ab.sh extract 3 base s6fused || exit $?; }
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1 || { tail -5 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log | cut -c1-400
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || { tail -5 gpurun_out/bench_c3.log; exit 1; }
tail -1 gpurun_out/bench_c3.log | cut -c1-300
