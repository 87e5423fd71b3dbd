#!/bin/bash
# round-4: runner schedule 7 (three voxel queues, one KNN queue) -- its GPU
# tests, interleaved c2 / pairs bench lines of schedules 6 and 7, a trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_extractor.py tests/test_gpu_registration.py -k "runner or ring or pair_step or multi_queue" > gpurun_out/pt_s7.log 2>&1
rc=$?; tail -3 gpurun_out/pt_s7.log; [ $rc -eq 0 ] || exit $rc
line() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/s7.tmp") if l.startswith("{")][-1])
k = d["roofline"]["kernel"]
print("%-16s %9.1f clouds/s  %.4f ms/step  grid kernel %s ms  verified %s" % (
    sys.argv[1], d["value"], d["ms_per_step"], k and k.get("avg_ms_in_step"), d["outputs_verified"]))
PY
}
for r in 1 2 3; do
  for sc in 6 7; do
    timeout -k 10 120 python bench.py --schedule $sc --no-cpu-baseline > gpurun_out/s7.tmp 2>&1 || { tail -3 gpurun_out/s7.tmp; exit 1; }
    line "sched$sc-200"
    timeout -k 10 120 python bench.py --schedule $sc --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/s7.tmp 2>&1 || { tail -3 gpurun_out/s7.tmp; exit 1; }
    line "sched$sc-20"
  done
done
for sc in 6 7; do
  timeout -k 10 200 python bench.py --workload pairs --schedule $sc --no-cpu-baseline > gpurun_out/s7.tmp 2>&1 || { tail -3 gpurun_out/s7.tmp; exit 1; }
  line "pairs-sched$sc"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s7 -o run --output-format csv -- python3 bench.py --schedule 7 --steps 80 --warmup 40 --no-cpu-baseline > gpurun_out/prof_c2s7.log 2>&1
echo "prof rc=$?"
