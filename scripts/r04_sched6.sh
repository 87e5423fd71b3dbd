#!/bin/bash
# round-4: runner schedule 6 (two independent pipelines per chain, no
# cross-queue events) -- its GPU tests, interleaved c2 bench lines of
# schedules 1, 5 and 6, then a kernel trace of schedule 6
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_extractor.py tests/test_gpu_registration.py -k "runner or ring or pair_step or schedule6" > gpurun_out/pt_sched.log 2>&1
rc=$?; tail -3 gpurun_out/pt_sched.log; [ $rc -eq 0 ] || exit $rc
line() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/sched.tmp") if l.startswith("{")][-1])
k = d["roofline"]["kernel"]
print("%-22s %9.1f clouds/s  %.4f ms/step  grid kernel %s ms  verified %s" % (
    sys.argv[1], d["value"], d["ms_per_step"], k and k.get("avg_ms_in_step"), d["outputs_verified"]))
PY
}
for r in 1 2 3; do
  for sc in 1 5 6; do
    timeout -k 10 120 python bench.py --schedule $sc --no-cpu-baseline > gpurun_out/sched.tmp 2>&1 || exit $?
    line "sched$sc-200"
    timeout -k 10 120 python bench.py --schedule $sc --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/sched.tmp 2>&1 || exit $?
    line "sched$sc-20"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2s6 -o run --output-format csv -- python3 bench.py --schedule 6 --steps 80 --warmup 40 --no-cpu-baseline > gpurun_out/prof_c2s6.log 2>&1
echo "prof rc=$?"
