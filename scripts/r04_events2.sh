#!/bin/bash
# round-4: the GPU suite on the product library (sync events without system
# fences, timing events with device-scope release), then the event A/B:
# base (product), evsys (system-fence sync events), tdefault (default timing
# events), and base without kernel timing; c2 default and driver-flag lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBDIR=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
line() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ev.tmp") if l.startswith("{")][-1])
k = d["roofline"]["kernel"]
print("%-26s %9.1f clouds/s  %.4f ms/step  grid kernel %s ms  verified %s" % (
    sys.argv[1], d["value"], d["ms_per_step"], k and k.get("avg_ms_in_step"), d["outputs_verified"]))
PY
}
for r in 1 2 3; do
  for v in base evsys tdefault; do
    PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/ev.tmp 2>&1 || exit $?
    line "$v-200"
    PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ev.tmp 2>&1 || exit $?
    line "$v-20"
  done
  PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_base.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing > gpurun_out/ev.tmp 2>&1 || exit $?
  line "base-20-notiming"
done
