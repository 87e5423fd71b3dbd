#!/bin/bash
# round-4: runner event scope A/B (base: default events; evnofence:
# hipEventDisableSystemFence; evdevice: hipEventReleaseToDevice), c2 default
# and driver-flag lines, then a kernel trace of the better variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBDIR=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
line() {
  python - "$1" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/ev.tmp") if l.startswith("{")][-1])
print("%-22s %9.1f clouds/s  %.4f ms/step  grid kernel %.4f ms  verified %s" % (
    sys.argv[1], d["value"], d["ms_per_step"], d["roofline"]["kernel"]["avg_ms_in_step"],
    d["outputs_verified"]))
PY
}
for r in 1 2 3; do
  for v in base evnofence evdevice; do
    PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/ev.tmp 2>&1 || exit $?
    line "$v-200"
    PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ev.tmp 2>&1 || exit $?
    line "$v-20"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
PCR_AMD_LIB=$LIBDIR/libpcr_amd_exp_evnofence.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ev -o run --output-format csv -- python3 bench.py --steps 80 --warmup 40 --no-cpu-baseline > gpurun_out/prof_ev.log 2>&1
echo "prof rc=$?"
