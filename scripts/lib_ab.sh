#!/bin/bash
# A/B of library builds (lib/libpcr_<name>.so: "amd" is the product, other
# builds are copied in by hand, e.g. lib/libpcr_ab_base.so from a worktree of
# the previous commit, and deleted after the A/B): interleaved bench.py runs
# of each workload per build, each under its own time limit; stops at the
# first crash / timeout.  BENCH_ARGS: extra bench.py flags; TAG: log prefix.
#   usage: scripts/lib_ab.sh "<workload> ..." <rounds> <name> [<name> ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIBDIR=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
wls=$1; rounds=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for wl in $wls; do
    for name in "$@"; do
      out=gpurun_out/${TAG:-ab}_${wl}_${name}_$r.log
      PCR_AMD_LIB=$LIBDIR/libpcr_$name.so timeout -k 10 300 \
        python bench.py --workload "$wl" --no-cpu-baseline $BENCH_ARGS > "$out" 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$wl $name rc=$rc"; tail -5 "$out"; exit $rc; fi
      python - "$out" "$wl" "$name" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
k = d["roofline"]["kernel"]
print("%-6s %-8s %9.1f clouds/s  %.4f ms/step  kernel %.4f ms  verified=%s" % (
    sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], k.get("avg_ms_in_step") or -1,
    d.get("outputs_verified")))
PY
    done
  done
done
