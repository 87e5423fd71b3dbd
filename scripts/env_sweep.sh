#!/bin/bash
# Diagnostic: bench value of the diagnostic library under several runner
# knob settings, interleaved twice.  Not part of the product.
#   usage: scripts/env_sweep.sh <lib> "" "PCR_RUN_FUSE=1" "PCR_RUN_SKIP=2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
L=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
lib=$1; shift
for rnd in 1 2; do
  for envs in "$@"; do
    v=$(env $envs PCR_AMD_LIB=$L/$lib.so timeout -k 10 120 python bench.py --no-cpu-baseline --no-verify $BENCH_ARGS \
        2>/dev/null | grep -o '"value": [0-9.]*')
    rc=$?
    echo "$lib [$envs] $v"
    [ $rc -gt 1 ] && exit $rc
  done
done
exit 0
