#!/bin/bash
# Diagnostic: bench value per library build (product, diag, experiment
# builds), interleaved twice.  Not part of the product.
#   usage: scripts/lib_sweep.sh libpcr_amd libpcr_amd_exp11 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
L=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
for rnd in 1 2; do
  for lib in "$@"; do
    v=$(PCR_AMD_LIB=$L/$lib.so timeout -k 10 120 python bench.py --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*')
    rc=$?
    echo "$lib $v"
    [ $rc -gt 1 ] && exit $rc
  done
done
