#!/bin/bash
# Diagnostic A/B of the voxel-stage variants (diag library knobs), bench
# line per variant.  Not part of the product.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export PCR_AMD_LIB=$PWD/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib/libpcr_amd_diag.so
for v in "PCR_VOX_SPLIT=0" "PCR_MEANS_CFG=0" "PCR_MEANS_CFG=1" "PCR_MEANS_CFG=2"; do
  echo "== $v"
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline 2>&1 | grep -o '"value": [0-9.]*\|"kernel_avg_ms": [0-9.]*' | tr '\n' ' '
  echo
  rc=${PIPESTATUS[0]}
done
