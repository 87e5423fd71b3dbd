#!/bin/bash
# Diagnostic: kernel time of the KNN neighbour stage for the diag library and
# each experiment build (lib/libpcr_amd_exp<v>.so) under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
L=point-cloud-registration-based-on-rotation-invariant-feature_amd/lib
mkdir -p gpurun_out
for lib in "$@"; do
  PCR_AMD_LIB=$PWD/$L/$lib.so timeout -k 10 150 rocprofv3 --kernel-trace --stats -d gpurun_out/kx_$lib -o run --output-format csv -- python3 scripts/knn_bench.py > gpurun_out/kx_$lib.log 2>&1 || exit $?
  PCR_AMD_LIB=$PWD/$L/$lib.so timeout -k 10 150 python3 scripts/diag_stamps.py > gpurun_out/ds_$lib.log 2>&1 || exit $?
  echo "== $lib"; grep -A6 "^knn" gpurun_out/ds_$lib.log
  python3 - "$lib" <<'PY'
import csv, sys
for r in csv.DictReader(open('gpurun_out/kx_%s/run_kernel_stats.csv' % sys.argv[1])):
    if 'knn' in r['Name']:
        print(r['Name'][:45].ljust(45), r['Calls'], round(float(r['AverageNs'])/1000, 1))
PY
done
