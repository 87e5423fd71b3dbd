#!/bin/bash
# Diagnostic: builds the product library of an earlier commit as
# lib/libpcr_amd_<name>.so for same-box A/B bench runs (scripts/lib_sweep.sh).
#   usage: scripts/build_ref_lib.sh <commit> <name>
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d /tmp/pcr_ref.XXXX)
git archive "$rev" include point-cloud-registration-based-on-rotation-invariant-feature_amd/csrc | tar -x -C "$tmp"
make -s -j8 -C "$tmp/point-cloud-registration-based-on-rotation-invariant-feature_amd/csrc"
cp "$tmp/point-cloud-registration-based-on-rotation-invariant-feature_amd/lib/libpcr_amd.so" \
   point-cloud-registration-based-on-rotation-invariant-feature_amd/lib/libpcr_amd_$name.so
rm -rf "$tmp"
