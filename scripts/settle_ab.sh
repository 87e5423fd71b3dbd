#!/bin/bash
# bench.py at the driver's flags (--steps 20 --warmup 5), alternating
# --settle-ms over SETTLES (default "0 50"), ROUNDS rounds (one process per run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for i in $(seq 1 "${ROUNDS:-5}"); do
  for st in ${SETTLES:-0 50}; do
    out=$(timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --settle-ms $st 2>/dev/null | tail -n 1) || exit 1
    v=$(echo "$out" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["settle"])')
    echo "settle $st: $v"
  done
done
