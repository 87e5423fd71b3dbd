#!/bin/bash
# PMC passes over a short c2 bench (one pass per counter group, each
# its own run): FETCH_SIZE, WRITE_SIZE, fabric read / write request counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python3 bench.py --steps 5 --warmup 5 --steps-per-launch 5 --no-cpu-baseline --no-verify"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- $B > gpurun_out/pmc_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
pass wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
python3 scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_traffic.json 32 1024 32 32 64 gpurun_out/pmc_rdreq gpurun_out/pmc_wrreq > gpurun_out/pmc_json.log 2>&1; tail -c 2000 gpurun_out/pmc_json.log
