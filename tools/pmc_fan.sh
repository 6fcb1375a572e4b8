#!/bin/bash
# Counter passes for the fan kernel (one rocprofv3 --pmc pass per set, kernel dispatch only).
# usage: tools/pmc_fan.sh [PCP_FAN_BATCH]   -> gpurun_out/pmcf*/ ; parse with tools/pmc_table.py
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
[ $# -ge 1 ] && export PCP_FAN_BATCH=$1
i=0
for set in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum" "TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d gpurun_out/pmcf$i -o pmc --output-format csv -- python3 bench.py --mode fan --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -20 gpurun_out/pmcf$i.log; exit $rc; fi
done
echo done
