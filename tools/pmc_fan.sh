#!/bin/bash
# Counter passes for the fan kernel (one rocprofv3 --pmc pass per set, kernel dispatch only).
# usage: tools/pmc_fan.sh [PCP_FAN_BATCH] [TAG]  -> gpurun_out/pmcf${TAG}_*/ ; parse with
#        python tools/pmc_table.py k_raycast_fan gpurun_out/pmcf${TAG}_*
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
[ $# -ge 1 ] && export PCP_FAN_BATCH=$1
TAG=${2:-}
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmcf${TAG}_$i -o pmc --output-format csv -- python3 bench.py --mode fan --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmcf${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -20 gpurun_out/pmcf${TAG}_$i.log; exit $rc; fi
done
echo done
