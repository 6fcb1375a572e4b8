#!/bin/bash
# Counter passes for reference mode's k_score_cells (bench.py --mode cells): the texture-path and
# wave-state sets of tools/pmc_fan.sh, then FETCH_SIZE / WRITE_SIZE (separate passes).
# -> gpurun_out/pmcc${TAG}_*/ ; parse: python tools/pmc_gather.py OUT.json cells gpurun_out/pmcc${TAG}_[0-9]*
#    and python tools/pmc_traffic.py cells "k_score_cells<" gpurun_out/pmcc${TAG}_fetch gpurun_out/pmcc${TAG}_write ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-}
i=0
for set in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" \
           "SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  d=gpurun_out/pmcc${TAG}_$i
  [ "$set" = FETCH_SIZE ] && d=gpurun_out/pmcc${TAG}_fetch
  [ "$set" = WRITE_SIZE ] && d=gpurun_out/pmcc${TAG}_write
  timeout -s KILL 180 rocprofv3 --pmc $set -d $d -o pmc --output-format csv -- python3 bench.py --mode cells --steps 2 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -20 $d.log; exit $rc; fi
done
echo done
