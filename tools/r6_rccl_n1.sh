#!/bin/bash
# round 6: the SCALE path's code (host group, libpcp's RCCL communicator, one collective per
# fan / reference-mode query, c4) at one rank on the one-GPU box (PCP_DIST_FORCE=1)
set -u
cd "$(dirname "$0")/.."
WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 PCP_DIST_FORCE=1 timeout -k 10 500 python bench.py --gpus 1 > gpurun_out/r6_rccl_n1.log 2>&1
rc=$?
grep '^{' gpurun_out/r6_rccl_n1.log | tail -1 > gpurun_out/r6_rccl_n1.json
tail -3 gpurun_out/r6_rccl_n1.log | cut -c1-300
exit $rc
