#!/bin/bash
# Divergent lane-load ceiling of gfx950 (tools/mb/gather_ceiling.hip): one plain run (rates,
# clocks), one rocprofv3 --pmc pass of the same runs (TA / TD busy, L1 tags and misses per
# dispatch), then tools/gather_ceiling.py -> gpurun_out/r05_gather_ceiling.json (committed as
# profiles/r05_gather_ceiling.json: bench.py's fan roofline peak).
# usage (GPU box): tools/gather_ceiling.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -x tools/mb/gather_ceiling ] || { echo "build tools/mb/gather_ceiling first"; exit 1; }
timeout -k 10 240 tools/mb/gather_ceiling 10 > gpurun_out/gceil.jsonl 2> gpurun_out/gceil.err \
  || { echo "gather_ceiling rc=$?"; cat gpurun_out/gceil.err; exit 1; }
# 2 reps: 3 dispatches per run (warm-up + 2), in the plain run's order
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
  -d gpurun_out/gceil_pmc -o pmc --output-format csv -- tools/mb/gather_ceiling 2 > gpurun_out/gceil_pmc.log 2>&1 \
  || { echo "pmc rc=$?"; tail -20 gpurun_out/gceil_pmc.log; exit 1; }
python3 tools/gather_ceiling.py gpurun_out/gceil.jsonl gpurun_out/r05_gather_ceiling.json gpurun_out/gceil_pmc
