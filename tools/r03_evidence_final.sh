#!/bin/bash
# Round-3 evidence at the final tree in one call: every GPU test + smoke, the default bench line,
# the C5 replay (200 frames), the default bench under rocprofv3 --kernel-trace --stats, and the
# C3 FETCH_SIZE / WRITE_SIZE passes.  Stops at the first GPU step that crashes or times out.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/r03_final.sh A || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python3 bench.py > gpurun_out/rocprof_default.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
bash tools/pmc_filter_traffic.sh r03c || exit 1
echo "=== evidence done"
