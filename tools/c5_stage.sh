#!/bin/bash
# C5 iteration: the excavation/node parity tests, the replay with per-callback stage times, and
# the runtime trace's per-frame kernel table.  Outputs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nodes_cli.py -x -q --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/c5s_tests.log 2>&1 || { tail -40 gpurun_out/c5s_tests.log; exit 1; }
tail -2 gpurun_out/c5s_tests.log
FRAMES=200 timeout -k 10 600 bash tools/replay.sh > gpurun_out/replay.log 2>&1 || { tail gpurun_out/replay.log; exit 1; }
grep -o '"chain": [01], "p50_ms": [0-9.]*, "p99_ms": [0-9.]*\|"stage_p50_ms": {[^}]*}\|"slowest": \[[^]]*\]' gpurun_out/replay.log
FRAMES=30 timeout -k 10 400 bash tools/replay_trace.sh > gpurun_out/trace.log 2>&1 || exit 1
python3 tools/c5_timeline.py gpurun_out/c5tl > gpurun_out/c5_timeline.txt
python3 tools/c5_sequence.py gpurun_out/c5tl > gpurun_out/c5_sequence.txt
head -14 gpurun_out/c5_timeline.txt
