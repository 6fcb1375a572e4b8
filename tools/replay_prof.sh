#!/bin/bash
# kernel-trace summary of the full-chain C5 replay (FRAMES frames)
set -eu
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
FRAMES=${FRAMES:-3} bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
rm -rf gpurun_out/prof_replay
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_replay -o run --output-format csv -- pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-3} 60032 1 > gpurun_out/prof_replay.log 2>&1
python3 tools/kstats.py gpurun_out/prof_replay/run_kernel_stats.csv ${FRAMES:-3}
