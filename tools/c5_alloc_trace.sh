#!/bin/bash
# C5 full chain with PCP_ALLOC_TRACE=1: every device / pinned (re)allocation and its site
# (offset into libpcp.so; resolve with addr2line), framed by "replay frame N" markers
set -u
cd "$(dirname "$0")/.."
FRAMES=${FRAMES:-40}
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
PCP_ALLOC_TRACE=1 timeout -k 10 200 pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
  gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB $FRAMES 60032 1 \
  > gpurun_out/c5_alloc_trace.json 2> gpurun_out/c5_alloc_trace.err
