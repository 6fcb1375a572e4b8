#!/bin/bash
# C5 A/B of a variant build of libpcp (LD_LIBRARY_PATH ahead of the CLI's $ORIGIN runpath)
# against the tree's own: the full-chain replay, 200 frames, alternating, two rounds.
#   LIBS="pointcloud_processor_amd/_lib/altp4 pointcloud_processor_amd/_lib" bash tools/c5_lib_ab.sh
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/replay
FRAMES=2 timeout -k 10 300 bash tools/replay.sh > /dev/null 2>&1 || exit 1
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do for l in $LIBS; do
  LD_LIBRARY_PATH=$l timeout -k 10 300 pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
    gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-200} 60032 1 > gpurun_out/c5lib.json || exit 1
  echo "round $r $(basename $l): $(grep -o '"p50_ms": [0-9.]*, "p99_ms": [0-9.]*' gpurun_out/c5lib.json) $(grep -o '"stage_p50_ms": {[^}]*}' gpurun_out/c5lib.json)"
done; done
