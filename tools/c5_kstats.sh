#!/bin/bash
# C5 replay kernel statistics (rocprofv3 --kernel-trace --stats): gpurun_out/c5ks_$TAG/
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
TAG=${TAG:-x}
rm -rf gpurun_out/c5ks_$TAG
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c5ks_$TAG -o run --output-format csv -- \
  pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
  gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-50} 60032 1 > gpurun_out/c5ks_$TAG.log 2>&1
