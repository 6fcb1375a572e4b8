#!/bin/bash
# C3 frame diagnostics on one GPU: per-tile phase stamps of the sort scatter / centroid
# (diagnostic build, tools/filter_stamps.py) and a rocprofv3 kernel trace of the filter bench.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/filter_stamps.py > gpurun_out/c3_stamps.log 2>&1 || { echo "stamps rc=$?"; tail -20 gpurun_out/c3_stamps.log; exit 1; }
cat gpurun_out/c3_stamps.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o run --output-format csv -- \
  python3 bench.py --mode filter --steps 20 --warmup 3 --no-pcie --no-cpu-baseline > gpurun_out/c3_bench.log 2>&1 || { echo "rocprof rc=$?"; tail -20 gpurun_out/c3_bench.log; exit 1; }
tail -1 gpurun_out/c3_bench.log
find gpurun_out/c3prof -name '*kernel_stats.csv' -exec cat {} \;
