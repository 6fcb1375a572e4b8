#!/bin/bash
# per-kernel rocprofv3 stats of the C3 frame for the committed build (alt_head) and the working tree's
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in alt_head new; do
  if [ $v = alt_head ]; then export PCP_LIB=pointcloud_processor_amd/_lib/alt_head/libpcp.so; else unset PCP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3p_$v -o run --output-format csv -- \
    python3 bench.py --mode filter --steps 20 --warmup 3 --no-pcie --no-cpu-baseline > gpurun_out/c3p_$v.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/c3p_$v.log; exit 1; }
  echo "== $v"; find gpurun_out/c3p_$v -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \;
done
