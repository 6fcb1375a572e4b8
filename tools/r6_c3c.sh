#!/bin/bash
# round 6: kernel timelines of the C3 frame, batched chain vs staggered (graph replays)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 0 1048576; do
  PCP_BK_STAGGER=$s timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c3tl_$s -o run --output-format csv -- \
    python3 bench.py --mode filter --steps 20 --warmup 3 --no-pcie --no-cpu-baseline > gpurun_out/c3tl_$s.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/c3tl_$s.log; exit 1; }
  echo "== PCP_BK_STAGGER=$s"; python3 tools/c3_timeline.py gpurun_out/c3tl_$s
done
