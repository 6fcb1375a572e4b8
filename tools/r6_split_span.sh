#!/bin/bash
# round 6: C5 frames' device span with and without the split scoring (kernel trace only)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do
  for v in "split:$L:PCP_SCORE_SPLIT=1" "nosplit:$L:PCP_SCORE_SPLIT=0" "head:$L/alt_head:PCP_X=0"; do
    name=${v%%:*}; rest=${v#*:}; d=${rest%%:*}; e=${rest#*:}
    rm -rf gpurun_out/span_${name}_$r
    env $e LD_LIBRARY_PATH=$d timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/span_${name}_$r -o k -- \
      $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB 60 60032 1 \
      > gpurun_out/span_${name}_$r.log 2>&1 || { tail -5 gpurun_out/span_${name}_$r.log; exit 1; }
  done
done
python3 tools/c5_span.py gpurun_out/span_*_[12]
