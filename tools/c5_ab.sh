#!/bin/bash
# C5 A/B over one env knob: the GPU tests once, then the replay (chain 1) alternating the knob's
# values, two rounds.  KNOB=NAME VALUES="a b" bash tools/c5_ab.sh; outputs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/replay
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nodes_cli.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5ab_tests.log 2>&1 || { tail -40 gpurun_out/c5ab_tests.log; exit 1; }
  tail -1 gpurun_out/c5ab_tests.log
fi
FRAMES=2 timeout -k 10 300 bash tools/replay.sh > /dev/null 2>&1 || exit 1   # writes the inputs
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do for v in $VALUES; do
  env "$KNOB=$v" timeout -k 10 300 pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
    gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-200} 60032 1 > gpurun_out/c5ab_$v.json || exit 1
  echo "round $r $KNOB=$v: $(grep -o '"p50_ms": [0-9.]*, "p99_ms": [0-9.]*' gpurun_out/c5ab_$v.json) $(grep -o '"stage_p50_ms": {[^}]*}' gpurun_out/c5ab_$v.json)"
done; done
