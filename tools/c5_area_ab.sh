#!/bin/bash
# C5 full chain, alternating processes, 200 frames each (p50 / p99 and the stage p50s):
#   new  = the filter + merger nodes composed (PCP_FRONT_FUSED=1) + the grid setup deferred to
#          the tick (PCP_AREA_ASYNC=1)  -- the replay's defaults
#   area = the grid deferred only;  old = neither (round 4's chain)
set -u
cd "$(dirname "$0")/.."
FRAMES=${FRAMES:-200}
ROUNDS=${ROUNDS:-3}
bash tools/replay.sh > /dev/null 2>&1 || true   # writes gpurun_out/replay/* (inputs)
read TN CN BB < gpurun_out/replay/args
CLI=pointcloud_processor_amd/_lib/pcp_nodes_cli
for r in $(seq 1 $ROUNDS); do
  for v in "new 1 1" "area 1 0" "old 0 0"; do
    set -- $v
    name=$1; a=$2; f=$3
    PCP_AREA_ASYNC=$a PCP_FRONT_FUSED=$f timeout -k 10 300 $CLI replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB $FRAMES 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('r$r $name p50 %.4f p99 %.4f max %.4f' % (d['p50_ms'], d['p99_ms'], d['max_ms']), d['stage_p50_ms'])" || exit 1
  done
done
