#!/bin/bash
# C5 full chain, alternating processes, 200 frames each, variants as environments:
#   bash tools/c5_env_ab.sh "name:ENV=V,ENV=V" ...      (ROUNDS, FRAMES)
set -u
cd "$(dirname "$0")/.."
FRAMES=${FRAMES:-200}
ROUNDS=${ROUNDS:-3}
bash tools/replay.sh > /dev/null 2>&1 || true   # writes gpurun_out/replay/* (inputs)
read TN CN BB < gpurun_out/replay/args
CLI=pointcloud_processor_amd/_lib/pcp_nodes_cli
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 300 $CLI replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB $FRAMES 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('r$r $name p50 %.4f p99 %.4f max %.4f realloc %d' % (d['p50_ms'], d['p99_ms'], d['max_ms'], d['reallocs_after_warmup']), d['stage_p50_ms'])" || exit 1
  done
done
