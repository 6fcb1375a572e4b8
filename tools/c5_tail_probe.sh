#!/bin/bash
# C5 replay repeated (ROUNDS x 200 frames), the slowest frames' stage times per run
set -u
cd "$(dirname "$0")/.."
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in $(seq 1 ${ROUNDS:-5}); do
  env ${ENVS:-X=1} timeout -k 10 200 pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
    gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('r$r p50 %.4f p99 %.4f max %.4f' % (d['p50_ms'], d['p99_ms'], d['max_ms']))
for s in d['slowest'][:3]:
    print('   ', {k: round(v, 3) if isinstance(v, float) else v for k, v in s.items()})" || exit 1
done
