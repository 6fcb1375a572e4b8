#!/bin/bash
# round 6: the tick's ray march beside the setup's normals (PCP_SCORE_SPLIT, default 1: march ->
# join -> k_score_finish) against the march after the join (0) and the committed build
# (alt_head): the GPU suite first, then C5 (200 frames) and C1, alternating processes
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r6_split_tests.log 2>&1 || { tail -40 gpurun_out/r6_split_tests.log; exit 1; }
tail -1 gpurun_out/r6_split_tests.log
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in 1 2 3; do
  for v in "split:$L:PCP_SCORE_SPLIT=1" "nosplit:$L:PCP_SCORE_SPLIT=0" "head:$L/alt_head:PCP_X=0"; do
    name=${v%%:*}; rest=${v#*:}; d=${rest%%:*}; e=${rest#*:}
    env $e LD_LIBRARY_PATH=$d timeout -k 10 300 $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c5 r$r $name p50 %.4f p99 %.4f max %.4f' % (d['p50_ms'], d['p99_ms'], d['max_ms']), d['stage_p50_ms'])" || exit 1
  done
done
for r in 1 2; do
  for v in "split:$L/libpcp.so:PCP_SCORE_SPLIT=1" "nosplit:$L/libpcp.so:PCP_SCORE_SPLIT=0" "head:$L/alt_head/libpcp.so:PCP_X=0"; do
    name=${v%%:*}; rest=${v#*:}; l=${rest%%:*}; e=${rest#*:}
    env $e PCP_LIB=$l timeout -k 10 200 python bench.py --mode c1 --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d.get('c1', d)
print('c1 r$r $name %.4f ms/frame p99 %.4f' % (c['value'], c['p99_ms']), 'oracle', c.get('matches_oracle'))" || exit 1
  done
done
