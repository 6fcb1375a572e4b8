#!/bin/bash
# reference-mode step A/B: the committed build (alt_head) against the working tree's
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for l in pointcloud_processor_amd/_lib/alt_head/libpcp.so pointcloud_processor_amd/_lib/libpcp.so; do
    PCP_LIB=$l timeout -k 10 120 python bench.py --mode cells --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l'.split('/')[-2], '%.0f poses/s  step %.4f ms' % (d['value'], d['ms_per_step']), d['detail']['kernel_avg_ms'])" || exit 1
  done
done
