#!/bin/bash
# whole-step A/B of one bench mode: the committed build (alt_head) against the working tree's,
# alternating processes.  usage: tools/ab_step.sh MODE [extra bench args]
set -u
cd "$(dirname "$0")/.."
MODE=$1; shift
for r in 1 2 3; do
  for l in pointcloud_processor_amd/_lib/alt_head/libpcp.so pointcloud_processor_amd/_lib/libpcp.so; do
    PCP_LIB=$l timeout -k 10 200 python bench.py --mode $MODE --steps 40 --warmup 5 --no-cpu-baseline "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$MODE', '$l'.split('/')[-2], 'step %.4f ms  value %.4g' % (d['ms_per_step'], d['value']))" || exit 1
  done
done
