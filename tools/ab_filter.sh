#!/bin/bash
# C3 frame A/B: the committed build (alt_head) against the working tree's, alternating processes
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for l in pointcloud_processor_amd/_lib/alt_head/libpcp.so pointcloud_processor_amd/_lib/libpcp.so; do
    PCP_LIB=$l timeout -k 10 120 python bench.py --mode filter --steps 30 --warmup 3 --no-pcie --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$l'.split('/')[-2], 'step %.4f ms  device %.4f ms' % (d['ms_per_step'], d['roofline']['avg_kernel_ms']), {k: round(v, 4) for k, v in d['roofline'].get('eager_stage_ms', {}).items()})" || exit 1
  done
done
