#!/bin/bash
# reference-mode step over several library builds, alternating: bash tools/ab_libs.sh DIR...
# (DIR under pointcloud_processor_amd/_lib; "." = the working tree's build)
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
  for d in "$@"; do
    PCP_LIB=pointcloud_processor_amd/_lib/$d/libpcp.so timeout -k 10 120 python bench.py --mode cells --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$d', '%.0f poses/s  step %.4f ms' % (d['value'], d['ms_per_step']), d['detail']['kernel_avg_ms'])" || exit 1
  done
done
