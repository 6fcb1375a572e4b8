#!/bin/bash
# Fan, VERDICT r4 item 7: the walk start folded into the probe record (PCP_FINE_TILE=1: one
# 8-byte record {walk start, z band} per fine cell in 4 x 4 tiles -- a candidate needs no second
# load) against the split records (PCP_FINE_TILE=2, default: 2-byte z-band probes in 8 x 8 tiles,
# the 4-byte walk start loaded by candidates only).  Alternating processes, bench.py --mode fan
# (50 steps): kernel time, step time, and each variant's lane-load split (pcp_raycast_fan_stats)
set -u
cd "$(dirname "$0")/.."
for r in 1 2 3; do
  for v in "split:PCP_FINE_TILE=2" "fold:PCP_FINE_TILE=1"; do
    name=${v%%:*}; env=${v#*:}
    env $env timeout -k 10 200 python bench.py --mode fan --steps 50 --warmup 5 --no-cpu-baseline 2>/dev/null \
      | grep '^{' | python3 -c "
import json, sys
d = json.loads(sys.stdin.read()); r = d['roofline']; st = r['diag']
print('r$r $name kernel %.4f ms  step %.4f ms  probes %.1fM walk-starts %.1fM point-records %.1fM lane-loads %.1fM  frac %.3f  value %.4g  layout %s tile %s' % (
    r['avg_kernel_ms'], d['ms_per_step'], st['samples_visited'] / 1e6, st['scanned_stencils'] / 1e6,
    st['point_tests'] / 1e6, r['executed_lane_loads'] / 1e6, r['frac'] or 0, d['value'], r['scan_layout'], r['kernel']))" || exit 1
  done
done
