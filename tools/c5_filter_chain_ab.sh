#!/bin/bash
# C5 replay (200 frames per run) with the bucket chain (PCP_FM_FAST=2, default) and the LSD fast chain (1) for the
# two 60k-point scans' crop + voxel, alternating runs: filter stage p50 and frame p50 (r04: the bucket chain stays)
set -u
cd /root/repo
for f in 2 1 2 1; do
  PCP_FM_FAST=$f FRAMES=200 timeout -k 10 300 bash tools/replay.sh > gpurun_out/fm_$f.log 2>&1 || { echo "fm $f failed"; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/fm_$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('FM=$f chain', d['chain'], 'p50', d['p50_ms'], 'p99', d['p99_ms'], 'filter', d['stage_p50_ms']['filter'], 'merge', d['stage_p50_ms']['merge'], 'best', d['best_idx'])"
done
