#!/bin/bash
# round 6: reference-mode k_score_cells builds, one per process, alternating rounds:
#   bash tools/r6_cells_variants.sh lib1 lib2 ...   (paths under pointcloud_processor_amd/_lib)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for l in "$@"; do
    PCP_LIB=pointcloud_processor_amd/_lib/$l timeout -k 10 200 python bench.py --mode cells --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/cv_$r.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/cv_$r.json')); rm=d['detail']
print('r$r $l', 'step %.4f ms' % d['ms_per_step'], 'score_cells burst %.4f ms' % rm['roofline']['avg_kernel_ms'], 'frac %.3f' % rm['roofline']['frac'])"
  done
done
