#!/bin/bash
# round 6: reference-mode scoring with correctly rounded acos / sin (pcp_score_sin_part, inline
# in k_score_cells: the default) vs ocml's (alt_ocml: make OUTDIR=../_lib/alt_ocml
# EXTRA=-DPCP_SCORE_OCML), alternating processes; then C1.  (Earlier variants of the round, each
# measured with this script: the Taylor double-double path inline 93 us, a separate compacted
# k_score_cr pass 62-90 us, an LDS queue per block 78 us; ocml 44 us.)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for l in alt_ocml/libpcp.so libpcp.so; do
    PCP_LIB=pointcloud_processor_amd/_lib/$l timeout -k 10 200 python bench.py --mode cells --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/crab_$r.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/crab_$r.json')); rm=d['detail']
print('$l', 'step %.4f ms' % d['ms_per_step'], 'score_cells burst %.4f ms' % rm['roofline']['avg_kernel_ms'], 'events', {k: round(v, 4) for k, v in rm['kernel_avg_ms'].items()})"
  done
done
for r in 1 2; do
  for l in alt_ocml/libpcp.so libpcp.so; do
    PCP_LIB=pointcloud_processor_amd/_lib/$l timeout -k 10 200 python bench.py --mode c1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/crc1_$r.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/crc1_$r.json')); print('$l C1', 'ms/frame %.4f p99 %.4f' % (d['value'], d['p99_ms']))"
  done
done
