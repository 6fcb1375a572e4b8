#!/bin/bash
# round 6: per-kernel times of reference mode (bench.py --mode cells) for the ocml build and the
# correctly rounded one (k_score_cells + k_score_cr)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in alt_ocml new; do
  if [ $v = alt_ocml ]; then export PCP_LIB=pointcloud_processor_amd/_lib/alt_ocml/libpcp.so; else unset PCP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/crp_$v -o run --output-format csv -- \
    python3 bench.py --mode cells --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/crp_$v.log 2>&1 || { echo "$v rc=$?"; tail -5 gpurun_out/crp_$v.log; exit 1; }
  echo "== $v"; find gpurun_out/crp_$v -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \; | grep -i "score\|sum_flags\|row_sum\|Name"
done
