#!/bin/bash
# round 6, VERDICT r5 item 1: k_bk_sort's in-order voxel sums read from LDS (the bucket's points
# staged as gathered, no second gather from xyz; build: _lib/alt_ldssum, the k_bk_sort hunks of
# tools/ab/r06_c3_stagger_and_lds_sums.patch) -- parity, PMC traffic per kernel, frame time A/B
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
ALT=pointcloud_processor_amd/_lib/alt_ldssum/libpcp.so
PCP_LIB=$ALT timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "bucket_chain or full_c3 or graph_redo or crop_voxel" > gpurun_out/r6_ldssum_tests.log 2>&1 || { tail -30 gpurun_out/r6_ldssum_tests.log; exit 1; }
tail -2 gpurun_out/r6_ldssum_tests.log
PCP_LIB=$ALT bash tools/pmc_filter_traffic.sh ldssum || exit 1
bash tools/pmc_filter_traffic.sh prod6 || exit 1
for r in 1 2 3; do
  for l in pointcloud_processor_amd/_lib/libpcp.so $ALT; do
    PCP_LIB=$l timeout -k 10 120 python bench.py --mode filter --steps 50 --warmup 5 --no-pcie --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r$r', '$l'.split('/')[-2], 'step %.4f ms  device %.4f ms' % (d['ms_per_step'], d['roofline']['avg_kernel_ms']))" || exit 1
  done
done
