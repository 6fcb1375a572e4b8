#!/bin/bash
# round 6: k_bk_sort with 256-thread blocks and a 2,048-point bucket cap (six blocks per CU
# instead of four: LDS 26.7 vs 37.0 KB) -- parity, then the C3 frame and C5, alternating
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
ALT=$L/alt_t256/libpcp.so
PCP_LIB=$ALT timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "bucket_chain or full_c3 or graph_redo or crop_voxel or filter_merge" > gpurun_out/r6_t256_tests.log 2>&1
tail -3 gpurun_out/r6_t256_tests.log
grep -E "FAILED|assert" gpurun_out/r6_t256_tests.log | head -10
for r in 1 2 3; do
  for l in $L/libpcp.so $ALT; do
    PCP_LIB=$l timeout -k 10 120 python bench.py --mode filter --steps 50 --warmup 5 --no-pcie --no-cpu-baseline 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r$r', '$l'.split('/')[-2], 'step %.4f ms  device %.4f ms' % (d['ms_per_step'], d['roofline']['avg_kernel_ms']))" || exit 1
  done
done
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do
  for d in $L $L/alt_t256; do
    LD_LIBRARY_PATH=$d timeout -k 10 300 $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c5 r$r $d p50 %.4f p99 %.4f' % (d['p50_ms'], d['p99_ms']), 'filter', d['stage_p50_ms']['filter'])" || exit 1
  done
done
