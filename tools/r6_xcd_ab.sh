#!/bin/bash
# round 6: k_score_cells rows grouped per XCD (PCP_SCORE_XCD=1: XCD x takes a run of
# neighbouring candidates) -- parity, reference mode and C5, alternating processes
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
ALT=$L/alt_xcd/libpcp.so
PCP_LIB=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "score or parity_bar or candidates_match" > gpurun_out/r6_xcd_tests.log 2>&1 || { tail -30 gpurun_out/r6_xcd_tests.log; exit 1; }
tail -1 gpurun_out/r6_xcd_tests.log
for r in 1 2 3; do
  for l in $L/libpcp.so $ALT; do
    PCP_LIB=$l timeout -k 10 120 python bench.py --mode cells --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | grep '^{' | python -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d['detail']; R=x['roofline']
print('cells r$r', '$l'.split('/')[-2], '%.0f poses/s step %.4f ms burst %.4f frac %.3f best %d' % (d['value'], d['ms_per_step'], R['avg_kernel_ms'], R['frac'], d['best_pose']))" || exit 1
  done
done
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do
  for d in $L $L/alt_xcd; do
    LD_LIBRARY_PATH=$d timeout -k 10 300 $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c5 r$r $d p50 %.4f p99 %.4f' % (d['p50_ms'], d['p99_ms']), 'tick', d['stage_p50_ms']['tick'])" || exit 1
  done
done
