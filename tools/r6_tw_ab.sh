#!/bin/bash
# round 6: k_score_cells with TW cells x 64/TW rows per wave (PCP_SCORE_TW) -- parity, then
# reference mode and C5, alternating processes
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
VARS="prod alt_tw16 alt_tw8 alt_tw4"
lib() { [ "$1" = prod ] && echo $L/libpcp.so || echo $L/$1/libpcp.so; }
for v in $VARS; do
  PCP_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
    -k "score or parity_bar" > gpurun_out/r6_tw_tests_$v.log 2>&1 || { echo "$v PARITY FAIL"; tail -30 gpurun_out/r6_tw_tests_$v.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/r6_tw_tests_$v.log)"
done
for r in 1 2 3; do
  for v in $VARS; do
    PCP_LIB=$(lib $v) timeout -k 10 120 python bench.py --mode cells --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | grep '^{' | python -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d['detail']; R=x['roofline']
print('cells r$r $v %.0f poses/s step %.4f ms' % (d['value'], d['ms_per_step']), 'burst %.4f' % R['avg_kernel_ms'], 'frac %.3f' % R['frac'], 'best', d['best_pose'])" || exit 1
  done
done
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
for r in 1 2; do
  for v in $VARS; do
    d=$L; [ "$v" != prod ] && d=$L/$v
    LD_LIBRARY_PATH=$d timeout -k 10 300 $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c5 r$r $v p50 %.4f p99 %.4f' % (d['p50_ms'], d['p99_ms']), 'tick', d['stage_p50_ms']['tick'])" || exit 1
  done
done
