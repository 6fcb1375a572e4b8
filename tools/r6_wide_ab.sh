#!/bin/bash
# round 6: k_score_cells_wide (G lanes per ray) for more than the default 32 k rays -- C5's tick
# (replay, 200 frames) and reference mode (bench.py --mode cells), alternating processes
set -u
cd "$(dirname "$0")/.."
ROUNDS=${ROUNDS:-2} bash tools/c5_env_ab.sh "base:PCP_X=0" "w2:PCP_SCORE_WIDE_RAYS=100000000,PCP_SCORE_WIDE_G=2" \
  "w4:PCP_SCORE_WIDE_RAYS=100000000,PCP_SCORE_WIDE_G=4" "w8:PCP_SCORE_WIDE_RAYS=100000000,PCP_SCORE_WIDE_G=8" || exit 1
for r in 1 2; do
  for v in "base:PCP_X=0" "w2:PCP_SCORE_WIDE_RAYS=100000000,PCP_SCORE_WIDE_G=2" "w4:PCP_SCORE_WIDE_RAYS=100000000,PCP_SCORE_WIDE_G=4"; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 120 python bench.py --mode cells --steps 30 --warmup 3 --no-cpu-baseline 2>/dev/null | grep '^{' | python -c "
import json,sys; d=json.loads(sys.stdin.read()); x=d['detail']
print('cells r$r $name %.0f poses/s  step %.4f ms' % (d['value'], d['ms_per_step']), x['kernel_avg_ms'], 'best', d['best_pose'], 'burst', x['roofline']['avg_kernel_ms'])" || exit 1
  done
done
