#!/bin/bash
# round 6: the one-collective queries' landing in one copy (fan: keys + units by one copy
# kernel; scoring: flags in the query's upload, one landing kernel) -- parity tests, then the
# distributed path at one rank (PCP_DIST_FORCE=1) for the per-step cost
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "allreduce or multi or keys or score or parity_bar" > gpurun_out/r6_land_tests.log 2>&1 || { tail -30 gpurun_out/r6_land_tests.log; exit 1; }
tail -1 gpurun_out/r6_land_tests.log
for r in 1 2; do
  WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 PCP_DIST_FORCE=1 timeout -k 10 300 python bench.py --gpus 1 --mode fan --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('fan dist r$r %.4f ms/step' % d['ms_per_step'], d.get('collective',{}).get('collective_ms'))" || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --mode fan --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('fan plain r$r %.4f ms/step' % d['ms_per_step'])" || exit 1
  WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 PCP_DIST_FORCE=1 timeout -k 10 300 python bench.py --gpus 1 --mode cells --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('cells dist r$r %.4f ms/step %.3g poses/s' % (d['ms_per_step'], d['value']), d['detail'].get('collective'))" || exit 1
  timeout -k 10 300 python bench.py --gpus 1 --mode cells --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('cells plain r$r %.4f ms/step %.3g poses/s' % (d['ms_per_step'], d['value']))" || exit 1
done
