#!/bin/bash
# A/B of a fine-copy walk knob on the C2 fan: the point-test census of both settings (census
# build, make census), the fan kernel in one process with interleaved rounds (tools/fan_ab.py,
# bit-identical outputs asserted), the copy's build time, and the fine-copy parity tests.
#   KNOB=PCP_FINE_SKIP A=1 B=2 bash tools/fan_skip_ab.sh
# (round 3: PCP_FINE_SKIP 1 vs 2 -> profiles/r03_fan_ab_skip2.log; quadrant sub-windows, a knob
# of that build since removed -> profiles/r03_fan_ab_subwin.log)
set -u
cd "$(dirname "$0")/.."
KNOB=${KNOB:-PCP_FINE_SKIP}; A=${A:-1}; B=${B:-2}
mkdir -p gpurun_out
for s in $A $B; do
  env $KNOB=$s PCP_LIB=pointcloud_processor_amd/_lib/census/libpcp.so timeout -k 10 300 \
    python3 -u tools/fan_walk_census.py > gpurun_out/fan_walk_census_$s.json || exit 1
  echo "census $KNOB=$s: $(cat gpurun_out/fan_walk_census_$s.json)"
done
timeout -k 10 300 python3 -u tools/fan_ab.py a:$KNOB=$A b:$KNOB=$B || exit 1
timeout -k 10 300 python3 -u tools/fan_ab.py b:$KNOB=$B a:$KNOB=$A || exit 1
for s in $A $B; do
  echo "fine build $KNOB=$s: $(env $KNOB=$s timeout -k 10 300 python3 -u tools/fine_build_time.py | tail -1)" || exit 1
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "poses_per_wave or far_from_origin or full_c2 or fine or score" > gpurun_out/skip_tests.log 2>&1
rc=$?; tail -3 gpurun_out/skip_tests.log; exit $rc
