#!/bin/bash
# Round-4 evidence, in calls that each fit the 20-minute gpurun limit:
#   A: every GPU test + smoke, the default bench line, the C5 replay (200 frames)
#   B: rocprofv3 kernel stats of the default bench, FETCH/WRITE passes (fan, filter), the gather
#      FETCH_SIZE calibration (tools/gather_cal.sh)
#   C: the C5 replay under a kernel trace (per-stage kernels of the exact normals)
# Each GPU step has its own limit; a crash or timeout ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
case "${1:-A}" in
A)
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -rf -s --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 600 python bench.py
  FRAMES=200 step replay 600 bash tools/replay.sh
  step top2 600 python tools/c5_top2.py 8 gpurun_out/r04_c5_top2_gaps.json
  ;;
B)
  step rocprof_default 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python3 bench.py
  step pmc_fan 300 bash tools/pmc_fan_traffic.sh r04
  step pmc_flt 300 bash tools/pmc_filter_traffic.sh r04
  step gather_cal 300 bash tools/gather_cal.sh
  ;;
C)
  FRAMES=50 step rocprof_replay 900 bash tools/replay_prof.sh
  ;;
esac
echo "=== done"
