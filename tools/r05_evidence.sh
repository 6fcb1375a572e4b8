#!/bin/bash
# Round-5 evidence, in calls that each fit the gpurun limit (every GPU step its own limit; a
# crash or timeout ends the script):
#   G: the divergent lane-load ceiling (tools/gather_ceiling.sh -> profiles/r05_gather_ceiling.json)
#      and the fan's texture-path counters at this tree (tools/pmc_fan.sh + tools/pmc_gather.py
#      -> profiles/r05_fan_gather_path.json)
#   T: FETCH/WRITE passes of the fan and the C3 chain (parsed afterwards by tools/pmc_traffic.py
#      -> profiles/r05_pmc_traffic.json), the C3 chain's eager kernel stats
#   C: the C5 chain under a runtime + kernel trace (tools/c5_timeline.py / c5_sequence.py)
#   S: rocprofv3 kernel stats of the default bench command
#   A: every GPU test + smoke, the default bench line
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
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for part in "$@"; do
case "$part" in
G)
  # (the ceiling itself, tools/gather_ceiling.sh, is code-independent: re-run it with GC=1)
  if [ "${GC:-0}" = 1 ]; then step gather_ceiling 600 bash tools/gather_ceiling.sh; fi
  step pmc_fan_path 600 bash tools/pmc_fan.sh "" r05
  step pmc_gather 60 python3 tools/pmc_gather.py gpurun_out/r05_fan_gather_path.json gpurun_out/pmcfr05_1 gpurun_out/pmcfr05_2 gpurun_out/pmcfr05_3 gpurun_out/pmcfr05_4 gpurun_out/pmcfr05_5
  ;;
T)
  # (the counter passes only: tools/pmc_traffic.py parses them afterwards in the tree they
  # came from -- only gpurun_out/ comes back from the box)
  step pmc_fan_traffic 300 bash tools/pmc_fan_traffic.sh r05
  step pmc_flt_traffic 300 bash tools/pmc_filter_traffic.sh r05
  step c3_stats 300 env PCP_NO_GRAPHS=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --mode filter --steps 20 --warmup 3 --no-pcie --no-cpu-baseline
  ;;
C)
  step c5_trace 300 env FRAMES=30 bash tools/replay_trace.sh
  ;;
S)
  step rocprof_default 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run --output-format csv -- python3 bench.py
  ;;
A)
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -rf -s --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step bench 600 python bench.py
  ;;
esac
done
echo "=== done"
