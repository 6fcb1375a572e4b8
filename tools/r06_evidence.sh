#!/bin/bash
# Round-6 evidence, in calls that each fit the gpurun limit (every GPU step its own limit; a
# crash or timeout ends the script):
#   G: the fan's texture-path counters (tools/pmc_fan.sh) and reference mode's k_score_cells
#      counter passes incl. FETCH/WRITE (tools/pmc_cells.sh) at this tree
#   T: FETCH/WRITE passes of the fan and the C3 chain, the C3 chain's eager kernel stats
#   C: the C5 chain under a runtime + kernel trace (tools/c5_timeline.py / c5_sequence.py)
#   S: rocprofv3 kernel stats of the default bench command
#   A: every GPU test + smoke, the default bench line
#   N: the N = 2 rehearsal (two ranks on the one GPU over gloo), reference mode
#   R: the default line through the distributed path at one rank (PCP_DIST_FORCE=1: host group,
#      libpcp's RCCL communicator, the one-collective queries, c4)
# parse afterwards (in this tree: only gpurun_out/ comes back):
#   python3 tools/pmc_gather.py profiles/r06_fan_gather_path.json fan gpurun_out/pmcfr06_[1-5]
#   python3 tools/pmc_gather.py profiles/r06_cells_gather_path.json cells gpurun_out/pmccr06_[1-5]
#   python3 tools/pmc_traffic.py fan "k_raycast_fan_xcd<0," gpurun_out/pmctr06_fetch gpurun_out/pmctr06_write per_dispatch r06_pmc_traffic.json profiles/r04_fetch_calibration.json
#   python3 tools/pmc_traffic.py filter "pcp::" gpurun_out/pmcfltr06_fetch gpurun_out/pmcfltr06_write steps=10 r06_pmc_traffic.json
#   python3 tools/pmc_traffic.py cells "k_score_cells<" gpurun_out/pmccr06_fetch gpurun_out/pmccr06_write per_dispatch r06_pmc_traffic.json
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
  step pmc_fan_path 600 bash tools/pmc_fan.sh "" r06
  step pmc_cells 900 bash tools/pmc_cells.sh r06
  ;;
T)
  step pmc_fan_traffic 300 bash tools/pmc_fan_traffic.sh r06
  step pmc_flt_traffic 300 bash tools/pmc_filter_traffic.sh r06
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
N)
  step bench_n2 600 python bench.py --gpus 2 --mode cells --steps 5 --warmup 2 --no-cpu-baseline
  ;;
R)
  step bench_rccl_n1 600 env WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 PCP_DIST_FORCE=1 python bench.py --gpus 1
  ;;
esac
done
echo "=== done"
