#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/timeout (exit >= 124 or signal) ends the
# script immediately; plain test failures (exit 1) do not stop the later measurements.
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
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = test ]; then
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu -rf --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench 600 python bench.py
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --mode fan --steps 5 --warmup 2 --no-cpu-baseline
fi
if [ "$WHAT" = modes ]; then
  step bench_filter 300 python bench.py --mode filter --steps 10 --warmup 2
  step bench_cells 300 python bench.py --mode cells --steps 5 --warmup 1
fi
if [ "$WHAT" = pmc ] || [ "$WHAT" = modes ]; then
  # counters in their own passes (no trace domains besides kernel dispatch)
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
             "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    step pmc$i 300 rocprofv3 --pmc $set -d gpurun_out/pmc$i -o pmc --output-format csv -- python3 bench.py ${BENCH_ARGS:---mode fan --steps 3 --warmup 1 --no-cpu-baseline}
  done
fi
if [ "$WHAT" = traffic ]; then
  # FETCH_SIZE and WRITE_SIZE in separate passes, for the fan kernel and the filter pipeline
  step pmc_fan_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fan_fetch -o pmc --output-format csv -- python3 bench.py --mode fan --steps 3 --warmup 1 --no-cpu-baseline
  step pmc_fan_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_fan_write -o pmc --output-format csv -- python3 bench.py --mode fan --steps 3 --warmup 1 --no-cpu-baseline
  export PCP_NO_GRAPHS=1   # every pipeline kernel its own dispatch: 1 + 3 + 3 = 7 pipeline runs
  step pmc_flt_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_flt_fetch -o pmc --output-format csv -- python3 bench.py --mode filter --steps 3 --warmup 1 --no-pcie
  step pmc_flt_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_flt_write -o pmc --output-format csv -- python3 bench.py --mode filter --steps 3 --warmup 1 --no-pcie
  unset PCP_NO_GRAPHS
fi
echo "=== done"
