#!/bin/bash
# kernel-trace summary of the C3 filter pipeline (eager = one dispatch per kernel, and graph)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_flt_eager gpurun_out/prof_flt_graph
PCP_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flt_eager -o run --output-format csv -- python3 bench.py --mode filter --steps 10 --warmup 2 > gpurun_out/prof_flt_eager.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_flt_graph -o run --output-format csv -- python3 bench.py --mode filter --steps 10 --warmup 2 > gpurun_out/prof_flt_graph.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/prof_flt_eager/run_kernel_stats.csv 15
python3 tools/kstats.py gpurun_out/prof_flt_graph/run_kernel_stats.csv 15
