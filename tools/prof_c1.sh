#!/bin/bash
# kernel-trace summary of bench.py --mode c1 (BASELINE configs[0]: the whole chain per frame)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run --output-format csv -- python3 bench.py --mode c1 --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/prof_c1.log 2>&1
rc=$?
echo "prof_c1 rc=$rc"
tail -2 gpurun_out/prof_c1.log
exit $rc
