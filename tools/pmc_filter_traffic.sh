#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes of the C3 filter chain (eager launches: every kernel its own
# dispatch), one pass each: gpurun_out/pmcflt${TAG}_{fetch,write}/
# parse: python tools/pmc_traffic.py filter "pcp::" gpurun_out/pmcflt${TAG}_fetch gpurun_out/pmcflt${TAG}_write steps=N
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PCP_NO_GRAPHS=1
TAG=${1:-}
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmcflt${TAG}_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $c -d $d -o pmc --output-format csv -- python3 bench.py --mode filter --steps 3 --warmup 1 --no-pcie --no-cpu-baseline > $d.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$c rc=$rc"; tail -20 $d.log; exit $rc; fi
done
echo done
