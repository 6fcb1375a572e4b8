#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate runs) of the fan kernel: gpurun_out/pmct${TAG}_{fetch,write}/
# parse: python tools/pmc_traffic.py fan "k_raycast_fan<0, 64, true, 8, 1>" gpurun_out/pmct${TAG}_fetch gpurun_out/pmct${TAG}_write
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-}
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmct${TAG}_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $c -d $d -o pmc --output-format csv -- python3 bench.py --mode fan --steps 3 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$c rc=$rc"; tail -20 $d.log; exit $rc; fi
done
echo done
