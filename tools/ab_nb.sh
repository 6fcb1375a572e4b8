#!/bin/bash
# A/B of the neighbour-list grid (PCP_NB_BLOCKS) under bench --mode c1, kernel stats per variant
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for nb in 2048 768 1536; do
  rm -rf gpurun_out/abnb_$nb
  PCP_NB_BLOCKS=$nb timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/abnb_$nb -o run --output-format csv -- python3 bench.py --mode c1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/abnb_$nb.log 2>&1 || { echo "nb $nb rc=$?"; exit 1; }
  echo "nb $nb ok"
done
