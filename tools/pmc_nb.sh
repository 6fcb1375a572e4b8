#!/bin/bash
# SQ counters of the exact-normals kernels (k_nb_*) under bench.py --mode c1, two passes of <= 8
# SQ counters each (no trace domains with --pmc)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE"
i=0
for P in "$A" "$B"; do
  rm -rf gpurun_out/pmc_nb$i
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "k_nb_" -d gpurun_out/pmc_nb$i -o run --output-format csv -- python3 bench.py --mode c1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_nb$i.log 2>&1 || { echo "pass $i rc=$?"; tail -5 gpurun_out/pmc_nb$i.log; exit 1; }
  echo "pass $i ok"
  i=$((i+1))
done
