#!/bin/bash
# C3 frame timing of libpcp builds / knobs, one variant per process, alternating rounds:
#   bash tools/c3_variants.sh "name:ENV=V,ENV=V[:lib]" ...
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; env=${rest%%:*}; lib=""
    [ "$rest" != "$env" ] && lib=${rest#*:}
    if [ -n "$lib" ]; then export PCP_LIB=$lib; else unset PCP_LIB; fi
    envs=$(echo "$env" | tr ',' ' ')
    env $envs timeout -k 10 200 python bench.py --mode filter --steps 50 --warmup 10 --no-pcie --no-cpu-baseline > gpurun_out/c3v_${name}_r$r.json 2>gpurun_out/c3v_${name}_r$r.err || { tail -20 gpurun_out/c3v_${name}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/c3v_${name}_r$r.json')); print(f\"r$r ${name}: step {d['ms_per_step']:.4f} ms, device {d['roofline']['avg_kernel_ms']:.4f} ms, n_out {d['config']['n_out']}\")"
  done
done
