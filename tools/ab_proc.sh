#!/bin/bash
# A/B with ONE variant per process (large terrain copies in one process evict each other from
# the Infinity Cache between interleaved launches): rounds of alternating processes.
#   bash tools/ab_proc.sh "name:ENV=V,ENV=V[:lib]" ...   (lib = path of another libpcp.so)
set -u
cd "$(dirname "$0")/.."
for r in 1 2; do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; env=${rest%%:*}; lib=""
    [ "$rest" != "$env" ] && lib=${rest#*:}
    if [ -n "$lib" ]; then export PCP_LIB=$lib; else unset PCP_LIB; fi
    out=$(timeout -k 10 200 python tools/fan_ab.py "$name:$env" 2>&1 | grep -v amdgpu.ids) || { echo "$out"; exit 1; }
    echo "r$r $(echo "$out" | head -1)   $(echo "$out" | grep stats | cut -c1-200)"
  done
done
