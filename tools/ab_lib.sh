#!/bin/bash
# A/B of the committed build (alt_head) against the working tree's build on one box, two
# alternating rounds: bash tools/ab_lib.sh "VARIANTS for alt_head" "VARIANTS for the new build"
set -u
cd "$(dirname "$0")/.."
OLD=${1:-fine:PCP_FAN_BATCH=0}
NEW=${2:-fine:PCP_FAN_BATCH=0}
for r in 1 2; do
  echo "== alt_head round $r"
  PCP_LIB=pointcloud_processor_amd/_lib/alt_head/libpcp.so timeout -k 10 200 python tools/fan_ab.py $OLD 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== new round $r"
  timeout -k 10 300 python tools/fan_ab.py $NEW 2>&1 | grep -v amdgpu.ids || exit 1
done
