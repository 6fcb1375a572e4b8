#!/bin/bash
# C3 restructure check on one GPU: filter-chain parity tests, then the committed build (alt_head)
# against the working tree's on the C3 frame, alternating processes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
  -k "crop or voxel or filter_merge or transform" > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -5 gpurun_out/c3_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_filter.sh 2>&1 | grep -v amdgpu.ids
