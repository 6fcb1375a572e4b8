#!/bin/bash
# round 6: the staggered two-stream C3 frame -- filter parity tests (default, and with every
# two-cloud frame staggered), then the frame A/B against alt_head (alternating processes)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
K="filter_merge or crop_voxel or voxel_grid or crop_"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "$K" > gpurun_out/r6_c3b_tests.log 2>&1 || { tail -60 gpurun_out/r6_c3b_tests.log; exit 1; }
tail -2 gpurun_out/r6_c3b_tests.log
PCP_BK_STAGGER=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "$K" > gpurun_out/r6_c3b_tests_s1.log 2>&1 || { tail -60 gpurun_out/r6_c3b_tests_s1.log; exit 1; }
tail -2 gpurun_out/r6_c3b_tests_s1.log
bash tools/ab_filter.sh 2>&1 | tee gpurun_out/r6_c3b_ab.log
