set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "filter_merge or crop_voxel or voxel_grid or crop_" > gpurun_out/r6_c3a_tests.log 2>&1 || { tail -60 gpurun_out/r6_c3a_tests.log; exit 1; }
tail -2 gpurun_out/r6_c3a_tests.log
bash tools/ab_filter.sh 2>&1 | tee gpurun_out/r6_c3a_ab.log
