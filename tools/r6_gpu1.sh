#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "allreduce or own_communicator" > gpurun_out/r6_comm_tests.log 2>&1 || { tail -60 gpurun_out/r6_comm_tests.log; exit 1; }
tail -4 gpurun_out/r6_comm_tests.log
bash tools/r6_c3c.sh
