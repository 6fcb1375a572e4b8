#!/bin/bash
# A/B of k_nb_lists' LDS footprint (build knobs PCP_NB_LDS / PCP_NB_BUCKETS: more blocks per CU
# for shorter LDS lists, longer lists through the global-memory path): bench C1 per library
# (PCP_LIB), interleaved, then the exact-normals parity tests on each variant.
#   libraries: pointcloud_processor_amd/_lib (default 4096 / 2048), _lib_nbA (2048 / 2048),
#   _lib_nbB (1024 / 1024)
# build the variants on the CPU first (from pointcloud_processor_amd/csrc):
#   make -j8 OUTDIR=../_lib_nbA EXTRA="-DPCP_NB_LDS=2048" ../_lib_nbA/libpcp.so
#   make -j8 OUTDIR=../_lib_nbB EXTRA="-DPCP_NB_LDS=1024 -DPCP_NB_BUCKETS=1024" ../_lib_nbB/libpcp.so
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for r in 1 2; do
  for v in _lib _lib_nbA _lib_nbB; do
    PCP_LIB=pointcloud_processor_amd/$v/libpcp.so timeout -k 10 300 python3 bench.py --mode c1 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/nblds_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/nblds_$v.log; exit 1; }
    echo "round $r $v: $(grep '^{' gpurun_out/nblds_$v.log | tail -1 | cut -c1-400)"
  done
done
for v in _lib_nbA _lib_nbB; do
  PCP_LIB=pointcloud_processor_amd/$v/libpcp.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "excavation_area" > gpurun_out/nblds_tests_$v.log 2>&1
  rc=$?; echo "tests $v: $(tail -1 gpurun_out/nblds_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
