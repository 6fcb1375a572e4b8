#!/bin/bash
# round 6: k_nb_lists' sorted lists assembled in LDS and stored as one coalesced run (default
# build) vs m scattered 4-byte stores (PCP_NB_STAGE_OUT=0, _lib/alt_nbold) -- normals parity,
# then the C5 replay and C1 alternating, then the kernel's own time per build (rocprof stats)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
L=pointcloud_processor_amd/_lib
ALT=$L/alt_nbold
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_nodes_cli.py -m gpu \
  -k "excavation_area or streaming_replay or generate_and_score or c1" > gpurun_out/r6_nbstage_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r6_nbstage_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r6_nbstage_tests.log | head -10; exit $rc; }
bash tools/replay.sh > /dev/null 2>&1 || exit 1
read TN CN BB < gpurun_out/replay/args
for r in 1 2 3; do
  for d in $L $ALT; do
    LD_LIBRARY_PATH=$d timeout -k 10 300 $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 \
      gpurun_out/replay/n.f32 $CN $BB 200 60032 1 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('c5 r$r $d p50 %.4f p99 %.4f' % (d['p50_ms'], d['p99_ms']), 'area', d['stage_p50_ms'].get('area'))" || exit 1
  done
done
for r in 1 2; do
  for d in $L/libpcp.so $ALT/libpcp.so; do
    PCP_LIB=$d timeout -k 10 200 python bench.py --mode c1 --steps 200 --warmup 10 --no-cpu-baseline 2>/dev/null | grep '^{' | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d.get('c1', d)
print('c1 r$r', '$d'.split('/')[-2], 'p50 %.4f p99 %.4f' % (c['value'], c['p99_ms']))" || exit 1
  done
done
for d in $L $ALT; do
  n=$(basename $d)
  LD_LIBRARY_PATH=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nbst_$n -o run --output-format csv -- \
    $L/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB 100 60032 1 > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/nbst_$n -name "run_kernel_stats.csv" | head -n 1)
  echo "== $n"; grep -E "k_nb_lists|k_nb_sums" "$f" | cut -d, -f1-4
done
