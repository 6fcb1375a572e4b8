#!/bin/bash
# C3 bucket-chain A/B (PCP_FM_FAST 2 = bucket chain vs 1 = LSD fast chain, alternating
# processes) after the filter parity tests, then the bucket chain's kernel stats.  Outputs under
# gpurun_out/.  TESTS=0 skips the tests, PROF=0 the rocprofv3 pass.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "filter_merge or crop_voxel or voxel_grid or crop_" > gpurun_out/bk_tests.log 2>&1 || { tail -60 gpurun_out/bk_tests.log; exit 1; }
  tail -2 gpurun_out/bk_tests.log
fi
for r in 1 2; do for f in 2 1; do
  PCP_FM_FAST=$f timeout -k 10 300 python bench.py --mode filter --steps 50 --warmup 10 --no-pcie --no-cpu-baseline > gpurun_out/c3_r${r}_m$f.json 2>gpurun_out/c3_r${r}_m$f.err || { tail -20 gpurun_out/c3_r${r}_m$f.err; exit 1; }
done; done
python3 - <<'PY'
import json
for r in (1, 2):
    for f in (2, 1):
        d = json.load(open(f"gpurun_out/c3_r{r}_m{f}.json"))
        print(f"round {r} PCP_FM_FAST={f}: step {d['ms_per_step']:.4f} ms, device {d['roofline']['avg_kernel_ms']:.4f} ms, n_out {d['config']['n_out']}")
PY
if [ "${PROF:-1}" = 1 ]; then
  PCP_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3bk -o c3bk --output-format csv -- python3 bench.py --mode filter --steps 20 --warmup 5 --no-pcie --no-cpu-baseline > gpurun_out/c3bk_prof.log 2>&1 || exit 1
  find gpurun_out/c3bk -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
fi
