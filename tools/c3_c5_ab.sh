#!/bin/bash
# C3 fast-chain A/B (PCP_FM_FAST 1 vs 0, alternating processes) + its parity tests, then the
# C5 replay and its runtime trace.  Outputs under gpurun_out/.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_nodes_cli.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for r in 1 2; do for f in 1 0; do
  PCP_FM_FAST=$f timeout -k 10 300 python bench.py --mode filter --steps 50 --warmup 10 --no-pcie --no-cpu-baseline > gpurun_out/c3_r${r}_fast$f.json 2>/dev/null || exit 1
done; done
python3 - <<'PY'
import json
for r in (1, 2):
    for f in (1, 0):
        d = json.load(open(f"gpurun_out/c3_r{r}_fast{f}.json"))
        print(f"round {r} PCP_FM_FAST={f}: step {d['ms_per_step']:.4f} ms, device {d['roofline']['avg_kernel_ms']:.4f} ms, n_out {d['config']['n_out']}")
PY
PCP_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o c3 --output-format csv -- python3 bench.py --mode filter --steps 20 --warmup 5 --no-pcie --no-cpu-baseline > gpurun_out/c3prof.log 2>&1 || exit 1
FRAMES=200 timeout -k 10 600 bash tools/replay.sh > gpurun_out/replay.log 2>&1 || exit 1
FRAMES=30 timeout -k 10 400 bash tools/replay_trace.sh > gpurun_out/trace.log 2>&1 || exit 1
python3 tools/c5_timeline.py gpurun_out/c5tl > gpurun_out/c5_timeline.txt
grep -o '"chain": [01], "p50_ms": [0-9.]*, "p99_ms": [0-9.]*' gpurun_out/replay.log
head -3 gpurun_out/c5_timeline.txt
