#!/bin/bash
# C5 tail study: the full-chain replay, 1000 frames, without and with the process pinned to a
# few cores of the box's share (the host-side stages are what inflate on the slow frames)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
FRAMES=2 timeout -k 10 300 bash tools/replay.sh > /dev/null 2>&1 || exit 1
read TN CN BB < gpurun_out/replay/args
run() {
  timeout -k 10 300 "$@" pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
    gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB 1000 60032 1
}
CPUS=$(python3 -c "import os; a=sorted(os.sched_getaffinity(0)); print(','.join(map(str,a[:4])))")
for r in 1 2; do
  run env > gpurun_out/tail_free_$r.json || exit 1
  run taskset -c $CPUS > gpurun_out/tail_pin_$r.json || exit 1
done
python3 - <<'PY'
import json, numpy as np
for r in (1, 2):
    for k in ("free", "pin"):
        d = json.loads(open(f"gpurun_out/tail_{k}_{r}.json").read().strip().splitlines()[-1])
        a = np.array(d["lat_ms"])
        print(f"round {r} {k:4s}: p50 {np.percentile(a,50):.3f} p90 {np.percentile(a,90):.3f} p99 {np.percentile(a,99):.3f} max {a.max():.3f} ms; >1.1 ms: {(a > 1.1).sum()} of {a.size}")
PY
