#!/bin/bash
# C5 full chain under a runtime + kernel + copy trace (no counters): per-frame syncs, copies
# and gaps.  Output: gpurun_out/c5tl/
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/replay gpurun_out/c5tl
python3 - <<'PY'
import sys
sys.path.insert(0, ".")
import numpy as np
from pointcloud_processor_amd import synth
sc = synth.terrain_scene()
cells = synth.excavation_cells(sc.area)
np.ascontiguousarray(sc.terrain).tofile("gpurun_out/replay/t.f32")
np.ascontiguousarray(cells.xyz).tofile("gpurun_out/replay/c.f64")
np.ascontiguousarray(cells.normals).tofile("gpurun_out/replay/n.f32")
open("gpurun_out/replay/args", "w").write(
    f"{sc.terrain.shape[0]} {cells.xyz.shape[0]} " + ",".join(repr(float(v)) for v in cells.grid_bbox) + "\n")
PY
read TN CN BB < gpurun_out/replay/args
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
  -d gpurun_out/c5tl -o c5 -- pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN \
  gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-30} 60032 1 > gpurun_out/c5tl/run.log 2>&1
ls gpurun_out/c5tl
