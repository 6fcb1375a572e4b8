#!/bin/bash
# C5 streaming replay through the C++ node cores (pcp_nodes_cli replay): fixed-terrain mode
# and the full per-frame chain (filter x2 -> merge -> carve -> virtual_lidar setup + search)
set -eu
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/replay
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
CLI=${CLI:-pointcloud_processor_amd/_lib/pcp_nodes_cli}
for chain in 0 1; do
  timeout -k 10 300 $CLI replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB ${FRAMES:-50} 60032 $chain
done
