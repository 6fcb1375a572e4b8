"""Diagnostic: how many of the fan's scanned stencils end in a hit (C2 workload).

Prints blocked rays (= scans that found a point), the scan / point-test counters of the
stats kernel, and the first-hit sample histogram."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402  (load torch's HIP runtime first, as bench.py does)

from pointcloud_processor_amd import _abi, synth  # noqa: E402

ctx = _abi.Context(0)
sc = synth.terrain_scene()
ctx.set_terrain(sc.terrain, point_step=32)
p = sc.area[:, :3].astype(np.float64)
bb = np.array([p[:, 0].min() - .1, p[:, 0].max() + .1, p[:, 1].min() - .1, p[:, 1].max() + .1,
               p[:, 2].min() - .1, p[:, 2].max() + .1])
poses = ctx.generate_candidates(bb, _abi.default_vl_params(num_candidates=348), sc.zx120_pose5)[:256]
fan = _abi.fan_params()
for _ in range(2):
    blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
print("rays", fh.size, "blocked", int(blocked.sum()), "units", int(units.sum()))
if hasattr(ctx, "raycast_fan_stats"):
    print("stats", ctx.raycast_fan_stats(poses, fan))
h = np.bincount(fh[fh >= 0].ravel(), minlength=49)
print("first-hit sample histogram", h.tolist())
