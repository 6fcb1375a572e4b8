"""Determinism stress: repeat the C3 frame (graph replays) and compare every output.
usage: python tools/filter_stress.py LIB [iters]"""
import math
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402

from pointcloud_processor_amd import _abi, synth  # noqa: E402

lp = sys.argv[1]
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
clouds = [synth.lidar_cloud(5_000_000, sensor_height=2.0, seed=1),
          synth.lidar_cloud(5_000_000, sensor_height=3.5, seed=2)]
box = [0.0, 15.0, -10.0, 10.0, -1.5, 10.0]
yaw = math.radians(30.0)
tfs = [((8.0, -3.0, 0.0), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))),
       ((0.55, 0.4, 3.5), (0.0, math.sin(0.4363 / 2), 0.0, math.cos(0.4363 / 2)))]
rgbs = [(255, 0, 0), (0, 0, 255)]
ctx = _abi.Context(0, lib_path=lp)
views = []
for c in clouds:
    p = ctx.dev_alloc(c.nbytes)
    ctx.h2d(p, c)
    views.append(_abi.CloudView(p, c.shape[0], 16, 0, 4, 8))
cap = sum(c.shape[0] for c in clouds)
out = ctx.dev_alloc(cap * 32)
ref = None
bad = 0
for it in range(iters):
    n, per = ctx.filter_merge_device(views, [box, box], 0.05, tfs, rgbs, out, cap)
    got = np.empty((n, 8), np.float32)
    ctx.d2h(got, out)
    g = got[:, :5].view(np.uint32)
    if ref is None:
        ref = g.copy()
        continue
    if g.shape != ref.shape or not np.array_equal(g, ref):
        nb = -1 if g.shape != ref.shape else int(np.count_nonzero((g != ref).any(1)))
        rows = [] if nb < 0 else np.nonzero((g != ref).any(1))[0][:5].tolist()
        print(f"iter {it}: shape {g.shape} vs {ref.shape}, rows differ {nb}, first {rows}",
              flush=True)
        bad += 1
print(f"{lp}: {bad} of {iters - 1} replays differ")
