"""Diagnostic: wave-lifetime breakdown of the fan kernel from s_memtime stamps."""
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
for _ in range(3):
    ctx.raycast_fan(poses, fan)
st = ctx.raycast_fan_stamps(poses, fan).astype(np.int64)
setup, march, tail = st[..., 1] - st[..., 0], st[..., 2] - st[..., 1], st[..., 3] - st[..., 2]
life = st[..., 3] - st[..., 0]
span = st[..., 3].max() - st[..., 0].min()
print(f"kernel span {span} clk; waves {life.size}")
for name, v in (("setup", setup), ("march", march), ("tail", tail), ("life", life)):
    print(f"{name:6s} mean {v.mean():10.0f} p50 {np.median(v):10.0f} p99 {np.percentile(v, 99):10.0f} max {v.max():10.0f}")
# concurrency: average live waves = sum(life) / span
print("avg live waves", life.sum() / span)
el = np.arange(life.shape[1]) // (fan.n_az // 64)
prof = np.array([life[:, el == j].mean() for j in range(fan.n_el)])
print("life by elevation ring (every 16th):", prof[::16].astype(int).tolist())
st0 = st[..., 0] - st[..., 0].min()
print("start-time quantiles:", np.percentile(st0, [0, 25, 50, 75, 100]).astype(int).tolist())
