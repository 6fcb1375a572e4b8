"""Diagnostic: fixed per-query cost of pcp_raycast_fan (host + launch + readback) from a tiny
fan, against the C2 query, and the Python wrapper's share (ctypes call timed alone)."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402

from pointcloud_processor_amd import _abi, synth  # noqa: E402

ctx = _abi.Context(0)
sc = synth.terrain_scene()
ctx.set_terrain(sc.terrain, point_step=32)
p = sc.area[:, :3].astype(np.float64)
bb = np.array([p[:, 0].min() - .1, p[:, 0].max() + .1, p[:, 1].min() - .1, p[:, 1].max() + .1,
               p[:, 2].min() - .1, p[:, 2].max() + .1])
poses = ctx.generate_candidates(bb, _abi.default_vl_params(num_candidates=348), sc.zx120_pose5)[:256]
poses = np.ascontiguousarray(poses)
for name, fan in (("tiny 64x1", _abi.fan_params(n_az=64, n_el=1)), ("C2 1024x256", _abi.fan_params())):
    for _ in range(5):
        ctx.raycast_fan(poses, fan)
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.raycast_fan(poses, fan)
    py = (time.perf_counter() - t0) / n * 1e3
    blocked = np.zeros(256, np.uint32)
    units = np.zeros(256, np.uint64)
    best = C.c_int64()
    pp = poses.ctypes.data_as(C.c_void_p)
    bp, up = blocked.ctypes.data_as(C.c_void_p), units.ctypes.data_as(C.c_void_p)
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.lib.pcp_raycast_fan(ctx.h, pp, 256, C.byref(fan), bp, up, None, C.byref(best))
    raw = (time.perf_counter() - t0) / n * 1e3
    print(f"{name}: wrapper {py:.4f} ms/query, raw ctypes {raw:.4f} ms/query")
