"""A/B of fan-kernel variants in ONE process, interleaved rounds (guide rule 24)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402

from pointcloud_processor_amd import _abi, synth  # noqa: E402

variants = [int(v) for v in (sys.argv[1:] or ["0", "1", "2"])]
sc = synth.terrain_scene()
p = sc.area[:, :3].astype(np.float64)
bb = np.array([p[:, 0].min() - .1, p[:, 0].max() + .1, p[:, 1].min() - .1, p[:, 1].max() + .1,
               p[:, 2].min() - .1, p[:, 2].max() + .1])
ctxs = {}
for v in variants:
    os.environ["PCP_FAN_BATCH"] = str(v)
    c = _abi.Context(0)
    c.set_terrain(sc.terrain, point_step=32)
    ctxs[v] = c
poses = ctxs[variants[0]].generate_candidates(bb, _abi.default_vl_params(num_candidates=348),
                                              sc.zx120_pose5)[:256]
fan = _abi.fan_params()
ref = None
times = {v: [] for v in variants}
for rnd in range(12):
    for v in variants:
        c = ctxs[v]
        c.profile(True)
        c.profile_reset()
        b, u, _, _ = c.raycast_fan(poses, fan)
        ms, n = c.profile_get("raycast_fan")
        if rnd >= 2:
            times[v].append(ms / n)
        if ref is None:
            ref = (b, u)
        if v < 90:      # >= 90: timing experiments that skip work (results differ)
            assert np.array_equal(b, ref[0]) and np.array_equal(u, ref[1]), v
for v in variants:
    t = np.array(times[v])
    print(f"batch={v}: median {np.median(t):.4f} ms  min {t.min():.4f} ms")
for v in variants:
    print("stats", v, ctxs[v].raycast_fan_stats(poses, fan))
