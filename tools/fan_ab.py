"""A/B of fan-kernel variants in ONE process, interleaved rounds (guide rule 24).

    python tools/fan_ab.py [VARIANT ...]

A variant is a name with optional context environment, e.g. `base:PCP_TERRAIN_FINE=0`
`fine:PCP_TERRAIN_FINE=1` `fine7:PCP_TERRAIN_FINE=1,PCP_FAN_BATCH=3`; a bare integer N is the
old form PCP_FAN_BATCH=N.  Every variant must give the same blocked counts and ray-hit tests
(names starting with `x` are timing experiments whose results may differ).
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402

from pointcloud_processor_amd import _abi, synth  # noqa: E402


def parse(v):
    if v.isdigit():
        return f"batch{v}", {"PCP_FAN_BATCH": v}
    name, _, env = v.partition(":")
    return name, dict(kv.split("=", 1) for kv in env.split(",") if kv)


variants = [parse(v) for v in (sys.argv[1:] or ["0", "1", "2"])]
sc = synth.terrain_scene()
p = sc.area[:, :3].astype(np.float64)
bb = np.array([p[:, 0].min() - .1, p[:, 0].max() + .1, p[:, 1].min() - .1, p[:, 1].max() + .1,
               p[:, 2].min() - .1, p[:, 2].max() + .1])
ctxs = {}
for name, env in variants:
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    c = _abi.Context(0)
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
    c.set_terrain(sc.terrain, point_step=32)
    ctxs[name] = c
names = [n for n, _ in variants]
poses = ctxs[names[0]].generate_candidates(bb, _abi.default_vl_params(num_candidates=348),
                                           sc.zx120_pose5)[:256]
fan = _abi.fan_params()
ref = None
times = {v: [] for v in names}
for rnd in range(12):
    for v in names:
        c = ctxs[v]
        c.profile(True)
        c.profile_reset()
        b, u, _, _ = c.raycast_fan(poses, fan)
        ms, n = c.profile_get("raycast_fan")
        if rnd >= 2:
            times[v].append(ms / n)
        if ref is None:
            ref = (b, u)
        if not v.startswith("x"):
            assert np.array_equal(b, ref[0]) and np.array_equal(u, ref[1]), v
# across processes (tools/ab_proc.sh): the first run of a box leaves its outputs, every later
# variant must reproduce them
reff = ROOT / "gpurun_out" / "fan_ab_ref.npz"
if reff.exists():
    z = np.load(reff)
    assert np.array_equal(z["b"], ref[0]) and np.array_equal(z["u"], ref[1]), "differs from " + str(reff)
else:
    reff.parent.mkdir(exist_ok=True)
    np.savez(reff, b=ref[0], u=ref[1])
for v in names:
    t = np.array(times[v])
    print(f"{v}: median {np.median(t):.4f} ms  min {t.min():.4f} ms")
for v in names:
    print("stats", v, ctxs[v].raycast_fan_stats(poses, fan))
