"""Census of the remaining libm differences (DESIGN.md §3 residual risks): device ocml vs glibc
double atan2 / acos / sin.  Candidate poses generated on the GPU and by the oracle compared bit
for bit (pitch, yaw come from atan2), and pose totals (sums of sin(pi/2 - acos(..)) + 1/L)
scored on the GPU and by the oracle over the same poses: how many differ in their bits, and by
how much.  Prints one JSON line.

    python tools/ulp_census.py [num_candidates ...]
"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
import pyoracle as O  # noqa: E402

from pointcloud_processor_amd import _abi, synth  # noqa: E402

O.lib()
O.set_threads(16)
sc = synth.terrain_scene()
cells = synth.excavation_cells(sc.area)
aux = synth.aux_cloud()
T, A = O.Cloud(sc.terrain), O.Cloud(aux)
out = []
with _abi.Context(0) as g:
    g.set_terrain(sc.terrain, point_step=32)
    g.set_aux_cloud(aux, point_step=32)
    g.set_cells(cells.xyz, cells.normals)
    for nc in [int(a) for a in sys.argv[1:]] or [100, 400, 1600]:
        params = _abi.default_vl_params(num_candidates=nc)
        pg = g.generate_candidates(cells.grid_bbox, params, sc.zx120_pose5)
        po = O.generate_candidates(T, cells.grid_bbox, O.vl_params(num_candidates=nc), sc.zx120_pose5)
        same_n = pg.shape == po.shape
        pose_bits = int((pg.view(np.uint64) != po.view(np.uint64)).sum()) if same_n else None
        pose_max = float(np.max(np.abs(pg - po))) if same_n and pg.size else 0.0
        fg = np.zeros(cells.xyz.shape[0], np.uint8)
        fo = fg.copy()
        tot, cov, rep = g.score_poses(pg, sc.zx120_pose5, params, fg)
        r_tot, r_cov, r_rep = O.score_poses(T, A, cells.xyz, cells.normals, pg, sc.zx120_pose5,
                                            O.vl_params(num_candidates=nc), fo)
        diff = tot.view(np.uint64) != r_tot.view(np.uint64)
        rel = np.abs(tot - r_tot) / np.maximum(1.0, np.abs(r_tot))
        out.append({"num_candidates": nc, "poses": int(pg.shape[0]), "poses_same_count": same_n,
                    "pose_values_differing_bits": pose_bits, "pose_max_abs_diff": pose_max,
                    "totals_differing_bits": int(diff.sum()), "totals_max_rel_diff": float(rel.max()),
                    "flags_equal": bool(np.array_equal(fg, fo)), "covered_equal": bool(np.array_equal(cov, r_cov)),
                    "best_equal": int(rep.best_idx) == int(r_rep.best_idx)})
print(json.dumps({"ulp_census": out}))
