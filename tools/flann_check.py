#!/usr/bin/env python3
"""Pin the grid-based radius predicate (oracle and GPU) against the restated KdTreeFLANN
(oracle/pcp_flann.c: FLANN 1.9.1 KDTreeSingleIndex, PCL 1.12.1 configuration) over the whole
C2 workload and the reference-mode node tick -> profiles/r02_flann_check.json.

  * fan: all 256 bench poses x the 1024 x 256 fan on the T1M terrain; every sample query the
    reference executes is answered by the tree (the reference's predicate) and compared with
    the exact grid count; first hits, blocked counts and ray-hit tests compared with the grid
    oracle (orc_raycast_fan), which the GPU matches bit for bit (tests/test_gpu_parity.py).
  * reference mode: runOptimization over the 3,704 excavation cells for the same 256 poses,
    the oracle in FLANN mode (march, relaxed zx120 check) vs grid mode: totals, covered counts,
    stale flags, colour report.
  * candidates: generateCandidatePositions with getGroundHeight through the tree's neighbour
    list vs the grid scan.
  * boundary stress: queries at float distance r(1 +- 4e-7) of terrain points for r = 0.056,
    0.24 and 2.0, tree count vs grid count.

    python tools/flann_check.py [--threads 8] [--poses 256]
"""
import argparse
import json
import math
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import pyoracle as O  # noqa: E402

from pointcloud_processor_amd import synth  # noqa: E402


def _poses(G, bbox, zx, total):
    nc = max(total, 100)
    while True:
        p = O.generate_candidates(G, bbox, O.vl_params(num_candidates=nc), zx)
        if p.shape[0] >= total:
            return p[:total], nc
        nc = int(nc * 1.3) + 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--poses", type=int, default=256)
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r02_flann_check.json"))
    args = ap.parse_args()
    O.set_threads(args.threads)
    sc = synth.terrain_scene()
    res = {"terrain_points": int(sc.terrain.shape[0]), "threads": args.threads,
           "flann": "FLANN 1.9.1 KDTreeSingleIndex (leaf 15, eps 0, unlimited checks) as PCL "
                    "1.12.1 KdTreeFLANN builds it, restated in oracle/pcp_flann.c"}
    t0 = time.time()
    tree = O.KdTree(sc.terrain)
    G = O.Cloud(sc.terrain)
    res["tree_build_s"] = time.time() - t0

    # ---- boundary stress
    rng = np.random.default_rng(20260227)
    pts = sc.terrain[:, :3]
    stress = {}
    for r, nq in ((0.056, 6_000_000), (0.24, 2_000_000), (2.0, 200_000)):
        sel = rng.integers(0, pts.shape[0], nq)
        u = rng.normal(size=(nq, 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        d = r * (1.0 + rng.uniform(-4e-7, 4e-7, nq))
        q = (pts[sel].astype(np.float64) + u * d[:, None]).astype(np.float32)
        stress[str(r)] = tree.check_queries(G, q, r)
        print("stress", r, stress[str(r)], flush=True)
    res["boundary_stress"] = stress

    # ---- C2 fan, every sample query through the tree
    import bench

    poses, nc = _poses(G, bench._grid_bbox(sc.area), sc.zx120_pose5, args.poses)
    el = math.radians(85.0)
    t0 = time.time()
    tot = {"queries": 0, "count_mismatch": 0, "any_mismatch": 0, "neighbours": 0}
    fh_bad = blk_bad = unit_bad = 0
    for k0 in range(0, poses.shape[0], 16):
        sel = poses[k0:k0 + 16]
        b, u, fh, st = O.raycast_fan_kd(tree, G, sel, 1024, 256, -el, el, 15.0)
        rb, ru, rfh = O.raycast_fan(G, sel, 1024, 256, -el, el, 15.0)
        for k in tot:
            tot[k] += st[k]
        fh_bad += int(np.count_nonzero(fh != rfh))
        blk_bad += int(np.count_nonzero(b != rb))
        unit_bad += int(np.count_nonzero(u != ru))
        print("fan", k0 + sel.shape[0], tot, fh_bad, flush=True)
    res["fan"] = {"poses": int(poses.shape[0]), "fan": [1024, 256],
                  "num_candidates_lattice": nc, "sample_queries": tot,
                  "first_hit_mismatch": fh_bad, "blocked_mismatch": blk_bad,
                  "units_mismatch": unit_bad, "seconds": time.time() - t0}

    # ---- candidates with getGroundHeight through the tree
    Gf = O.Cloud(sc.terrain, flann=True)
    cells = synth.excavation_cells(sc.area)
    pf, _ = _poses(Gf, cells.grid_bbox, sc.zx120_pose5, args.poses)
    pg, _ = _poses(G, cells.grid_bbox, sc.zx120_pose5, args.poses)
    res["candidates"] = {"poses": int(pg.shape[0]), "identical": bool(np.array_equal(pf, pg))}

    # ---- reference mode: the oracle in FLANN mode vs grid mode
    aux = synth.aux_cloud()
    A, Af = O.Cloud(aux), O.Cloud(aux, flann=True)
    t0 = time.time()
    fg = np.zeros(cells.xyz.shape[0], np.uint8)
    ff = fg.copy()
    prm = O.vl_params()
    tg, cg, rg = O.score_poses(G, A, cells.xyz, cells.normals, pg, sc.zx120_pose5, prm, fg)
    tf, cf, rf = O.score_poses(Gf, Af, cells.xyz, cells.normals, pg, sc.zx120_pose5, prm, ff)
    res["reference_mode"] = {
        "poses": int(pg.shape[0]), "cells": int(cells.xyz.shape[0]),
        "totals_identical": bool(np.array_equal(tg, tf)),
        "covered_identical": bool(np.array_equal(cg, cf)),
        "flags_identical": bool(np.array_equal(fg, ff)),
        "report_identical": rg.as_dict() == rf.as_dict(), "best_idx": int(rf.best_idx),
        "seconds": time.time() - t0}
    ok = (all(v["count_mismatch"] == 0 and v["any_mismatch"] == 0 for v in stress.values())
          and tot["count_mismatch"] == 0 and fh_bad == 0 and blk_bad == 0 and unit_bad == 0
          and res["candidates"]["identical"]
          and all(res["reference_mode"][k] for k in ("totals_identical", "covered_identical",
                                                     "flags_identical", "report_identical")))
    res["all_identical"] = ok
    Path(args.out).write_text(json.dumps(res, indent=2) + "\n")
    print(json.dumps(res, indent=2))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
