#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the CPU restatement (oracle/).

The reference ships no tests, fixtures or golden data and cannot be built here (SURVEY.md
§4, §8c), so these vectors are produced by the restatement and pin it against regressions;
tests/test_oracle.py cross-checks the restatement with independent numpy/scipy code.
Inputs are stored in the fixtures, so the GPU parity tests consume exactly these bytes.

    python tests/golden/make_golden.py
"""
import math
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

import pyoracle as O  # noqa: E402

SEED = 20260227
BOX = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])


def mini_terrain(seed=SEED):
    """5 m x 5 m lattice at 0.05 m with a 1 m x 0.6 m, 0.5 m deep box pit and a wall."""
    rng = np.random.default_rng(seed)
    xs = 2.0 + 0.05 * np.arange(100)
    ys = -2.5 + 0.05 * np.arange(100)
    X, Y = np.meshgrid(xs, ys)
    Z = rng.normal(0, 0.01, X.shape)
    pit = (X > 3.5) & (X < 4.5) & (Y > -0.3) & (Y < 0.3)
    Z[pit] -= 0.5
    pts = [np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1)]
    # a 1.2 m high wall segment that occludes some rays
    wz = np.arange(0.05, 1.2, 0.05)
    wy = np.arange(-1.0, 1.0, 0.05)
    WY, WZ = np.meshgrid(wy, wz)
    pts.append(np.stack([np.full(WY.size, 5.5), WY.ravel(), WZ.ravel()], 1))
    xyz = np.concatenate(pts).astype(np.float32)
    out = np.zeros((xyz.shape[0], 8), np.float32)
    out[:, :3] = xyz
    out[:, 3] = 1.0
    return out


def main():
    rng = np.random.default_rng(SEED)
    # ---- crop (pointcloud_filter.cpp:106-116) incl. NaN and exact boundary values
    n = 1500
    c = np.zeros((n, 4), np.float32)
    c[:, 0] = rng.uniform(-3, 18, n)
    c[:, 1] = rng.uniform(-12, 12, n)
    c[:, 2] = rng.uniform(-3, 12, n)
    c[:10, 0] = 0.0
    c[10:20, 0] = 15.0
    c[20:30, 1] = 10.0
    c[30:40, 2] = -1.5
    c[40:45, 1] = np.nan
    kept = O.crop_box(c, BOX)
    np.savez_compressed(HERE / "crop.npz", cloud=c, box=BOX, kept=kept)

    # ---- voxel (pcl::VoxelGrid, leaf 0.2) on the cropped cloud
    vin = c[kept]
    vx, vidx, vcnt, vpt = O.voxel_grid(vin, 0.2)
    # dense clusters so voxels hold several points
    d = np.repeat(rng.uniform(0, 5, (300, 3)).astype(np.float32), 6, 0)
    d += rng.normal(0, 0.03, d.shape).astype(np.float32)
    dd = np.zeros((d.shape[0], 4), np.float32)
    dd[:, :3] = d
    dx, didx, dcnt, _ = O.voxel_grid(dd, 0.1)
    np.savez_compressed(HERE / "voxel.npz", cloud_a=vin, leaf_a=np.float32(0.2), xyz_a=vx,
                        idx_a=vidx, cnt_a=vcnt, cloud_b=dd, leaf_b=np.float32(0.1), xyz_b=dx,
                        idx_b=didx, cnt_b=dcnt)

    # ---- transform + colour (tf2::doTransform, pointcloud_merger.cpp:370-387)
    yaw = math.radians(30.0)
    t = np.array([8.0, -3.0, 0.0])
    q = np.array([0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2)])
    tr = O.transform_rgb(vin[:500], t, q, (255, 0, 0))
    np.savez_compressed(HERE / "transform.npz", cloud=vin[:500], t=t, q=q,
                        rgb=np.array([255, 0, 0], np.uint8), out=tr)

    # ---- fan raycast + candidate poses on the mini terrain
    terr = mini_terrain()
    T = O.Cloud(terr)
    poses = np.array([[1.0, 0.0, 1.1, -0.4, 0.0], [4.0, -2.0, 0.9, -0.6, 1.2],
                      [7.0, 1.5, 1.6, -0.3, -2.7]])
    el_min, el_max = -85.0 * math.pi / 180.0, 85.0 * math.pi / 180.0
    blocked, units, fh = O.raycast_fan(T, poses, 64, 32, el_min, el_max, 15.0)
    np.savez_compressed(HERE / "fan.npz", terrain=terr, poses=poses, n_az=64, n_el=32,
                        el_min=el_min, el_max=el_max, max_distance=15.0, first_hit=fh,
                        blocked=blocked, units=units)

    # ---- cell scoring (runOptimization :460-519) on a small cell lattice over the pit
    cx, cy, cz = np.meshgrid(np.arange(3.4, 4.61, 0.2), np.arange(-0.4, 0.41, 0.2),
                             np.array([-0.45, -0.25, 0.05]), indexing="ij")
    cells = np.stack([cx.ravel(), cy.ravel(), cz.ravel()], 1)
    nrm = np.tile(np.array([0.0, 0.0, 1.0], np.float32), (cells.shape[0], 1))
    nrm[::3] = np.array([0.6, 0.0, 0.8], np.float32)
    aux = terr[::37].copy()
    A = O.Cloud(aux)
    params = O.vl_params(max_distance=12.0)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    bb = np.array([3.3, 4.7, -0.5, 0.5, -0.6, 0.15])
    cand = O.generate_candidates(T, bb, O.vl_params(num_candidates=36), zx)
    flags = np.zeros(cells.shape[0], np.uint8)
    tot, cov, rep = O.score_poses(T, A, cells, nrm, cand, zx, params, flags)
    np.savez_compressed(HERE / "score.npz", terrain=terr, aux=aux, cells=cells, normals=nrm,
                        zx=zx, grid_bbox=bb, num_candidates=36, max_distance=12.0,
                        candidates=cand, flags=flags, total=tot, covered=cov,
                        report=np.array([rep.best_idx, rep.total_cells, rep.green, rep.red,
                                         rep.blue, rep.yellow, rep.zx120_green, rep.zx120_red,
                                         rep.zx120_blue, rep.zx120_yellow], np.int64),
                        best_score=rep.best_score, zx120_total=rep.zx120_total_score)
    # ---- excavation-area setup (computeTerrainNormals + generateExcavationGrid3D, :164-340)
    from pointcloud_processor_amd import synth

    area = np.ascontiguousarray(synth.terrain_scene(n_side=200, x0=-2.0, y0=-4.0).area[::3, :4])
    anrm = O.area_normals(area, 1.5)
    cxyz, cn, gbb, dims = O.excavation_grid(area, 0.1, 10, anrm)
    np.savez_compressed(HERE / "excavation.npz", area=area, normals=anrm, cells=cxyz,
                        cell_normals=cn, grid_bbox=gbb, dims=np.array(dims, np.int32))
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)


if __name__ == "__main__":
    main()
