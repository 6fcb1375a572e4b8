"""The second checker: FLANN 1.9.1 KDTreeSingleIndex as PCL 1.12.1 KdTreeFLANN runs it
(oracle/pcp_flann.c), against the exact grid scan that the oracle and the GPU both use.

The reference answers every radius query with KdTreeFLANN::radiusSearch
(virtual_lidar.cpp:782 in the ray march, :745 relaxed zx120 check, :611 getGroundHeight).
FLANN prunes subtrees with an incrementally updated float lower bound, so in principle it could
drop a point whose float distance is below r^2; the grid scan tests every point of the
candidate cells.  These tests check (1) the restated tree against numpy brute force, (2) the
tree against the grid on adversarial queries placed at distance ~r from points, where pruning
rounding would show, and (3) the whole oracle in FLANN mode against the committed golden
fixtures.  tools/flann_check.py runs the same comparison over the full C2 workload
(profiles/r02_flann_check.json).
"""
import math
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def _brute(pts, q, r):
    """L2_Simple<float>: ((0 + dx^2) + dy^2) + dz^2 < float(r*r), float arithmetic."""
    q = np.asarray(q, np.float32)
    d = pts[:, :3] - q
    acc = np.float32(0) + d[:, 0] * d[:, 0]
    acc = acc + d[:, 1] * d[:, 1]
    acc = acc + d[:, 2] * d[:, 2]
    return np.nonzero(acc < np.float32(r * r))[0]


def _clouds():
    rng = np.random.default_rng(3)
    uni = rng.uniform(-2, 2, (30_000, 3)).astype(np.float32)
    # a lattice (many exactly equal coordinates, ties on every split plane)
    g = np.arange(-20, 20) * 0.05
    X, Y = np.meshgrid(g, g)
    lat = np.stack([X.ravel(), Y.ravel(), np.zeros(X.size)], 1).astype(np.float32)
    # duplicates and a degenerate column (identical x, y)
    dup = np.repeat(rng.uniform(-1, 1, (500, 3)), 7, 0).astype(np.float32)
    col = np.c_[np.zeros(2000), np.zeros(2000), rng.uniform(-1, 1, 2000)].astype(np.float32)
    return {"uniform": uni, "lattice": lat, "dup": dup, "column": col}


@pytest.mark.parametrize("name", ["uniform", "lattice", "dup", "column"])
def test_tree_matches_brute_force(oracle, name):
    pts = _clouds()[name]
    tree = oracle.KdTree(pts)
    assert tree.n == pts.shape[0]
    rng = np.random.default_rng(11)
    lo, hi = pts.min(0) - 0.2, pts.max(0) + 0.2
    for r in (0.056, 0.24, 1.0):
        for _ in range(150):
            q = rng.uniform(lo, hi).astype(np.float32)
            n, idx = tree.radius_search(q, r, want_idx=True)
            ref = _brute(pts, q, r)
            assert n == ref.size
            np.testing.assert_array_equal(idx, ref)


def test_tree_drops_nonfinite_points(oracle):
    pts = np.array([[0, 0, 0], [np.nan, 0, 0], [0.01, 0, 0], [0, np.inf, 0]], np.float32)
    tree = oracle.KdTree(pts)
    n, idx = tree.radius_search([0.0, 0.0, 0.0], 0.056, want_idx=True)
    assert n == 2 and idx.tolist() == [0, 2]    # indices of the caller's cloud


@pytest.mark.parametrize("r", [0.056, 0.24])
def test_tree_vs_grid_at_the_radius(oracle, scene, r):
    """Queries placed at float distance r (1 +- 4e-7) from terrain points, in random
    directions: every neighbour count of the pruned tree equals the exact grid count."""
    pts = scene.terrain[:, :3]
    rng = np.random.default_rng(5)
    sel = rng.integers(0, pts.shape[0], 400_000)
    u = rng.normal(size=(sel.size, 3))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    d = r * (1.0 + rng.uniform(-4e-7, 4e-7, sel.size))
    q = (pts[sel].astype(np.float64) + u * d[:, None]).astype(np.float32)
    tree = oracle.KdTree(scene.terrain)
    grid = oracle.Cloud(scene.terrain)
    oracle.set_threads(8)
    try:
        st = tree.check_queries(grid, q, r)
    finally:
        oracle.set_threads(1)
    assert st["queries"] == sel.size and st["neighbours"] > 0
    assert st["count_mismatch"] == 0 and st["any_mismatch"] == 0, st


def test_flann_mode_reproduces_golden_fan(oracle):
    d = np.load(GOLD / "fan.npz")
    T = oracle.Cloud(d["terrain"], flann=True)
    b, u, fh = oracle.raycast_fan(T, d["poses"], int(d["n_az"]), int(d["n_el"]),
                                  float(d["el_min"]), float(d["el_max"]),
                                  float(d["max_distance"]))
    np.testing.assert_array_equal(fh, d["first_hit"])
    np.testing.assert_array_equal(b, d["blocked"])
    np.testing.assert_array_equal(u, d["units"])


def test_flann_mode_reproduces_golden_scores(oracle):
    """generateCandidatePositions (getGroundHeight through the tree's neighbour list), then
    runOptimization's scoring with the relaxed zx120 check and the march through the tree."""
    d = np.load(GOLD / "score.npz")
    T = oracle.Cloud(d["terrain"], flann=True)
    A = oracle.Cloud(d["aux"], flann=True)
    cand = oracle.generate_candidates(T, d["grid_bbox"],
                                      oracle.vl_params(num_candidates=int(d["num_candidates"])),
                                      d["zx"])
    np.testing.assert_array_equal(cand, d["candidates"])
    flags = np.zeros(d["cells"].shape[0], np.uint8)
    tot, cov, rep = oracle.score_poses(T, A, d["cells"], d["normals"], cand, d["zx"],
                                       oracle.vl_params(max_distance=float(d["max_distance"])),
                                       flags)
    np.testing.assert_array_equal(tot, d["total"])
    np.testing.assert_array_equal(cov, d["covered"])
    np.testing.assert_array_equal(flags, d["flags"])
    assert rep.best_idx == d["report"][0]


def test_flann_fan_sample_queries_small_scene(oracle, small_scene):
    """Every sample query the reference executes on 6 poses x a 256 x 64 fan over the 200 x
    200 pit scene: tree count == grid count at each sample, and the first hits agree."""
    T = oracle.KdTree(small_scene.terrain)
    G = oracle.Cloud(small_scene.terrain)
    poses = np.array([[8.0, -3.0, 1.1, -0.5, 2.6], [1.0, 3.0, 1.1, -0.4, -1.2],
                      [2.5, -1.0, 0.3, -0.2, 0.0], [6.0, 2.0, 2.5, -0.8, -2.0],
                      [3.0, -6.0, 1.0, -0.3, 1.4], [20.0, 20.0, 1.0, 0.0, 0.0]])
    el = math.radians(85.0)
    oracle.set_threads(8)
    try:
        b, u, fh, st = oracle.raycast_fan_kd(T, G, poses, 256, 64, -el, el, 15.0)
        rb, ru, rfh = oracle.raycast_fan(G, poses, 256, 64, -el, el, 15.0)
    finally:
        oracle.set_threads(1)
    assert st["queries"] == int(u.sum()) and st["neighbours"] > 0
    assert st["count_mismatch"] == 0 and st["any_mismatch"] == 0, st
    np.testing.assert_array_equal(fh, rfh)
    np.testing.assert_array_equal(b, rb)
    np.testing.assert_array_equal(u, ru)
