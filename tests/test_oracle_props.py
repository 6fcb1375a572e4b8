"""Property tests (hypothesis) of the checker: the oracle's crop, VoxelGrid and FLANN radius
predicate against the independent numpy restatements of tests/test_oracle.py, on generated
clouds, boxes and leaf sizes -- including points placed exactly on box faces and voxel
boundaries, where the float-vs-double compares and the float keying decide the outcome."""
import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from test_oracle import _flann_any, _pcl_voxel_numpy  # noqa: E402

F32 = np.float32
SETTINGS = settings(max_examples=40, deadline=None, derandomize=True)


def _cloud(seed, n, span, on_grid):
    rng = np.random.default_rng(seed)
    p = rng.uniform(-span, span, (n, 4)).astype(F32)
    if on_grid:   # many coordinates exactly on multiples of 0.05 (voxel faces, box faces)
        k = n // 3
        p[:k, :3] = (np.round(p[:k, :3] / F32(0.05)) * F32(0.05)).astype(F32)
    return p


@SETTINGS
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(0, 3000),
       lo=st.lists(st.floats(-3, 1, width=32), min_size=3, max_size=3),
       ext=st.lists(st.floats(0, 4, width=32), min_size=3, max_size=3),
       on_grid=st.booleans())
def test_crop_matches_numpy(oracle, seed, n, lo, ext, on_grid):
    p = _cloud(seed, n, 4.0, on_grid)
    box = np.array([lo[0], lo[0] + ext[0], lo[1], lo[1] + ext[1], lo[2], lo[2] + ext[2]])
    if n:   # points exactly on the faces: the compares are strict
        p[: min(n, 6), 0] = F32(box[0])
        p[6:12, 1] = F32(box[3])
    x, y, z = (p[:, i].astype(np.float64) for i in range(3))
    m = (x > box[0]) & (x < box[1]) & (y > box[2]) & (y < box[3]) & (z > box[4]) & (z < box[5])
    np.testing.assert_array_equal(oracle.crop_box(p, box), np.nonzero(m)[0])


@SETTINGS
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(1, 2500),
       leaf=st.sampled_from([0.05, 0.1, 0.2, 0.37, 1.0]), span=st.floats(0.1, 6.0),
       on_grid=st.booleans())
def test_voxel_matches_numpy(oracle, seed, n, leaf, span, on_grid):
    p = _cloud(seed, n, span, on_grid)[:, :3].copy()
    ref = _pcl_voxel_numpy(p, leaf)
    xyz, idx, cnt, pt = oracle.voxel_grid(p, leaf)
    if ref is None:
        assert pt
        return
    keys, counts, cent = ref
    assert not pt
    np.testing.assert_array_equal(idx, keys)
    np.testing.assert_array_equal(cnt, counts)
    np.testing.assert_array_equal(xyz, cent)


@SETTINGS
@given(seed=st.integers(0, 2**31 - 1), sigma=st.floats(0.005, 0.2),
       radius=st.sampled_from([0.056, 0.24, 1.5]))
def test_radius_predicate_matches_bruteforce(oracle, small_scene, seed, sigma, radius):
    pts = small_scene.terrain
    C = oracle.Cloud(pts)
    rng = np.random.default_rng(seed)
    base = pts[rng.integers(0, pts.shape[0], 40), :3]
    q = (base + rng.normal(0, sigma, base.shape)).astype(F32)
    for i in range(q.shape[0]):
        assert C.any_within(q[i], radius) == _flann_any(pts[:, :3], q[i], radius)
