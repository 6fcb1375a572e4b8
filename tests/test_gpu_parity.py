"""GPU parity: libpcp (HIP, gfx950) against the CPU restatement (oracle/) on the same inputs.

Bar (BASELINE.json north_star): crop indices, voxel keys/counts, ray first-hit indices, cell
flags/covered counts and best-pose indices bit-exact; voxel centroids <= 1e-5 m; transformed
xyz exact (same float evaluation order); per-pose score totals (double, through ocml acos/sin vs
glibc) within 4 ulps each and at most max(2, 25 %) of them not bit-identical; candidate pitch/yaw
(correctly rounded atan2) at most 2 values one ulp off (tests/parity.py).
All calls go through the C ABI (pointcloud_processor_amd/_abi.py -> libpcp.so).
"""
import ctypes
import math
from pathlib import Path

import numpy as np
import parity
import pytest

from pointcloud_processor_amd import _abi, synth

pytestmark = pytest.mark.gpu

BOX = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])   # pointcloud_filter.cpp:30-36,111-113
GOLD = Path(__file__).resolve().parent / "golden"
C_u64, C_ref = ctypes.c_uint64, ctypes.byref


def _cloud(n, seed, step_floats=4, nan_frac=0.01):
    rng = np.random.default_rng(seed)
    a = np.zeros((n, step_floats), np.float32)
    a[:, 0] = rng.uniform(-5, 20, n)
    a[:, 1] = rng.uniform(-12, 12, n)
    a[:, 2] = rng.uniform(-3, 12, n)
    if n:
        k = max(1, int(n * nan_frac))
        a[rng.integers(0, n, k), rng.integers(0, 3, k)] = np.nan
        # exact boundary values of the strict box
        b = rng.integers(0, n, min(n, 64))
        a[b[:16], 0] = 0.0
        a[b[16:32], 0] = 15.0
        a[b[32:48], 1] = -10.0
        a[b[48:], 2] = -1.5
    return a


# ---------------------------------------------------------------------------------- filter
@pytest.mark.parametrize("n", [0, 1, 97, 4096, 100_003, 1_000_000])
def test_crop_indices_bit_exact(gpu, oracle, n):
    a = _cloud(n, 1 + n)
    kept, xyz = gpu.crop_box(a, BOX)
    ref = oracle.crop_box(a, BOX)
    np.testing.assert_array_equal(kept, ref)
    np.testing.assert_array_equal(xyz[:, :3], a[ref, :3])


def test_crop_point_step_32_offsets(gpu, oracle):
    a = _cloud(50_000, 7, step_floats=8)
    # fields at x@16, y@20, z@24 of a 32-byte record
    b = np.zeros_like(a)
    b[:, 4:7] = a[:, :3]
    kept, _ = gpu.crop_box(b, BOX, point_step=32, offs=(16, 20, 24))
    np.testing.assert_array_equal(kept, oracle.crop_box(a, BOX))


@pytest.mark.parametrize("n,leaf", [(1, 0.2), (5000, 0.2), (300_000, 0.2), (300_000, 0.05),
                                    (2_000_000, 0.05)])
def test_voxel_grid_exact(gpu, oracle, n, leaf):
    a = _cloud(n, 11 + n, nan_frac=0.0)
    out, idx, cnt, pt = gpu.voxel_grid(a, leaf)
    r_xyz, r_idx, r_cnt, r_pt = oracle.voxel_grid(a, leaf)
    assert pt == r_pt
    np.testing.assert_array_equal(idx, r_idx)
    np.testing.assert_array_equal(cnt, r_cnt)
    # same (stable) in-voxel summation order -> identical floats; the reference's own
    # spreadsort order may differ, hence the documented 1e-5 m tolerance
    np.testing.assert_allclose(out[:, :3], r_xyz, rtol=0, atol=1e-5)
    assert np.array_equal(out[:, :3], r_xyz)


@pytest.mark.parametrize("n,span", [(200_000, 1.0), (100_000, 0.01)])
def test_voxel_grid_dense_voxels(gpu, oracle, n, span):
    """Thousands of points per voxel (span 1 m / leaf 0.2 = 125 voxels) and a single voxel
    holding every point: segments crossing many sort tiles, long in-order centroid sums."""
    rng = np.random.default_rng(n)
    a = np.zeros((n, 4), np.float32)
    a[:, :3] = rng.uniform(0.0, span, (n, 3))
    out, idx, cnt, pt = gpu.voxel_grid(a, 0.2)
    r_xyz, r_idx, r_cnt, _ = oracle.voxel_grid(a, 0.2)
    assert not pt
    np.testing.assert_array_equal(idx, r_idx)
    np.testing.assert_array_equal(cnt, r_cnt)
    np.testing.assert_array_equal(out[:, :3], r_xyz)


def test_voxel_grid_nan_and_overflow(gpu, oracle):
    a = _cloud(20_000, 3, nan_frac=0.05)
    out, idx, cnt, pt = gpu.voxel_grid(a, 0.2)
    fin = np.isfinite(a[:, :3]).all(1)
    r_xyz, r_idx, r_cnt, _ = oracle.voxel_grid(a[fin], 0.2)
    np.testing.assert_array_equal(idx, r_idx)
    np.testing.assert_array_equal(out[:, :3], r_xyz)
    # PCL int32 overflow guard -> passthrough of the (finite) input
    big = np.array([[0, 0, 0, 0], [1000, 1000, 1000, 0], [5, 5, 5, 0]], np.float32)
    out, idx, cnt, pt = gpu.voxel_grid(big, 0.001)
    r_xyz, _, _, r_pt = oracle.voxel_grid(big, 0.001)
    assert pt and r_pt
    np.testing.assert_array_equal(out[:, :3], r_xyz)


@pytest.mark.parametrize("leaf", [0.0, 0.2])
def test_crop_voxel_pipeline(gpu, oracle, leaf):
    a = _cloud(400_000, 5)
    out, ncrop = gpu.crop_voxel(a, BOX, leaf)
    kept = oracle.crop_box(a, BOX)
    assert ncrop == kept.size
    if leaf > 0:
        r_xyz, _, _, _ = oracle.voxel_grid(a[kept], leaf)
    else:
        r_xyz = a[kept, :3]
    np.testing.assert_array_equal(out[:, :3], r_xyz)


@pytest.mark.parametrize("seed", range(8))
def test_crop_voxel_random_boxes(gpu, oracle, seed):
    """Random boxes, leaf sizes and clouds with a third of the coordinates on the 0.05 grid (box
    faces and voxel boundaries), through the GPU crop + voxel against the oracle."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(1, 300_000))
    a = rng.uniform(-6, 6, (n, 4)).astype(np.float32)
    k = n // 3
    a[:k, :3] = (np.round(a[:k, :3] / np.float32(0.05)) * np.float32(0.05)).astype(np.float32)
    lo = rng.uniform(-5, 1, 3)
    box = np.array([lo[0], lo[0] + rng.uniform(0, 8), lo[1], lo[1] + rng.uniform(0, 8),
                    lo[2], lo[2] + rng.uniform(0, 8)])
    box[::2] = np.round(box[::2] / 0.05) * 0.05      # faces on the grid too
    leaf = float(rng.choice([0.0, 0.05, 0.1, 0.2, 0.37]))
    out, ncrop = gpu.crop_voxel(a, box, leaf)
    kept = oracle.crop_box(a, box)
    assert ncrop == kept.size
    ref = oracle.voxel_grid(a[kept], leaf)[0] if leaf > 0 and kept.size else a[kept, :3]
    np.testing.assert_array_equal(out[:, :3], ref)


# ---------------------------------------------------------------------------------- merger
def _tfs():
    yaw = math.radians(30.0)
    q_robot = (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))
    return [((8.0, -3.0, 0.0), q_robot), ((0.55, 0.4, 3.5), (0.0, math.sin(0.4363 / 2), 0.0,
                                                              math.cos(0.4363 / 2)))]


def test_transform_concat_exact(gpu, oracle):
    a = _cloud(70_001, 21, nan_frac=0.0)
    b = _cloud(33_333, 22, nan_frac=0.0)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    out = gpu.transform_concat([a, b], tfs, rgbs)
    ref = np.concatenate([oracle.transform_rgb(a, *tfs[0], rgbs[0]),
                          oracle.transform_rgb(b, *tfs[1], rgbs[1])])
    assert out.shape == ref.shape
    np.testing.assert_array_equal(out[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))


def test_filter_merge_pipeline(gpu, oracle):
    a = synth.lidar_cloud(300_000, seed=1)
    b = synth.lidar_cloud(200_000, seed=2, sensor_height=3.5)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    out, per = gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs)
    parts = []
    for c, tf, rgb in zip([a, b], tfs, rgbs):
        k = oracle.crop_box(c, BOX)
        v, _, _, _ = oracle.voxel_grid(c[k], 0.05)
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    assert list(per) == [p.shape[0] for p in parts]
    np.testing.assert_array_equal(out[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))


def test_filter_merge_full_c3_frame(gpu, oracle):
    """The whole C3 frame of bench.py --mode filter (2 x 5 M LiDAR-like points, crop + voxel
    0.05 + transform + colour): every output record bit-exact against the oracle."""
    import math

    a = synth.lidar_cloud(5_000_000, sensor_height=2.0, seed=1)
    b = synth.lidar_cloud(5_000_000, sensor_height=3.5, seed=2)
    yaw = math.radians(30.0)
    tfs = [((8.0, -3.0, 0.0), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))),
           ((0.55, 0.4, 3.5), (0.0, math.sin(0.4363 / 2), 0.0, math.cos(0.4363 / 2)))]
    rgbs = [(255, 0, 0), (0, 0, 255)]
    out, per = gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs)
    parts = []
    for c, tf, rgb in zip([a, b], tfs, rgbs):
        k = oracle.crop_box(c, BOX)
        v, _, _, _ = oracle.voxel_grid(c[k], 0.05)
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    assert list(per) == [p.shape[0] for p in parts]
    np.testing.assert_array_equal(out[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))


@pytest.mark.parametrize("second", ["direct", "unbounded", "empty"])
def test_filter_merge_sparse_survivors(gpu, oracle, second):
    """A certainly-voxelised cloud whose ~3,000 survivors are spread over ~1,500 crop tiles
    (one sort tile spans more crop tiles than the first sort pass stages in LDS), batched with a
    second cloud that is voxelised the same way, through the compaction-kernel path (unbounded
    box) or is empty; three calls in a row (the crop's block tickets reset)."""
    rng = np.random.default_rng(77)
    n = 6_000_000
    a = rng.uniform(20.0, 40.0, (n, 4)).astype(np.float32)          # outside BOX
    idx = rng.choice(n, 3000, replace=False)
    a[idx, :3] = rng.uniform([0.5, -5.0, 0.0], [10.0, 5.0, 5.0], (3000, 3)).astype(np.float32)
    b = synth.lidar_cloud(150_000, seed=3) if second != "empty" else np.zeros((0, 4), np.float32)
    box_b = BOX if second != "unbounded" else np.array([-np.inf, np.inf] * 3)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    parts = []
    for c, box, tf, rgb in zip([a, b], [BOX, box_b], tfs, rgbs):
        if c.shape[0] == 0:
            continue
        k = oracle.crop_box(c, box)
        v, _, _, pt = oracle.voxel_grid(c[k], 0.05)
        assert not pt
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    for _ in range(3):
        out, per = gpu.filter_merge([a, b], [BOX, box_b], 0.05, tfs, rgbs)
        assert list(per)[:len(parts)] == [p.shape[0] for p in parts]
        np.testing.assert_array_equal(out[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))


@pytest.mark.parametrize("case", ["dense_groups", "far_box", "one_pass", "fine_leaf"])
def test_filter_merge_fast_chain(gpu, oracle, case, monkeypatch):
    """The fast chain (box-relative keys formed in the crop, pass 0 straight from the crop
    tiles in groups of 8) against the oracle and the general chain (PCP_FM_FAST=0):
    dense_groups -- every point survives, so one pass-0 group holds 8 x 4096 items (8 chunks)
    and one voxel holds 100 k points; far_box -- a box 2 km from the origin with negative
    coordinates; one_pass -- a box of < 2^9 voxels (a single radix pass); fine_leaf -- leaf
    0.013 m (four passes over the key)."""
    rng = np.random.default_rng({"dense_groups": 1, "far_box": 2, "one_pass": 3,
                                 "fine_leaf": 4}[case])
    leaf = 0.05
    if case == "dense_groups":
        box = np.array([-1.0, 30.0, -10.0, 10.0, -3.0, 5.0])
        a = np.zeros((200_000, 4), np.float32)
        a[:, :3] = rng.uniform([0, -5, -1], [20, 5, 2], (200_000, 3))
        a[50_000:150_000, :3] = [3.01, 2.02, 0.33]
        b = synth.lidar_cloud(100_000, seed=8)
    elif case == "far_box":
        box = np.array([-2105.0, -2085.0, 1990.0, 2010.0, -1.5, 9.0])
        a = np.zeros((400_000, 4), np.float32)
        a[:, :3] = rng.uniform([-2110, 1985, -3], [-2080, 2015, 10], (400_000, 3))
        b = a[::-1].copy()
    elif case == "one_pass":
        box = np.array([1.0, 1.3, -0.2, 0.1, 0.0, 0.2])
        a = np.zeros((300_000, 4), np.float32)
        a[:, :3] = rng.uniform([0.8, -0.4, -0.1], [1.5, 0.3, 0.3], (300_000, 3))
        b = a.copy()
        b[:, 2] += np.float32(0.05)
    else:
        leaf = 0.013
        box = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 1.5])
        a = synth.lidar_cloud(600_000, seed=9)
        b = synth.lidar_cloud(400_000, seed=10, sensor_height=3.5)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    parts = []
    for c, tf, rgb in zip([a, b], tfs, rgbs):
        k = oracle.crop_box(c, box)
        v, _, _, pt = oracle.voxel_grid(c[k], leaf)
        assert not pt
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    out, per = gpu.filter_merge([a, b], [box, box], leaf, tfs, rgbs)
    assert list(per) == [p.shape[0] for p in parts]
    np.testing.assert_array_equal(out[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
    monkeypatch.setenv("PCP_FM_FAST", "0")
    ctx = _abi.Context(0)
    try:
        out2, per2 = ctx.filter_merge([a, b], [box, box], leaf, tfs, rgbs)
    finally:
        ctx.close()
    assert list(per2) == list(per)
    np.testing.assert_array_equal(out2.view(np.uint32), out.view(np.uint32))


@pytest.mark.parametrize("case", ["lidar", "three_clouds", "tiny", "one_bucket", "dense_redo",
                                  "near_cap", "dense_voxel"])
def test_filter_merge_bucket_chain(oracle, case, monkeypatch):
    """The bucket chain (PCP_FM_FAST=2, the default: crop -> per-group counting sort by bucket ->
    per-bucket LDS sort + input-order sums + look-back offsets) against the oracle and the LSD
    fast chain (PCP_FM_FAST=1).  lidar: two LiDAR clouds; three_clouds: a middle cloud with
    nothing cropped (no buckets) between two that voxelise; tiny: 5 points; one_bucket: a box of
    < 2^11 voxels (one bucket, bs = 0); dense_redo: one voxel of 60 k points (its bucket passes
    the LDS capacity, the frame is redone on the LSD chain: voxel_redo counts it); near_cap: a
    dense cluster whose bucket stays just under the capacity, but whose ONE voxel of ~3,500
    points passes kBkDense (512: the in-voxel rank is quadratic) -- redone too;
    dense_voxel: 400 points in one voxel, ranked in the bucket chain."""
    rng = np.random.default_rng(50 + len(case))
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    box = BOX
    redo = 0
    if case == "lidar":
        clouds = [synth.lidar_cloud(700_000, seed=31), synth.lidar_cloud(500_000, seed=32,
                                                                         sensor_height=3.5)]
    elif case == "three_clouds":
        far = rng.uniform(30, 40, (50_000, 4)).astype(np.float32)
        clouds = [synth.lidar_cloud(200_000, seed=33), far, synth.lidar_cloud(90_000, seed=34)]
        tfs = [tfs[0], tfs[1], tfs[0]]
        rgbs = [(255, 0, 0), (0, 255, 0), (0, 0, 255)]
    elif case == "tiny":
        clouds = [np.array([[1, 1, 1, 0], [1.01, 1.01, 1.01, 0], [5, -3, 2, 0], [2, 2, 2, 0],
                            [1.02, 1.0, 1.03, 0]], np.float32), synth.lidar_cloud(1000, seed=35)]
    elif case == "one_bucket":
        box = np.array([1.0, 1.5, -0.2, 0.3, 0.0, 0.2])
        a = np.zeros((200_000, 4), np.float32)
        a[:, :3] = rng.uniform([0.9, -0.3, -0.1], [1.6, 0.4, 0.3], (200_000, 3))
        clouds = [a, a[::-1].copy()]
    elif case == "dense_redo":
        a = synth.lidar_cloud(300_000, seed=36)
        a[100_000:160_000, :3] = [3.01, 2.02, 0.33]
        clouds = [a, synth.lidar_cloud(100_000, seed=37)]
        redo = 1
    elif case == "near_cap":   # ~3,500 points in one voxel of an otherwise sparse cloud
        a = synth.lidar_cloud(200_000, seed=38)
        a[50_000:53_500, :3] = [7.51, -1.02, 0.43]
        clouds = [a, synth.lidar_cloud(100_000, seed=39)]
        redo = 1
    else:   # dense_voxel: 400 points in one voxel (under kBkDense), spread over the input
        a = synth.lidar_cloud(200_000, seed=40)
        a[7:200_000:500, :3] = [4.26, 3.17, 0.12]
        clouds = [a, synth.lidar_cloud(100_000, seed=41)]
    parts = []
    for c, tf, rgb in zip(clouds, tfs, rgbs):
        k = oracle.crop_box(c, box)
        if k.size == 0:
            parts.append(np.zeros((0, 8), np.float32))
            continue
        v, _, _, pt = oracle.voxel_grid(c[k], 0.05)
        assert not pt
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    outs = {}
    for mode in ("2", "1"):
        monkeypatch.setenv("PCP_FM_FAST", mode)
        ctx = _abi.Context(0)
        try:
            for _ in range(2):
                out, per = ctx.filter_merge(clouds, [box] * len(clouds), 0.05, tfs, rgbs)
                assert list(per) == [p.shape[0] for p in parts]
                np.testing.assert_array_equal(out[:, :5].view(np.uint32),
                                              ref[:, :5].view(np.uint32))
            outs[mode] = out
            if mode == "2":
                assert ctx.profile_get("voxel_redo")[1] == 2 * redo
        finally:
            ctx.close()
    np.testing.assert_array_equal(outs["2"].view(np.uint32), outs["1"].view(np.uint32))


@pytest.mark.parametrize("case", ["scans", "dense_redo", "empty_crop"])
def test_filter_merge_nodes(gpu, oracle, case):
    """pcp_filter_merge_nodes (the filter node for both sensors + the merger node composed, ONE
    synchronisation): each cloud's filtered message bit-identical to pcp_crop_voxel's (and the
    oracle's crop + VoxelGrid), the merged records bit-identical to pcp_transform_concat over
    them (and the oracle's), the cropped counts exact.  scans: two C5 scans (leaf 0.2, bucket
    chain); dense_redo: a 60 k-point voxel (the bucket chain's redo -> the general chain);
    empty_crop: a cloud with nothing in its box."""
    rng = np.random.default_rng(77)
    a = synth.lidar_cloud(60_032, sensor_height=2.0, seed=101)
    b = synth.lidar_cloud(60_032, sensor_height=3.5, seed=102)
    leaf = 0.2
    if case == "dense_redo":
        a = synth.lidar_cloud(200_000, seed=36)
        a[10_000:70_000, :3] = [3.01, 2.02, 0.33]
        leaf = 0.05
    elif case == "empty_crop":
        b = rng.uniform(30, 40, (5_000, 4)).astype(np.float32)
    clouds = [a, b]
    tfs = [((8.0, -3.0, 2.0), (0.0, 0.0, 0.2588190451025208, 0.9659258262890683)),
           ((0.55, 0.4, 3.5), (0.0, 0.21633, 0.0, 0.97632))]
    rgbs = [(255, 0, 0), (0, 0, 255)]
    merged, filt, crop = gpu.filter_merge_nodes(clouds, [BOX, BOX], leaf, tfs, rgbs)
    # the same bytes where they landed (pcp_filter_merge_landed: what the C++ composed front
    # builds its messages from and the composed carve reads in place)
    mp = ctypes.c_void_p()
    fp = (ctypes.c_void_p * 2)()
    assert gpu.lib.pcp_filter_merge_landed(gpu.h, 2, ctypes.byref(mp), fp) == 0
    if merged.size:
        got = np.ctypeslib.as_array(ctypes.cast(mp, ctypes.POINTER(ctypes.c_float)),
                                    (merged.shape[0], 8))
        np.testing.assert_array_equal(got.view(np.uint32), merged.view(np.uint32))
    for i, f in enumerate(filt):
        if f.shape[0]:
            got = np.ctypeslib.as_array(ctypes.cast(fp[i], ctypes.POINTER(ctypes.c_float)),
                                        (f.shape[0], 4))
            np.testing.assert_array_equal(got[:, :3].view(np.uint32), f[:, :3].view(np.uint32))
    assert gpu.lib.pcp_filter_merge_landed(gpu.h, 3, ctypes.byref(mp), fp) != 0   # (k differs)
    ref_f = []
    for c, f, m in zip(clouds, filt, crop):
        kept = oracle.crop_box(c, BOX)
        assert int(m) == kept.size
        v = oracle.voxel_grid(c[kept], leaf)[0] if kept.size else np.zeros((0, 3), np.float32)
        np.testing.assert_array_equal(f[:, :3], v)
        g, ncrop = gpu.crop_voxel(c, BOX, leaf)
        assert ncrop == kept.size
        np.testing.assert_array_equal(f[:, :3], g[:, :3])
        ref_f.append(v)
    ref = np.concatenate([oracle.transform_rgb(v, *tf, rgb) for v, tf, rgb in
                          zip(ref_f, tfs, rgbs)])
    np.testing.assert_array_equal(merged[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
    tc = gpu.transform_concat([f[:, :3].copy() for f in filt], tfs, rgbs)
    np.testing.assert_array_equal(merged[:, :5].view(np.uint32), tc[:, :5].view(np.uint32))


def test_crop_voxel_bucket_chain_voxel_order(gpu, oracle):
    """pcp_voxel_grid's idx / count outputs come from the general chain; pcp_crop_voxel's
    centroids from the bucket chain (run_single): the same centroids, in PCL idx order."""
    a = synth.lidar_cloud(400_000, seed=41)
    out, ncrop = gpu.crop_voxel(a, BOX, 0.05)
    kept = oracle.crop_box(a, BOX)
    r_xyz, r_idx, r_cnt, _ = oracle.voxel_grid(a[kept], 0.05)
    assert ncrop == kept.size
    np.testing.assert_array_equal(out[:, :3], r_xyz)
    assert np.all(np.diff(r_idx.astype(np.int64)) > 0)


def test_filter_merge_device_graph_replay(gpu, oracle):
    """Device-resident inputs: the pipeline is captured into a hipGraph and replayed; every
    replay must equal the eager host-path result and the oracle."""
    a = synth.lidar_cloud(250_000, seed=5)
    b = synth.lidar_cloud(150_000, seed=6, sensor_height=3.5)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    ref, per_ref = gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs)
    dp = [gpu.dev_alloc(c.nbytes) for c in (a, b)]
    for p, c in zip(dp, (a, b)):
        gpu.h2d(p, c)
    views = [_abi.CloudView(p, c.shape[0], 16, 0, 4, 8) for p, c in zip(dp, (a, b))]
    cap = a.shape[0] + b.shape[0]
    out_d = gpu.dev_alloc(cap * 32)
    try:
        for _ in range(3):   # capture, then replays
            n, per = gpu.filter_merge_device(views, [BOX, BOX], 0.05, tfs, rgbs, out_d, cap)
            assert n == ref.shape[0] and list(per) == list(per_ref)
            got = np.empty((n, 8), np.float32)
            gpu.d2h(got, out_d)
            np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
        # the prepared steady-state call replays the same graph
        frame = gpu.filter_merge_device_prepared(views, [BOX, BOX], 0.05, tfs, rgbs, out_d, cap)
        for _ in range(2):
            n3, per3 = frame()
            assert n3 == ref.shape[0] and list(per3) == list(per_ref)
            got = np.empty((n3, 8), np.float32)
            gpu.d2h(got, out_d)
            np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
        # a different box invalidates the captured graph
        box2 = BOX.copy()
        box2[1] = 8.0
        n2, _ = gpu.filter_merge_device(views, [box2, box2], 0.05, tfs, rgbs, out_d, cap)
        ref2, _ = gpu.filter_merge([a, b], [box2, box2], 0.05, tfs, rgbs)
        assert n2 == ref2.shape[0] and n2 < n
    finally:
        for p in dp + [out_d]:
            gpu.dev_free(p)
    parts = []
    for c, tf, rgb in zip([a, b], tfs, rgbs):
        k = oracle.crop_box(c, BOX)
        v, _, _, _ = oracle.voxel_grid(c[k], 0.05)
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    np.testing.assert_array_equal(ref[:, :5].view(np.uint32),
                                  np.concatenate(parts)[:, :5].view(np.uint32))


def test_filter_merge_device_graph_redo(oracle):
    """Device-resident inputs through the captured graph when the bucket chain must redo the
    frame (one 30 k-point voxel: its bucket passes the LDS capacity): every replay redoes the
    frame on the LSD chain inside the call and returns the oracle's bytes; a later frame whose
    buckets fit replays the same graph without a redo."""
    a = synth.lidar_cloud(200_000, seed=61)
    a[20_000:50_000, :3] = [4.01, -2.02, 0.51]
    b = synth.lidar_cloud(100_000, seed=62, sensor_height=3.5)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    parts = []
    for c, tf, rgb in zip([a, b], tfs, rgbs):
        k = oracle.crop_box(c, BOX)
        v, _, _, _ = oracle.voxel_grid(c[k], 0.05)
        parts.append(oracle.transform_rgb(v, *tf, rgb))
    ref = np.concatenate(parts)
    ctx = _abi.Context(0)
    dp = [ctx.dev_alloc(c.nbytes) for c in (a, b)]
    cap = a.shape[0] + b.shape[0]
    out_d = ctx.dev_alloc(cap * 32)
    try:
        for p, c in zip(dp, (a, b)):
            ctx.h2d(p, c)
        views = [_abi.CloudView(p, c.shape[0], 16, 0, 4, 8) for p, c in zip(dp, (a, b))]
        for i in range(3):   # capture, then replays
            n, per = ctx.filter_merge_device(views, [BOX, BOX], 0.05, tfs, rgbs, out_d, cap)
            assert n == ref.shape[0] and list(per) == [p.shape[0] for p in parts]
            got = np.empty((n, 8), np.float32)
            ctx.d2h(got, out_d)
            np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
            assert ctx.profile_get("voxel_redo")[1] == i + 1
        # the dense voxel gone (same views, same graph): no redo
        a2 = synth.lidar_cloud(200_000, seed=61)
        ctx.h2d(dp[0], a2)
        n2, _ = ctx.filter_merge_device(views, [BOX, BOX], 0.05, tfs, rgbs, out_d, cap)
        assert ctx.profile_get("voxel_redo")[1] == 3
        k2 = oracle.crop_box(a2, BOX)
        v2, _, _, _ = oracle.voxel_grid(a2[k2], 0.05)
        ref2 = np.concatenate([oracle.transform_rgb(v2, *tfs[0], rgbs[0]), parts[1]])
        got = np.empty((n2, 8), np.float32)
        ctx.d2h(got, out_d)
        np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref2[:, :5].view(np.uint32))
    finally:
        for p in dp + [out_d]:
            ctx.dev_free(p)
        ctx.close()


def test_filter_merge_pinned_staging(gpu):
    """PointCloud2 boundary with page-locked buffers: clouds and the output pinned in place
    (pcp_host_register) and a pcp_host_alloc block must give the pageable path's bytes."""
    a = synth.lidar_cloud(120_000, seed=9)
    b = synth.lidar_cloud(80_000, seed=10, sensor_height=3.5)
    tfs = _tfs()
    rgbs = [(255, 0, 0), (0, 0, 255)]
    ref, per_ref = gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs)
    out = np.empty((a.shape[0] + b.shape[0], 8), np.float32)
    for x in (a, b, out):
        gpu.host_register(x)
    try:
        got, per = gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs, out=out)
        assert list(per) == list(per_ref)
        np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
    finally:
        for x in (a, b, out):
            gpu.host_unregister(x)
    # a pinned allocation from the library, filled in place and used as the input cloud
    hp = ctypes.c_void_p()
    assert gpu.lib.pcp_host_alloc(gpu.h, a.nbytes, C_ref(hp)) == 0 and hp.value
    try:
        pinned = np.ctypeslib.as_array(ctypes.cast(hp, ctypes.POINTER(ctypes.c_float)),
                                       shape=a.shape)
        pinned[:] = a
        got, per = gpu.filter_merge([pinned, b], [BOX, BOX], 0.05, tfs, rgbs)
        assert list(per) == list(per_ref)
        np.testing.assert_array_equal(got[:, :5].view(np.uint32), ref[:, :5].view(np.uint32))
    finally:
        assert gpu.lib.pcp_host_free(gpu.h, hp) == 0
    with pytest.raises(ValueError):                       # output too small
        gpu.filter_merge([a, b], [BOX, BOX], 0.05, tfs, rgbs, out=out[:10])


# ---------------------------------------------------------------------------------- virtual_lidar
@pytest.fixture(scope="module")
def loaded(gpu, oracle, scene, cells, aux):
    gpu.set_terrain(scene.terrain, point_step=32)
    gpu.set_aux_cloud(aux, point_step=32)
    gpu.set_cells(cells.xyz, cells.normals)
    T = oracle.Cloud(scene.terrain)
    A = oracle.Cloud(aux)
    return T, A


def test_terrain_index_info(gpu, loaded, scene):
    info = gpu.terrain_info()
    assert info["n_points"] == scene.terrain.shape[0]
    assert info["cell"] >= 2 * (0.08 * 0.7)


def test_candidates_match(gpu, oracle, loaded, scene, cells):
    """generateCandidatePositions: positions bit-exact; pitch and yaw (atan2, correctly rounded
    on the device, pcp_crmath.h) bit-identical to glibc's but for its rare near-tie misroundings
    (at most 2 values here, one ulp each: tests/parity.py; ocml's own atan2 left ~8 % one ulp
    off)."""
    T, _ = loaded
    for nc in (100, 400, 1000):
        p = _abi.default_vl_params(num_candidates=nc)
        g = gpu.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5)
        r = oracle.generate_candidates(T, cells.grid_bbox, oracle.vl_params(num_candidates=nc),
                                       scene.zx120_pose5)
        assert g.shape == r.shape
        np.testing.assert_array_equal(g[:, :3], r[:, :3])
        np.testing.assert_allclose(g[:, 3:], r[:, 3:], rtol=0, atol=1e-12)
        parity.assert_angles(g[:, 3:], r[:, 3:])   # <= 2 values, one ulp each


def test_step_table():
    s = _abi.step_table(15.0 - 0.08)
    assert s.size == 49 and s[0] == 0.5
    ref = [0.5]
    while True:
        x = ref[-1] + 0.3
        if not x < 15.0 - 0.08:
            break
        ref.append(x)
    assert np.array_equal(s, np.array(ref))


def test_raycast_fan_first_hit_exact(gpu, oracle, loaded, scene, cells):
    T, _ = loaded
    p = _abi.default_vl_params(num_candidates=100)
    poses = gpu.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5)[:6]
    fan = _abi.fan_params(n_az=256, n_el=64)
    blocked, units, fh, best = gpu.raycast_fan(poses, fan, want_first_hit=True)
    r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, 256, 64, fan.el_min, fan.el_max,
                                                  fan.max_distance)
    np.testing.assert_array_equal(fh, r_fh)
    np.testing.assert_array_equal(blocked, r_blocked)
    np.testing.assert_array_equal(units, r_units)
    assert best == int(np.argmin(r_blocked))
    # depths = step table entries (exact), within the 1e-4 m bar trivially
    steps = _abi.step_table(fan.max_distance - 0.08)
    d = np.where(fh >= 0, steps[np.maximum(fh, 0)], np.nan)
    rd = np.where(r_fh >= 0, steps[np.maximum(r_fh, 0)], np.nan)
    np.testing.assert_allclose(d, rd, atol=1e-4, equal_nan=True)


def test_raycast_fan_random_poses(gpu, oracle, loaded, scene):
    """Poses anywhere around the terrain: inside and outside its bbox, below the ground, in
    the pit, at any pitch/yaw; odd fan sizes and elevation limits."""
    T, _ = loaded
    rng = np.random.default_rng(7)
    pts = scene.terrain[:, :3]
    lo, hi = pts.min(0) - 3.0, pts.max(0) + 3.0
    poses = np.column_stack([rng.uniform(lo[0], hi[0], 24), rng.uniform(lo[1], hi[1], 24),
                             rng.uniform(lo[2] - 1.0, hi[2] + 3.0, 24),
                             rng.uniform(-1.5, 1.5, 24), rng.uniform(-np.pi, np.pi, 24)])
    for n_az, n_el, el_lo, el_hi, dmax in ((96, 17, -80.0, 80.0, 15.0), (130, 9, -17.0, 6.0, 7.5)):
        fan = _abi.fan_params(n_az=n_az, n_el=n_el, el_min_deg=el_lo, el_max_deg=el_hi,
                              max_distance=dmax)
        blocked, units, fh, _ = gpu.raycast_fan(poses, fan, want_first_hit=True)
        r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, n_az, n_el, fan.el_min,
                                                      fan.el_max, dmax)
        np.testing.assert_array_equal(fh, r_fh)
        np.testing.assert_array_equal(blocked, r_blocked)
        np.testing.assert_array_equal(units, r_units)


def test_into_wrappers_match(gpu, loaded, scene, cells):
    """The allocation-free steady-state calls give the allocating calls' results."""
    p = _abi.default_vl_params(num_candidates=100)
    poses = np.ascontiguousarray(gpu.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5))
    fan = _abi.fan_params(n_az=128, n_el=16)
    blocked, units, _, best = gpu.raycast_fan(poses, fan)
    b2 = np.zeros(poses.shape[0], np.uint32)
    u2 = np.zeros(poses.shape[0], np.uint64)
    assert gpu.raycast_fan_into(poses, fan, b2, u2) == best
    np.testing.assert_array_equal(b2, blocked)
    np.testing.assert_array_equal(u2, units)
    f1 = np.zeros(cells.xyz.shape[0], np.uint8)
    f2 = f1.copy()
    tot, cov, rep = gpu.score_poses(poses, scene.zx120_pose5, p, f1)
    t2 = np.zeros(poses.shape[0], np.float64)
    c2 = np.zeros(poses.shape[0], np.int32)
    r2 = _abi.VlReport()
    gpu.score_poses_into(poses, np.ascontiguousarray(scene.zx120_pose5, np.float64), p, f2, t2, c2,
                         r2)
    np.testing.assert_array_equal(t2, tot)
    np.testing.assert_array_equal(c2, cov)
    np.testing.assert_array_equal(f2, f1)
    assert r2.best_idx == rep.best_idx and r2.green == rep.green


@pytest.mark.parametrize("npw,tile,skip", [("1", "2", "1"), ("2", "2", "1"), ("8", "2", "1"),
                                           ("8", "1", "1"), ("8", "2", "2")])
def test_raycast_fan_poses_per_wave(oracle, loaded, scene, cells, npw, tile, skip, monkeypatch):
    """64 poses (P % 64 == 0: the XCD-chunk kernel with NPW poses per wave, its step table in
    LDS) on split and 8-byte fine records, split records with one or two walk-start skip
    thresholds (PCP_FINE_SKIP): blocked counts, units and first hits exact."""
    T, _ = loaded
    monkeypatch.setenv("PCP_FAN_NPW", npw)
    monkeypatch.setenv("PCP_FINE_SKIP", skip)
    monkeypatch.setenv("PCP_FINE_TILE", tile.rstrip("u"))
    monkeypatch.setenv("PCP_FINE_PACK", "0" if tile.endswith("u") else "1")
    monkeypatch.setenv("PCP_TERRAIN_BLOCKS", "2")
    ctx = _abi.Context(0)
    try:
        ctx.set_terrain(scene.terrain, point_step=32)
        p = _abi.default_vl_params(num_candidates=100)
        poses = ctx.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5)
        poses = np.ascontiguousarray(np.resize(poses, (64, 5)))
        fan = _abi.fan_params(n_az=256, n_el=32)
        blocked, units, fh, best = ctx.raycast_fan(poses, fan, want_first_hit=True)
        info = ctx.terrain_info()
        assert info["scan_layout"] == "fine" and info["fine_tile"] == int(tile)
    finally:
        ctx.close()
    oracle.set_threads(8)
    r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, 256, 32, fan.el_min, fan.el_max,
                                                  fan.max_distance)
    oracle.set_threads(1)
    np.testing.assert_array_equal(fh, r_fh)
    np.testing.assert_array_equal(blocked, r_blocked)
    np.testing.assert_array_equal(units, r_units)
    assert best == int(np.argmin(r_blocked))


def test_raycast_fan_full_size_two_poses(gpu, oracle, loaded, scene, cells):
    """BASELINE configs[1] fan (1024 x 256) on two poses, bit-exact against the oracle."""
    T, _ = loaded
    p = _abi.default_vl_params(num_candidates=400)
    poses = gpu.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5)
    poses = poses[[0, len(poses) // 2]]
    fan = _abi.fan_params()
    blocked, units, fh, best = gpu.raycast_fan(poses, fan, want_first_hit=True)
    oracle.set_threads(8)
    r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, 1024, 256, fan.el_min, fan.el_max,
                                                  fan.max_distance)
    oracle.set_threads(1)
    np.testing.assert_array_equal(fh, r_fh)
    np.testing.assert_array_equal(blocked, r_blocked)
    np.testing.assert_array_equal(units, r_units)


def _clutter_cloud(seed=17):
    """A volumetric cloud (not a surface): a noisy floor, a dense box of random points, a thin
    vertical wall and a few isolated points -- cells hold many points spread in z, so the z
    bands are wide and the run walks go deep."""
    rng = np.random.default_rng(seed)
    floor = np.c_[rng.uniform(-6, 6, (60_000, 2)), rng.normal(-1.0, 0.02, 60_000)]
    box = rng.uniform([-1.5, -1.5, -1.0], [1.5, 1.5, 1.5], (50_000, 3))
    wall = np.c_[np.full(8_000, 3.0) + rng.normal(0, 0.01, 8_000), rng.uniform(-4, 4, 8_000),
                 rng.uniform(-1, 2, 8_000)]
    iso = rng.uniform([-6, -6, -1], [6, 6, 3], (300, 3))
    pts = np.concatenate([floor, box, wall, iso]).astype(np.float32)
    out = np.zeros((pts.shape[0], 4), np.float32)
    out[:, :3] = pts
    return out


@pytest.mark.parametrize("n_az,n_el", [(100, 37), (64, 3)])
def test_raycast_fan_clutter_and_odd_fans(oracle, n_az, n_el):
    """Fan sizes that are not multiples of the 64-lane wave (a ring spans waves, partial last
    wave), against a volumetric cloud; poses inside the box, at its edge, above, below the
    floor and far outside.  First hits, blocked counts and ray-hit tests bit-exact."""
    cloud = _clutter_cloud()
    ctx = _abi.Context(0)
    try:
        ctx.set_terrain(cloud)
        poses = np.array([[0.0, 0.0, 0.2, 0.0, 0.3], [1.5, -1.5, 1.5, 0.0, -2.0],
                          [-4.0, 2.0, 2.5, 0.0, 1.0], [0.5, 4.0, -1.5, 0.0, 0.0],
                          [40.0, 40.0, 0.0, 0.0, 0.0], [2.9, 0.0, 0.5, 0.0, 3.1]])
        fan = _abi.fan_params(n_az=n_az, n_el=n_el)
        blocked, units, fh, best = ctx.raycast_fan(poses, fan, want_first_hit=True)
        T = oracle.Cloud(cloud)
        r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, n_az, n_el, fan.el_min,
                                                      fan.el_max, fan.max_distance)
        np.testing.assert_array_equal(fh, r_fh)
        np.testing.assert_array_equal(blocked, r_blocked)
        np.testing.assert_array_equal(units, r_units)
        assert best == int(np.argmin(r_blocked))
        assert blocked[4] == 0 and blocked[0] > 0
    finally:
        ctx.close()


@pytest.mark.parametrize("dz,skip", [(3000.0, "1"), (-2500.0, "1"), (3000.0, "2"),
                                     (-2500.0, "2")])
def test_raycast_fan_far_from_origin(oracle, scene, cells, dz, skip, monkeypatch):
    """The terrain and the poses shifted by kilometres in z, where float spacing (~2.4e-4 m)
    exceeds the fixed 1e-4 m margins: the split-record walk skip widens its margin with |z|
    (pcp_vlidar.hip), so first hits, blocked counts and ray-hit tests stay exact on the
    fine-window copy (built at the first query), with one or two skip thresholds."""
    monkeypatch.setenv("PCP_TERRAIN_BLOCKS", "2")
    monkeypatch.setenv("PCP_FINE_SKIP", skip)
    terr = np.ascontiguousarray(scene.terrain.copy())
    terr[:, 2] += np.float32(dz)
    ctx = _abi.Context(0)
    try:
        ctx.set_terrain(terr, point_step=32)
        p = _abi.default_vl_params(num_candidates=100)
        g = _abi.Context(0)
        try:
            g.set_terrain(scene.terrain, point_step=32)
            poses = g.generate_candidates(cells.grid_bbox, p, scene.zx120_pose5)[::9][:8].copy()
        finally:
            g.close()
        poses[:, 2] += dz
        fan = _abi.fan_params(n_az=256, n_el=64)
        blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
        assert ctx.terrain_info()["scan_layout"] == "fine"
    finally:
        ctx.close()
    oracle.set_threads(8)
    r_blocked, r_units, r_fh = oracle.raycast_fan(oracle.Cloud(terr), poses, 256, 64,
                                                  fan.el_min, fan.el_max, fan.max_distance)
    oracle.set_threads(1)
    np.testing.assert_array_equal(fh, r_fh)
    np.testing.assert_array_equal(blocked, r_blocked)
    np.testing.assert_array_equal(units, r_units)
    assert blocked.sum() > 0


def test_raycast_fan_without_terrain_and_empty(oracle):
    """No terrain tree: every ray runs to the end unblocked (the reference's visible = true);
    zero poses: nothing to do, best index -1; an all-NaN terrain: an empty tree."""
    ctx = _abi.Context(0)
    try:
        fan = _abi.fan_params(n_az=128, n_el=16)
        poses = np.array([[0.0, 0.0, 1.0, 0.0, 0.0], [3.0, 1.0, 2.0, 0.0, 1.0]])
        K = len(_abi.step_table(fan.max_distance - 0.08))
        blocked, units, _, best = ctx.raycast_fan(poses, fan)
        assert blocked.tolist() == [0, 0] and units.tolist() == [128 * 16 * K] * 2
        assert best == 0
        b0, u0, _, best0 = ctx.raycast_fan(np.zeros((0, 5)), fan)
        assert b0.size == 0 and u0.size == 0 and best0 == -1
        nan_cloud = np.full((1000, 4), np.nan, np.float32)
        ctx.set_terrain(nan_cloud)
        blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
        assert blocked.tolist() == [0, 0] and (fh == -1).all()
    finally:
        ctx.close()


def test_raycast_fan_full_c2_workload(gpu, oracle, loaded, scene):
    """The whole headline workload of bench.py (BASELINE configs[1]: 256 candidate poses x the
    1024 x 256 fan on the 1M-point terrain), every first hit bit-exact against the oracle
    (67 M rays; the oracle's OpenMP build takes a few seconds on the box's 16 cores)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    T, _ = loaded
    poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, 256)
    fan = _abi.fan_params()
    blocked, units, fh, best = gpu.raycast_fan(poses, fan, want_first_hit=True)
    oracle.set_threads(16)
    try:
        r_blocked, r_units, r_fh = oracle.raycast_fan(T, poses, 1024, 256, fan.el_min,
                                                      fan.el_max, fan.max_distance)
    finally:
        oracle.set_threads(1)
    assert np.array_equal(blocked, r_blocked) and np.array_equal(units, r_units)
    bad = np.count_nonzero(fh != r_fh)
    assert bad == 0, f"{bad} of {fh.size} first hits differ"
    assert best == int(np.argmin(r_blocked))


def test_c4_sharded_4096_poses(gpu, oracle, loaded, scene):
    """BASELINE configs[3]: 4096 candidate poses split into 8 contiguous shards of 512 (one
    per GPU of the 8-GPU node), each shard through pcp_raycast_fan, combined as the RCCL
    all-reduce(MIN) combines them (dist.reduce_fan key vectors, elementwise min).  Blocked
    counts and ray-hit tests of all 4096 poses and the best index against the oracle; first
    hits bit-exact for every 4th pose of EVERY shard (1,024 poses x 262,144 rays)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from pointcloud_processor_amd import dist as pd

    T, _ = loaded
    P, G = 4096, 8
    poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, P)
    assert poses.shape == (P, 5)
    fan = _abi.fan_params()
    key = np.full(P, pd.INT64_MAX, np.int64)
    units = np.zeros(P, np.uint64)
    oracle.set_threads(16)
    try:
        for g in range(G):
            lo, hi = pd.shard(P, G, g)
            assert hi - lo == 512
            b, u, fh, _ = gpu.raycast_fan(poses[lo:hi], fan, want_first_hit=True)
            k, _ = pd.reduce_fan(b, lo, hi, P)          # this rank's contribution
            key = np.minimum(key, k)                      # = all_reduce(MIN) over the ranks
            units[lo:hi] = u
            sel = np.arange(lo, hi, 4)                    # 128 poses of the shard
            _, _, r_fh = oracle.raycast_fan(T, poses[sel], 1024, 256, fan.el_min, fan.el_max,
                                            fan.max_distance)
            bad = np.count_nonzero(fh[sel - lo] != r_fh)
            assert bad == 0, f"shard {g}: {bad} first hits differ"
            del fh, r_fh
        best = int(np.argmin(key))
        r_blocked, r_units, _ = oracle.raycast_fan(T, poses, 1024, 256, fan.el_min, fan.el_max,
                                                   fan.max_distance, want_first_hit=False)
    finally:
        oracle.set_threads(1)
    np.testing.assert_array_equal(key, r_blocked.astype(np.int64))
    np.testing.assert_array_equal(units, r_units)
    assert best == int(np.argmin(r_blocked))


def test_terrain_replaced_after_block_copy(oracle, small_scene, scene):
    """set_terrain(A), two fan queries (the second builds A's block-major copy), then
    set_terrain(B) and a query: B's results must match the oracle on B (no stale copy or z
    bands of A paired with B's grid)."""
    ctx = _abi.Context(0)
    try:
        fan = _abi.fan_params(n_az=256, n_el=32)
        poses = np.array([[1.0, 0.5, 1.5, -0.3, 0.4], [6.0, -2.0, 1.2, -0.4, 2.5]])
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.raycast_fan(poses, fan)
        ctx.raycast_fan(poses, fan)
        B = small_scene.terrain
        ctx.set_terrain(B, point_step=32)
        for _ in range(3):   # before and after B's own block copy
            blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
            r_b, r_u, r_fh = oracle.raycast_fan(oracle.Cloud(B), poses, 256, 32, fan.el_min,
                                                fan.el_max, fan.max_distance)
            np.testing.assert_array_equal(fh, r_fh)
            np.testing.assert_array_equal(blocked, r_b)
            np.testing.assert_array_equal(units, r_u)
    finally:
        ctx.close()


def _rel_close(a, b):
    """The totals' parity bar (tests/parity.py): every value within 2 ulps of the oracle's and
    at most max(5, 10 %) of them not bit-identical -- the census's 3-5 %, <= 2 ulps (was a
    1e-12 relative tolerance, ~2,600x looser than the kernels' results)."""
    return parity.totals_match(a, b)


PERTURB_LIB = Path(__file__).resolve().parents[1] / "pointcloud_processor_amd" / "_lib" / \
    "perturb" / "libpcp.so"
PERTURB8_LIB = Path(__file__).resolve().parents[1] / "pointcloud_processor_amd" / "_lib" / \
    "perturb8" / "libpcp.so"


def test_parity_bar_catches_one_ulp(oracle, loaded, scene, cells, aux):
    """The totals' bar is tight enough to see a one-ulp error in evaluateCellScore
    (virtual_lidar.cpp:689-700): the `make perturb` build (every cell score nextafter'd up, all
    else the production objects) fails it on the 91-candidate tick, the production build passes
    it on the same inputs, and the flags / covered counts / best index stay equal (only the
    totals' bits can show such an error)."""
    assert PERTURB_LIB.exists() and PERTURB8_LIB.exists(), \
        "build first (__graft_entry__.build(): make perturb perturb8)"
    T, A = loaded
    params = _abi.default_vl_params()
    res = {}
    for tag, path in (("prod", None), ("perturbed", str(PERTURB_LIB)),
                      ("perturbed8", str(PERTURB8_LIB))):
        with _abi.Context(0, lib_path=path) as ctx:
            ctx.set_terrain(scene.terrain, point_step=32)
            ctx.set_aux_cloud(aux, point_step=32)
            ctx.set_cells(cells.xyz, cells.normals)
            poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
            fl = np.zeros(cells.xyz.shape[0], np.uint8)
            tot, cov, rep = ctx.score_poses(poses, scene.zx120_pose5, params, fl)
            res[tag] = (poses, tot, cov, rep.best_idx, fl)
    poses = res["prod"][0]
    r_tot, r_cov, r_rep = oracle.score_poses(T, A, cells.xyz, cells.normals, poses,
                                             scene.zx120_pose5, oracle.vl_params(),
                                             np.zeros(cells.xyz.shape[0], np.uint8))
    prod = parity.totals_report(res["prod"][1], r_tot)
    print("parity bar: production", prod)
    assert parity.totals_match(res["prod"][1], r_tot), prod
    for tag in ("perturbed", "perturbed8"):   # every cell / every 8th cell one ulp up
        bad = parity.totals_report(res[tag][1], r_tot)
        print("parity bar:", tag, bad)
        assert not parity.totals_match(res[tag][1], r_tot), (tag, bad)
        np.testing.assert_array_equal(res[tag][2], r_cov)
        assert res[tag][3] == r_rep.best_idx == res["prod"][3]


def test_score_poses_matches_reference_loop(gpu, oracle, loaded, scene, cells):
    T, A = loaded
    params = _abi.default_vl_params()
    poses = gpu.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
    assert len(poses) == 91
    flags_g = np.zeros(cells.xyz.shape[0], np.uint8)
    flags_r = flags_g.copy()
    tot, cov, rep = gpu.score_poses(poses, scene.zx120_pose5, params, flags_g)
    r_tot, r_cov, r_rep = oracle.score_poses(T, A, cells.xyz, cells.normals, poses,
                                             scene.zx120_pose5, oracle.vl_params(), flags_r)
    np.testing.assert_array_equal(flags_g, flags_r)
    np.testing.assert_array_equal(cov, r_cov)
    assert _rel_close(tot, r_tot), np.max(np.abs(tot - r_tot))
    gd, rd = rep.as_dict(), r_rep.as_dict()
    for k in gd:
        if k in ("best_score", "zx120_total_score"):
            assert _rel_close(gd[k], rd[k]), k
        else:
            assert gd[k] == rd[k], k
    srt = np.sort(r_tot)[::-1]
    assert (srt[0] - srt[1]) > 1e-9 * srt[0]     # the argmax is decidable at this tolerance
    # a second tick starts from the stale flags (GridCell state persists between ticks)
    tot2, _, rep2 = gpu.score_poses(poses[::-1].copy(), scene.zx120_pose5, params, flags_g)
    r_tot2, _, r_rep2 = oracle.score_poses(T, A, cells.xyz, cells.normals, poses[::-1].copy(),
                                           scene.zx120_pose5, oracle.vl_params(), flags_r)
    np.testing.assert_array_equal(flags_g, flags_r)
    assert rep2.best_idx == r_rep2.best_idx


@pytest.mark.parametrize("wide", ["1", "0"])
@pytest.mark.parametrize("npose", [1, 3])
def test_score_few_poses_wide_lanes(oracle, scene, cells, aux, wide, npose, monkeypatch):
    """Few rays (C1 / C5 score one candidate): k_score_cells_wide splits each ray's samples
    over 16 lanes and ANDs their verdicts.  Same flags, coverage, totals and best pose as the
    reference loop, with the wide kernel on (default) and off (PCP_SCORE_WIDE=0)."""
    monkeypatch.setenv("PCP_SCORE_WIDE", wide)
    params = _abi.default_vl_params()
    T, A = oracle.Cloud(scene.terrain), oracle.Cloud(aux)
    with _abi.Context(0) as ctx:
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.set_aux_cloud(aux, point_step=32)
        ctx.set_cells(cells.xyz, cells.normals)
        poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)[:npose]
        assert (npose + 1) * cells.xyz.shape[0] <= 1 << 15   # the wide kernel's range
        fg = np.zeros(cells.xyz.shape[0], np.uint8)
        fr = fg.copy()
        tot, cov, rep = ctx.score_poses(poses, scene.zx120_pose5, params, fg)
        r_tot, r_cov, r_rep = oracle.score_poses(T, A, cells.xyz, cells.normals, poses,
                                                 scene.zx120_pose5, oracle.vl_params(), fr)
        np.testing.assert_array_equal(fg, fr)
        np.testing.assert_array_equal(cov, r_cov)
        assert _rel_close(tot, r_tot), np.max(np.abs(tot - r_tot))
        assert rep.best_idx == r_rep.best_idx
        assert rep.as_dict()["total_cells"] == r_rep.as_dict()["total_cells"]


def test_generate_and_score_matches_two_calls(gpu, loaded, scene, cells):
    """pcp_generate_and_score (one round trip: the scoring reads the candidates and their count
    where the generation left them) against pcp_generate_candidates + pcp_score_poses on the
    same context: poses, totals, covered counts, flags and the report bit-identical over ticks
    whose flags carry over, lattice sizes that change between calls, and a context without
    cells."""
    fa = np.zeros(cells.xyz.shape[0], np.uint8)
    fb = fa.copy()
    for nc in (None, 400, 100, None):
        params = _abi.default_vl_params() if nc is None else _abi.default_vl_params(num_candidates=nc)
        poses = gpu.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
        tot, cov, rep = gpu.score_poses(poses, scene.zx120_pose5, params, fa)
        p2, tot2, cov2, rep2 = gpu.generate_and_score(cells.grid_bbox, params, scene.zx120_pose5, fb)
        np.testing.assert_array_equal(p2, poses)
        np.testing.assert_array_equal(tot2.view(np.uint64), tot.view(np.uint64))
        np.testing.assert_array_equal(cov2, cov)
        np.testing.assert_array_equal(fb, fa)
        assert rep2.as_dict() == rep.as_dict()
    with _abi.Context(0) as ctx:   # no cells, no terrain: the zeroed report, flat candidates
        params = _abi.default_vl_params(num_candidates=9)
        f0 = np.zeros(0, np.uint8)
        poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
        tot, cov, rep = ctx.score_poses(poses, scene.zx120_pose5, params, f0)
        p2, tot2, cov2, rep2 = ctx.generate_and_score(cells.grid_bbox, params, scene.zx120_pose5, f0)
        np.testing.assert_array_equal(p2, poses)
        np.testing.assert_array_equal(tot2, tot)
        assert rep2.as_dict() == rep.as_dict()


def test_score_fov_boundary(oracle):
    """The FOV decision (virtual_lidar.cpp:665-672, |elevation - pitch| <= fov / 2) at and around
    its boundary: cells straight below and above a pose (elevation exactly -pi/2, +pi/2) and a
    hair off the vertical, pitches 0, +-1e-7, +-3e-6 (inside the band the kernel settles with
    the double atan2) and +-2e-5, +-1e-3 (settled by its float atan2).  No terrain: every cell
    in range and in view is visible, so the flags carry the FOV bits.  Flags, covered counts
    and totals against the oracle."""
    xyz = np.array([[0.0, 0.0, 0.0], [0.0, 0.0, 4.0], [1e-6, 0.0, 0.0], [0.0, -1e-4, 0.0],
                    [0.01, 0.0, 0.0], [0.0, 0.0, 0.5], [3.0, 0.0, 2.0], [0.0, 1e-7, 4.0],
                    [-2.0, 1.0, -3.0]])
    nrm = np.tile(np.array([[0.0, 0.0, 1.0]], np.float32), (xyz.shape[0], 1))
    pitches = [0.0, 1e-7, -1e-7, 3e-6, -3e-6, 2e-5, -2e-5, 1e-3, -1e-3]
    poses = np.array([[0.0, 0.0, 2.0, pt, 0.4] for pt in pitches])
    zx = np.array([0.0, 0.0, 2.0, 1e-7, 0.0])
    params = _abi.default_vl_params()
    with _abi.Context(0) as ctx:
        ctx.set_cells(xyz, nrm)
        fg = np.zeros(xyz.shape[0], np.uint8)
        fr = fg.copy()
        for tick in range(2):   # each pose alone: the flags show every pose's own bits
            for k in range(len(pitches)):
                tot, cov, rep = ctx.score_poses(poses[k:k + 1].copy(), zx, params, fg)
                r_tot, r_cov, r_rep = oracle.score_poses(None, None, xyz, nrm, poses[k:k + 1],
                                                         zx, oracle.vl_params(), fr)
                np.testing.assert_array_equal(fg, fr)
                np.testing.assert_array_equal(cov, r_cov)
                assert _rel_close(tot, r_tot)
                assert rep.green == r_rep.green and rep.yellow == r_rep.yellow
    # both sides of the boundary occur (the same double expression, in numpy)
    d = xyz[None, :, :] - poses[:, None, :3]
    L = np.linalg.norm(d, axis=2)
    ediff = np.arctan2(d[..., 2], np.hypot(d[..., 0], d[..., 1])) - poses[:, 3:4]
    fov = np.abs(ediff) <= (180.0 * np.pi / 180.0) / 2.0
    inr = (L >= 0.5) & (L <= params.max_distance)
    assert (inr & fov).any() and (inr & ~fov).any()


def test_score_poses_clutter(oracle):
    """Reference-mode scoring against the volumetric cloud: visibility marches that end at the
    cell (s_k < L - 0.08), cells inside the clutter, behind the wall and in the open."""
    cloud = _clutter_cloud(23)
    rng = np.random.default_rng(5)
    xyz = np.c_[rng.uniform(-5, 5, (400, 2)), rng.uniform(-1, 1.5, 400)]
    nrm = rng.normal(size=(400, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    ctx = _abi.Context(0)
    try:
        ctx.set_terrain(cloud)
        ctx.set_cells(xyz, nrm)
        params = _abi.default_vl_params()
        poses = np.array([[0.0, 0.0, 2.5, -0.6, 0.0], [-4.0, -4.0, 1.0, -0.2, 0.8],
                          [4.5, 0.0, 0.5, 0.0, 3.1], [0.0, 5.0, 3.0, -1.2, -1.57]])
        zx = np.array([-5.0, 5.0, 2.0, -0.5, -0.7])
        flags_g = np.zeros(400, np.uint8)
        flags_r = flags_g.copy()
        tot, cov, rep = ctx.score_poses(poses, zx, params, flags_g)
        T = oracle.Cloud(cloud)
        r_tot, r_cov, r_rep = oracle.score_poses(T, None, xyz, nrm, poses, zx, oracle.vl_params(),
                                                 flags_r)
        np.testing.assert_array_equal(flags_g, flags_r)
        np.testing.assert_array_equal(cov, r_cov)
        assert _rel_close(tot, r_tot)
        assert rep.best_idx == r_rep.best_idx
        assert 0 < cov.min() and cov.max() < 400
    finally:
        ctx.close()


def test_score_poses_sparse_terrain(oracle):
    """A sparse terrain (a few thousand points over 40 m x 40 m, like the chain's carved
    terrain) takes the sparse z-band build and the coarse occupancy map that the cell march
    reads from LDS before each probe: flags and covered counts exact, totals within the parity bar,
    against the oracle.  Pillars between the poses and the cells make some rays blocked."""
    rng = np.random.default_rng(11)
    ground = np.c_[rng.uniform(-20, 20, (2_500, 2)), rng.normal(0.0, 0.05, 2_500)]
    pillars = [np.c_[x + rng.normal(0, 0.05, 300), y + rng.normal(0, 0.05, 300),
                     rng.uniform(0.0, 3.0, 300)] for x, y in ((3.0, 2.0), (-4.0, 5.0), (6.0, -6.0),
                                                            (0.5, 0.5))]
    pts = np.concatenate([ground] + pillars).astype(np.float32)
    cloud = np.zeros((pts.shape[0], 4), np.float32)
    cloud[:, :3] = pts
    xyz = np.c_[rng.uniform(-8, 8, (400, 2)), rng.uniform(-0.3, 0.6, 400)]
    nrm = rng.normal(size=(400, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    poses = np.array([[0.0, 0.0, 2.5, -0.6, 0.0], [-6.0, -6.0, 1.5, -0.3, 0.8],
                      [7.0, 1.0, 3.0, -0.9, 3.1], [1.0, 7.0, 1.2, 0.0, -1.57]])
    zx = np.array([-9.0, 9.0, 2.0, -0.5, -0.7])
    params = _abi.default_vl_params()
    with _abi.Context(0) as ctx:
        ctx.set_terrain(cloud)
        ctx.set_cells(xyz, nrm)
        fg = np.zeros(400, np.uint8)
        fr = fg.copy()
        T = oracle.Cloud(cloud)
        for tick in range(2):
            tot, cov, rep = ctx.score_poses(poses, zx, params, fg)
            r_tot, r_cov, r_rep = oracle.score_poses(T, None, xyz, nrm, poses, zx,
                                                     oracle.vl_params(), fr)
            np.testing.assert_array_equal(fg, fr)
            np.testing.assert_array_equal(cov, r_cov)
            assert _rel_close(tot, r_tot)
            assert rep.best_idx == r_rep.best_idx
        info = ctx.terrain_info()
        assert info["dims"][0] * info["dims"][1] * info["dims"][2] > 32 * cloud.shape[0]   # sparse
        assert cov.max() > 0


def test_score_poses_edge_states(oracle, scene, cells, aux):
    """No terrain (visible), no aux cloud, zero poses, zero cells, stale terrain tree."""
    params = _abi.default_vl_params(max_distance=12.0)
    zx = scene.zx120_pose5
    poses = np.array([[8.0, -3.0, 1.1, -0.3, 2.5], [0.0, 4.0, 1.1, -0.2, -1.0]])
    with _abi.Context(0) as ctx:
        # nothing loaded: every visibility check returns true (:721,:727)
        ctx.set_cells(cells.xyz, cells.normals)
        fg = np.zeros(cells.xyz.shape[0], np.uint8)
        fr = fg.copy()
        t, c, rep = ctx.score_poses(poses, zx, params, fg)
        rt, rc, rrep = oracle.score_poses(None, None, cells.xyz, cells.normals, poses, zx,
                                          oracle.vl_params(max_distance=12.0), fr)
        np.testing.assert_array_equal(fg, fr)
        np.testing.assert_array_equal(c, rc)
        assert _rel_close(t, rt)
        # zero poses: stats only, best -1
        t, c, rep = ctx.score_poses(np.zeros((0, 5)), zx, params, fg)
        assert rep.best_idx == -1 and t.size == 0 and rep.total_cells == cells.xyz.shape[0]
        # terrain then an empty terrain: ray casts keep the stale index, ground height sees
        # the empty cloud (0.0)
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.set_terrain(np.zeros((0, 8), np.float32), point_step=32)
        g = ctx.generate_candidates(cells.grid_bbox, params, zx)
        T = oracle.Cloud(scene.terrain)
        r = oracle.generate_candidates(T, cells.grid_bbox, oracle.vl_params(max_distance=12.0),
                                       zx, terrain_empty=True)
        np.testing.assert_array_equal(g[:, :3], r[:, :3])
        fg[:] = 0
        fr[:] = 0
        t, c, rep = ctx.score_poses(poses, zx, params, fg)
        rt, rc, rrep = oracle.score_poses(T, None, cells.xyz, cells.normals, poses, zx,
                                          oracle.vl_params(max_distance=12.0), fr)
        np.testing.assert_array_equal(fg, fr)
        np.testing.assert_array_equal(c, rc)
        # zero cells
        ctx.set_cells(np.zeros((0, 3)), np.zeros((0, 3), np.float32))
        t, c, rep = ctx.score_poses(poses, zx, params, np.zeros(0, np.uint8))
        assert rep.best_idx == 0 and np.all(t == 0)


# ---------------------------------------------------------------- excavation-area setup
def _normals_equal(got, ref):
    """Bit-identical normals, NaN where the reference has NaN (< 3 neighbours, non-finite)."""
    fin = np.isfinite(ref).all(1)
    assert np.array_equal(np.isfinite(got).all(1), fin)
    np.testing.assert_array_equal(got[fin].view(np.uint32), ref[fin].view(np.uint32))


@pytest.mark.parametrize("mode", ["exact", "exact_ordered", "exact_two_builds", "fixed"])
def test_excavation_area_setup(oracle, scene, mode, monkeypatch):
    """pcp_set_excavation_area against the oracle: grid bounds and the valid cells (positions,
    reference loop order) bit-exact.  Default path (PCP_NORMALS_EXACT=1): point normals and cell
    normals BIT-IDENTICAL -- PCL's float covariance sums in FLANN's (distance, index) order,
    eigen33 with glibc's float libm restated (pcp_libm.h), the cells' double sums where their
    order cannot change them in any order (k_cell_sums_exact), the others in FLANN's order;
    exact_ordered (PCP_CELLS_ORDER_FREE=0) sends every cell through the ordered lists;
    exact_two_builds builds the area's two grids separately (PCP_INDEX_PAIR=0).  The
    order-free fixed-point A/B kernels (PCP_NORMALS_EXACT=0): point normals within 2e-3, cells
    within 1e-4.  An empty area keeps the previous cells (virtual_lidar.cpp:168)."""
    exact = "0" if mode == "fixed" else "1"
    monkeypatch.setenv("PCP_NORMALS_EXACT", exact)
    # exact_two_builds: the area's two grids by two build_index calls + k_area_prep instead of
    # the paired build (PCP_INDEX_PAIR=0)
    monkeypatch.setenv("PCP_INDEX_PAIR", "0" if mode == "exact_two_builds" else "1")
    monkeypatch.setenv("PCP_CELLS_ORDER_FREE", "0" if mode == "exact_ordered" else "1")
    d = np.load(GOLD / "excavation.npz")
    ctx = _abi.Context(0)
    try:
        for area, ref in ((d["area"], None), (scene.area, "full")):
            if ref is None:
                r_n, r_xyz, r_cn, r_bb = d["normals"], d["cells"], d["cell_normals"], d["grid_bbox"]
            else:
                r_n = oracle.area_normals(area, 1.5)
                r_xyz, r_cn, r_bb, _ = oracle.excavation_grid(area, 0.1, 10, r_n)
            bb, n = ctx.set_excavation_area(area, 0.1, 10, point_step=area.shape[1] * 4)
            np.testing.assert_array_equal(bb, r_bb)
            assert n == r_xyz.shape[0]
            xyz, cn = ctx.get_cells()
            np.testing.assert_array_equal(xyz, r_xyz)
            an = ctx.get_area_normals()
            if exact == "1":
                _normals_equal(an, r_n)
                np.testing.assert_array_equal(cn.view(np.uint32), r_cn.view(np.uint32))
            else:
                fin = np.isfinite(r_n).all(1)
                assert np.array_equal(np.isfinite(an).all(1), fin)
                np.testing.assert_allclose(an[fin], r_n[fin], atol=2e-3)
                np.testing.assert_allclose(cn, r_cn, atol=1e-4)
        bb, n2 = ctx.set_excavation_area(np.zeros((0, 4), np.float32), 0.1, 10)
        assert n2 == n and np.array_equal(ctx.get_cells()[0], xyz)
    finally:
        ctx.close()


@pytest.mark.parametrize("order_free,small", [("1", "1"), ("0", "1"), ("1", "0")])
def test_excavation_area_normals_long_lists_and_ties(oracle, order_free, small, monkeypatch):
    """The exact normals where the neighbour lists pass the LDS sort (> 4,096 neighbours within
    1.5 m: sorted in global memory), with exact distance ties (a lattice, duplicated points: the
    reference's order breaks them by index), non-finite points (NaN normals, absent from every
    list) and isolated points (< 3 neighbours: NaN).  A plane tilted by 1e-6 beside it gives
    normals with components ~2^-20 of their largest: the cells near it fail
    k_cell_sums_exact's bound and take the ordered path in the same frame as the others.
    Point and cell normals bit-identical, cells order-free where exact (default) and all
    ordered (PCP_CELLS_ORDER_FREE=0); the lists' LDS keys with 16-bit indices (areas below 2^16
    points, default) and 32-bit (PCP_NB_SMALL=0, every larger area)."""
    monkeypatch.setenv("PCP_CELLS_ORDER_FREE", order_free)
    monkeypatch.setenv("PCP_NB_SMALL", small)
    rng = np.random.default_rng(11)
    g = np.arange(90) * 0.025
    X, Y = np.meshgrid(g, g)
    P = np.stack([X.ravel(), Y.ravel(), 0.3 * np.sin(X.ravel()) + rng.normal(0, 0.002, X.size)], 1)
    P[::7, 2] = np.round(P[::7, 2], 2)                        # many exact-distance ties
    t = np.arange(30) * 0.05
    TX, TY = np.meshgrid(4.0 + t, t)
    tilt = np.stack([TX.ravel(), TY.ravel(), 1e-6 * TX.ravel()], 1)   # tiny normal components
    P = np.concatenate([P, P[100:140], tilt, [[9.0, 9.0, 0.0], [9.5, 9.0, 0.1]]])   # dups, isolated
    a = np.zeros((P.shape[0], 4), np.float32)
    a[:, :3] = P
    a[rng.integers(0, a.shape[0], 6), 1] = np.nan
    r_n = oracle.area_normals(a, 1.5)
    r_xyz, r_cn, r_bb, _ = oracle.excavation_grid(a, 0.1, 4, r_n)
    with _abi.Context(0) as ctx:
        for _ in range(2):                                   # the regrown list buffer, reused
            bb, n = ctx.set_excavation_area(a, 0.1, 4)
            np.testing.assert_array_equal(bb, r_bb)
            assert n == r_xyz.shape[0]
            _normals_equal(ctx.get_area_normals(), r_n)
            xyz, cn = ctx.get_cells()
            np.testing.assert_array_equal(xyz, r_xyz)
            np.testing.assert_array_equal(cn.view(np.uint32), r_cn.view(np.uint32))


@pytest.mark.parametrize("region_pct,guess", [("10", None), ("100", "4096"), ("10", "4096"),
                                              ("75", "4096")])
def test_excavation_area_list_spill_pool(oracle, region_pct, guess, monkeypatch):
    """The neighbour lists' capacity paths (k_nb_lists): a list its block's region cannot hold
    spills to the shared pool behind the regions (PCP_NB_REGION_PCT=10: most lists spill), and a
    list that fits neither sets the overflow, after which the host regrows both buffers and runs
    the normals again (PCP_NB_GUESS_WORDS=4096: a first buffer far too small; 100: no pool, the
    regions alone).  Point and cell normals bit-identical to the oracle on every path, and the
    second setup of the same area reallocates nothing."""
    monkeypatch.setenv("PCP_NB_REGION_PCT", region_pct)
    if guess:
        monkeypatch.setenv("PCP_NB_GUESS_WORDS", guess)
    a = _long_list_area()
    r_n = oracle.area_normals(a, 1.5)
    r_xyz, r_cn, r_bb, _ = oracle.excavation_grid(a, 0.1, 4, r_n)
    with _abi.Context(0) as ctx:
        for rep in range(2):
            before = _abi.alloc_stats()["device"]
            bb, n = ctx.set_excavation_area(a, 0.1, 4)
            grew = _abi.alloc_stats()["device"] - before
            np.testing.assert_array_equal(bb, r_bb)
            assert n == r_xyz.shape[0]
            _normals_equal(ctx.get_area_normals(), r_n)
            xyz, cn = ctx.get_cells()
            np.testing.assert_array_equal(xyz, r_xyz)
            np.testing.assert_array_equal(cn.view(np.uint32), r_cn.view(np.uint32))
            if rep:
                assert grew == 0, grew


def _long_list_area():
    rng = np.random.default_rng(11)
    g = np.arange(90) * 0.025
    X, Y = np.meshgrid(g, g)
    P = np.stack([X.ravel(), Y.ravel(), 0.3 * np.sin(X.ravel()) + rng.normal(0, 0.002, X.size)], 1)
    P[::7, 2] = np.round(P[::7, 2], 2)
    a = np.zeros((P.shape[0], 4), np.float32)
    a[:, :3] = P
    return a


@pytest.mark.parametrize("which,guess", [("golden", None), ("long_lists", None),
                                         ("long_lists", "4096"), ("golden", "4096")])
def test_excavation_area_async_then_tick(oracle, scene, which, guess, monkeypatch):
    """pcp_set_excavation_area_async (the composed chain's grid setup: enqueued, not waited for)
    followed by the terrain and the tick (pcp_generate_and_score, which settles it after its own
    synchronisation -- and, on a fresh context whose first neighbour-list guess overflows, regrows
    the lists, reruns them and ticks again): poses, totals, covered counts, flags, the report and
    the cells bit-identical to the synchronous setup's; a second tick from the stale flags too;
    an async setup settled by pcp_get_cells gives the same cells.  PCP_NB_GUESS_WORDS=4096: the
    first list buffers far too small, so the tick finds the overflow after its wait (the setup
    ran on its side stream), regrows, reruns the normals and ticks again."""
    if guess:
        monkeypatch.setenv("PCP_NB_GUESS_WORDS", guess)
    area = np.load(GOLD / "excavation.npz")["area"] if which == "golden" else _long_list_area()
    params = _abi.default_vl_params(num_candidates=36)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    out = {}
    for mode in ("sync", "async"):
        with _abi.Context(0) as ctx:
            ctx.set_terrain(scene.terrain, point_step=32)
            if mode == "sync":
                bb, n = ctx.set_excavation_area(area, 0.1, 10, point_step=area.shape[1] * 4)
                flags = np.zeros(max(n, 1), np.uint8)
            else:
                bb, cap = ctx.set_excavation_area_async(area, 0.1, 10, point_step=area.shape[1] * 4)
                flags = np.zeros(max(cap, 1), np.uint8)
            poses, tot, cov, rep = ctx.generate_and_score(bb, params, zx, flags)
            n = ctx.cells_count()
            fl1 = flags[:n].copy()
            poses2, tot2, cov2, rep2 = ctx.generate_and_score(bb, params, zx, fl1)
            xyz, cn = ctx.get_cells()
            out[mode] = (bb, n, poses, tot, cov, rep.as_dict(), fl1, tot2, rep2.as_dict(), xyz, cn)
            if mode == "async":   # an async setup settled by a reader of the cells
                ctx.set_excavation_area_async(area, 0.1, 10, point_step=area.shape[1] * 4)
                xyz3, cn3 = ctx.get_cells()
                np.testing.assert_array_equal(xyz3, xyz)
                np.testing.assert_array_equal(cn3.view(np.uint32), cn.view(np.uint32))
    a, b = out["sync"], out["async"]
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1] == b[1] and a[1] > 0
    for i in (2, 3, 4, 6, 7, 9):
        np.testing.assert_array_equal(np.asarray(a[i]).view(np.uint8), np.asarray(b[i]).view(np.uint8))
    np.testing.assert_array_equal(a[10].view(np.uint32), b[10].view(np.uint32))
    assert a[5] == b[5] and a[8] == b[8]


def test_excavate_area_async_matches_three_calls():
    """pcp_excavate_area_async (the carve node and virtual_lidar's area + terrain callbacks
    composed: the carve's landed records feed the grid setup and the terrain index in place)
    against pcp_excavate + pcp_set_excavation_area + pcp_set_terrain on the same merged cloud:
    both messages, the pose, the grid bounds, the cells and their normals, and a tick's poses,
    totals, covered counts, flags and report bit-identical.  Three frames in a row on one
    context (the landing is reused while the previous setup is pending: the call settles it
    first), the third with the carve moved (a new generated lattice).  "landed": the composed
    call with null outputs, the messages read in place (pcp_excavate_landed) after the zx120
    index and the tick -- the same bytes."""
    box = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])
    tfs = [((8.0, -3.0, 2.0), (0.0, 0.0, 0.2588190451025208, 0.9659258262890683)),
           ((0.55, 0.4, 3.5), (0.0, 0.21633, 0.0, 0.97632))]
    params = _abi.default_vl_params(num_candidates=36)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    frames = []
    for f, (seed, base) in enumerate([(101, ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))),
                                      (131, ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))),
                                      (131, ((0.3, -0.2, 0.0), (0.0, 0.0, 0.0998, 0.9950)))]):
        scans = [synth.lidar_cloud(60_032, sensor_height=2.0, seed=seed),
                 synth.lidar_cloud(60_032, sensor_height=3.5, seed=seed + 1)]
        frames.append((scans, base))
    out = {}
    for mode in ("calls", "composed", "landed"):
        res = []
        with _abi.Context(0) as ctx:
            for scans, base in frames:
                filt = [ctx.crop_voxel(sc, box, 0.2)[0] for sc in scans]
                merged = ctx.transform_concat(filt, tfs, [(255, 0, 0), (0, 0, 255)])
                if mode == "calls":
                    terr, area, pose = ctx.excavate(merged, base)
                    bb, n = ctx.set_excavation_area_async(area, 0.1, 10, point_step=32)
                    ctx.set_terrain(terr, point_step=32)
                else:
                    terr, area, pose, bb, n = ctx.excavate_area_async(merged, base,
                                                                      landed=mode == "landed")
                    tp = ctypes.c_void_p()
                    rc = ctx.lib.pcp_excavate_landed(ctx.h, ctypes.byref(tp), None)
                    # left in place only by the null-output call
                    assert (rc == _abi.PCP_OK) == (mode == "landed"), rc
                ctx.set_aux_cloud(filt[1])
                flags = np.zeros(max(n, 1), np.uint8)
                poses, tot, cov, rep = ctx.generate_and_score(bb, params, zx, flags)
                nc = ctx.cells_count()
                xyz, cn = ctx.get_cells()
                res.append((terr.copy(), area.copy(), pose, bb, nc, poses, tot, cov, flags[:nc].copy(),
                            rep.as_dict(), xyz, cn))
        out[mode] = res
    for a, b, c in zip(out["calls"], out["composed"], out["landed"]):
        for i in (0, 1, 2, 3, 5, 6, 7, 8, 10, 11):
            np.testing.assert_array_equal(np.asarray(a[i]).view(np.uint8), np.asarray(b[i]).view(np.uint8))
            np.testing.assert_array_equal(np.asarray(a[i]).view(np.uint8), np.asarray(c[i]).view(np.uint8))
        assert a[4] == b[4] == c[4] and a[4] > 0
        assert a[9] == b[9] == c[9]


def test_excavation_area_async_back_to_back(scene):
    """Async grid setups in a row with no tick between them (each settles the one before it:
    its side stream joined, its lists checked), a terrain change and a zx120 cloud between
    setup and tick, then the tick: cells, normals, poses, totals, flags and report equal to a
    context that ran only the last setup synchronously."""
    d = np.load(GOLD / "excavation.npz")
    areas = [_long_list_area(), d["area"], _long_list_area()[::3].copy()]
    params = _abi.default_vl_params(num_candidates=25)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    aux = scene.terrain[::50, :4].copy()
    out = []
    for mode in ("sync_last", "async_chain"):
        with _abi.Context(0) as ctx:
            ctx.set_terrain(scene.terrain[:1000], point_step=32)
            if mode == "sync_last":
                ctx.set_terrain(scene.terrain, point_step=32)
                bb, n = ctx.set_excavation_area(areas[-1], 0.1, 10, point_step=areas[-1].shape[1] * 4)
                flags = np.zeros(max(n, 1), np.uint8)
            else:
                for a in areas:
                    bb, cap = ctx.set_excavation_area_async(a, 0.1, 10, point_step=a.shape[1] * 4)
                ctx.set_terrain(scene.terrain, point_step=32)
                flags = np.zeros(max(cap, 1), np.uint8)
            ctx.set_aux_cloud(aux)
            poses, tot, cov, rep = ctx.generate_and_score(bb, params, zx, flags)
            n = ctx.cells_count()
            xyz, cn = ctx.get_cells()
            out.append((bb, n, poses, tot, cov, flags[:n].copy(), rep.as_dict(), xyz, cn))
    a, b = out
    assert a[1] == b[1] and a[1] > 0 and a[6] == b[6]
    for i in (0, 2, 3, 4, 5, 7, 8):
        np.testing.assert_array_equal(np.asarray(a[i]).view(np.uint8), np.asarray(b[i]).view(np.uint8))


def _degenerate_areas():
    rng = np.random.default_rng(23)
    out = {}
    out["three_points"] = np.array([[0.0, 0.0, 0.0], [0.1, 0.0, 0.0], [0.0, 0.1, 0.01]])
    out["identical"] = np.concatenate([np.tile([[1.0, 2.0, 0.5]], (50, 1)),
                                       rng.uniform(0, 0.4, (30, 3)) + [1.0, 2.0, 0.3]])
    t = np.arange(200) * 0.01
    out["collinear"] = np.stack([t, 0.5 * t, 0.1 * t], 1)                 # rank-1 covariance
    g = np.arange(40) * 0.05
    X, Y = np.meshgrid(g, g)
    plane = np.stack([X.ravel(), Y.ravel(), 0.2 * X.ravel() + rng.normal(0, 0.003, X.size)], 1)
    out["far_from_origin"] = plane + [2000.0, -1500.0, 300.0]            # float spacing ~1e-4 m
    return out


@pytest.mark.parametrize("case", ["three_points", "identical", "collinear", "far_from_origin"])
def test_excavation_area_normals_degenerate(oracle, case):
    """Degenerate areas through the exact normals: three points (lists below PCL's minimum),
    50 identical points beside a few others (zero distances: the order is the index order, zero
    covariance), a line (rank-1 covariance: eigen33's degenerate branches), and a plane
    kilometres from the origin (coarse float spacing in the distances and the sums).  Point and
    cell normals and the cells bit-identical to the oracle."""
    P = _degenerate_areas()[case]
    a = np.zeros((P.shape[0], 4), np.float32)
    a[:, :3] = P
    r_n = oracle.area_normals(a, 1.5)
    r_xyz, r_cn, r_bb, _ = oracle.excavation_grid(a, 0.1, 4, r_n)
    with _abi.Context(0) as ctx:
        bb, n = ctx.set_excavation_area(a, 0.1, 4)
        np.testing.assert_array_equal(bb, r_bb)
        assert n == r_xyz.shape[0]
        _normals_equal(ctx.get_area_normals(), r_n)
        if n:
            xyz, cn = ctx.get_cells()
            np.testing.assert_array_equal(xyz, r_xyz)
            np.testing.assert_array_equal(cn.view(np.uint32), r_cn.view(np.uint32))


# ---------------------------------------------------------------- excavated-terrain carve
def _matched_cloud(seed=3):
    """A /matched_point_cloud stand-in: a noisy 0.05 m lattice (PointXYZRGB, 32 B), a raised
    block over the pit, a hole with a few points 0.8 m up (nearest-point fallbacks), NaNs."""
    rng = np.random.default_rng(seed)
    xs, ys = np.arange(-2.0, 9.0, 0.05), np.arange(-3.0, 6.0, 0.05)
    X, Y = np.meshgrid(xs, ys)
    P = np.stack([X.ravel(), Y.ravel(), rng.normal(0, 0.01, X.size)], 1)
    hole = np.hypot(P[:, 0] - 5.0, P[:, 1] - 0.0) < 0.8
    P = P[~hole]
    block = np.stack(np.meshgrid(np.arange(4.0, 4.6, 0.05), np.arange(1.0, 1.6, 0.05),
                                 np.array([0.3, 1.5])), -1).reshape(-1, 3)
    lifted = np.array([[5.0, 0.0, 0.8], [5.1, 0.2, 0.8], [4.8, -0.3, 0.85]])
    P = np.concatenate([P, block, lifted])
    c = np.zeros((P.shape[0], 8), np.float32)
    c[:, :3] = P
    c[:, 4] = np.frombuffer(np.full(P.shape[0], 0xFF00FF00, np.uint32).tobytes(), np.float32)
    c[rng.integers(0, P.shape[0], 20), 0] = np.nan
    return c


def test_excavate_matches_oracle(gpu, oracle):
    """pcp_excavate against the CPU restatement: kept points (order, bytes), the generated
    excavated surface and /excavation_area records, and the marker pose, all bit-exact.  The
    sequence covers the device copy of the generated lattice: reused for a new cloud under the
    same pose, regenerated for a new pose, and for a cloud that outgrows its buffer."""
    for seed, yaw_deg, twice in ((3, 20.0, False), (4, 20.0, False), (3, -35.0, False),
                                 (7, -35.0, True), (3, 20.0, False)):
        c = _matched_cloud(seed)
        if twice:
            c = np.concatenate([c, _matched_cloud(seed + 1)])
        yaw = math.radians(yaw_deg)
        t, q = (0.3, -0.2, 0.1), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))
        terr, area, pose = gpu.excavate(c, (t, q))
        keep, surf, r_area, r_pose = oracle.excavate(c, t, q)
        np.testing.assert_array_equal(pose, r_pose)
        nk = int(keep.sum())
        assert 0 < nk < c.shape[0] and terr.shape[0] == nk + surf.shape[0]
        kept = c[keep]
        np.testing.assert_array_equal(terr[:nk, :3].view(np.uint32), kept[:, :3].view(np.uint32))
        np.testing.assert_array_equal(terr[:nk, 4].view(np.uint32), kept[:, 4].view(np.uint32))
        np.testing.assert_array_equal(terr[nk:, [0, 1, 2, 4]].view(np.uint32), surf.view(np.uint32))
        np.testing.assert_array_equal(area[:, [0, 1, 2, 4]].view(np.uint32), r_area.view(np.uint32))


@pytest.mark.parametrize("case", ["empty", "all_nan", "far", "rect", "dense_deep"])
def test_excavate_edge_cases(gpu, oracle, case):
    """pcp_excavate against the CPU restatement on the edges: an empty cloud, an all-NaN cloud,
    a cloud 200 m away from the pit (every height from the nearest-point fallback), the
    rectangle mode (l_shape_enabled 0) and a denser, deeper surface (point_density 0.1, depth
    0.5).  Kept points, generated surface, /excavation_area records and the marker pose
    bit-exact."""
    c = _matched_cloud(6)
    kw = {}
    if case == "empty":
        c = np.zeros((0, 8), np.float32)
    elif case == "all_nan":
        c[:, 0] = np.nan
    elif case == "far":
        c[:, 0] += 200.0
    elif case == "rect":
        kw = {"l_shape_enabled": 0}
    else:
        kw = {"point_density": 0.1, "depth": 0.5}
    yaw = math.radians(15.0)
    t, q = (0.3, -0.2, 0.1), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))
    terr, area, pose = gpu.excavate(c, (t, q), _abi.excavation_params(**kw))
    keep, surf, r_area, r_pose = oracle.excavate(c, t, q, oracle.exc_params(**kw))
    np.testing.assert_array_equal(pose, r_pose)
    nk = int(keep.sum())
    assert terr.shape[0] == nk + surf.shape[0]
    kept = c[keep]
    np.testing.assert_array_equal(terr[:nk, :3].view(np.uint32), kept[:, :3].view(np.uint32))
    np.testing.assert_array_equal(terr[:nk, 4].view(np.uint32), kept[:, 4].view(np.uint32))
    np.testing.assert_array_equal(terr[nk:, [0, 1, 2, 4]].view(np.uint32), surf.view(np.uint32))
    np.testing.assert_array_equal(area[:, [0, 1, 2, 4]].view(np.uint32), r_area.view(np.uint32))


def test_excavate_bounds_hold(gpu):
    """pcp_excavate_bounds caps every output the carve can produce (rectangle and L modes)."""
    c = _matched_cloud(5)
    for kw in ({}, {"l_shape_enabled": 0}, {"point_density": 0.1, "depth": 0.5}):
        p = _abi.excavation_params(**kw)
        terr, area, _ = gpu.excavate(c, ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0)), p)
        nt, na = C_u64(), C_u64()
        assert gpu.lib.pcp_excavate_bounds(C_ref(p), c.shape[0], C_ref(nt), C_ref(na)) == 0
        assert terr.shape[0] <= nt.value and area.shape[0] <= na.value


# ---------------------------------------------------------------- drivable-area grid
@pytest.mark.parametrize("kw", [{}, {"grid_resolution": 0.5, "map_width": 60.0, "map_height": 40.0,
                                     "min_points_per_cell": 3, "max_gradient": 0.2}])
def test_drivable_area_matches_oracle(gpu, oracle, kw):
    """calc_drivable_area (robotCloudCallback :67-226) against the CPU restatement: the int8
    occupancy grid and its origin bit-exact (start-clear disc, unknown, obstacle, free)."""
    rng = np.random.default_rng(11)
    n = 200_000
    c = np.zeros((n, 4), np.float32)
    c[:, 0] = rng.uniform(-45, 45, n)
    c[:, 1] = rng.uniform(-45, 45, n)
    c[:, 2] = rng.normal(-1.5, 0.05, n)
    steep = (c[:, 0] > 5) & (c[:, 0] < 15)
    c[steep, 2] += rng.uniform(0, 1.5, steep.sum())
    c[rng.integers(0, n, 50), 1] = np.nan
    yaw = math.radians(25.0)
    t, q = (3.0, -2.0, 1.8), (0.0, 0.05, math.sin(yaw / 2), math.cos(yaw / 2))
    p = _abi.drivable_params(**kw)
    grid, origin = gpu.drivable_area(c, (t, q), (3.0, -2.0), (1.0, 0.5), p)
    ref, r_origin = oracle.drivable_area(c, t, q, (3.0, -2.0), (1.0, 0.5), p.grid_resolution,
                                         p.map_width, p.map_height, p.max_gradient,
                                         p.min_points_per_cell, p.start_clear_radius)
    np.testing.assert_array_equal(origin, r_origin)
    np.testing.assert_array_equal(grid, ref)
    assert {-1, 0, 100} <= set(np.unique(grid).tolist())


@pytest.mark.parametrize("case", ["empty", "all_nan", "outside_map", "one_cell"])
def test_drivable_area_edge_cases(gpu, oracle, case):
    """calc_drivable_area on the edges: an empty cloud and an all-NaN one (only the start-clear
    disc is free; an empty cloud leaves the whole grid free, as the reference's), every point
    outside the map, and one column of points (a single cell, an obstacle by its z spread).
    Grid and origin bit-exact against the CPU restatement."""
    rng = np.random.default_rng(5)
    if case == "empty":
        c = np.zeros((0, 4), np.float32)
    else:
        n = 5_000
        c = np.zeros((n, 4), np.float32)
        c[:, 0] = rng.uniform(-2, 2, n)
        c[:, 1] = rng.uniform(-2, 2, n)
        c[:, 2] = rng.normal(-1.5, 0.05, n)
        if case == "all_nan":
            c[:, 0] = np.nan
        elif case == "outside_map":
            c[:, 0] += 500.0
        else:
            c[:, 0] = 4.0
            c[:, 1] = 6.0
    yaw = math.radians(-40.0)
    t, q = (1.0, 2.0, 1.8), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))
    p = _abi.drivable_params(min_points_per_cell=3)
    grid, origin = gpu.drivable_area(c, (t, q), (1.0, 2.0), (0.0, 0.0), p)
    ref, r_origin = oracle.drivable_area(c, t, q, (1.0, 2.0), (0.0, 0.0), p.grid_resolution,
                                         p.map_width, p.map_height, p.max_gradient,
                                         p.min_points_per_cell, p.start_clear_radius)
    np.testing.assert_array_equal(origin, r_origin)
    np.testing.assert_array_equal(grid, ref)


# (PCP_TERRAIN_BLOCKS, PCP_TERRAIN_FINE) -> the layout the scans walk from the first query
# (PCP_TERRAIN_BLOCKS, PCP_TERRAIN_FINE, PCP_FINE_TILE, expected scan layout); fine tile 0:
# x-fastest 8-byte records, 1: 4 x 4 tiles of them, 2: split records (2-byte thresholds +
# 4-byte starts) in 8 x 8 tiles
# (the fine-window entries are 12-byte packed unless the tile field carries "u": PCP_FINE_PACK=0)
LAYOUTS = [("0", "3", "1", "cells"), ("2", "0", "1", "blocks"), ("2", "2", "1", "fine"),
           ("2", "3", "1", "fine"), ("2", "2", "0", "fine"), ("2", "2", "2", "fine"),
           ("2", "3", "2", "fine"), ("2", "2", "2u", "fine")]


@pytest.mark.parametrize("mode,fine,tile,layout", LAYOUTS)
def test_terrain_block_copy_paths(oracle, scene, cells, aux, mode, fine, tile, layout,
                                  monkeypatch):
    """PCP_TERRAIN_BLOCKS=0 scans the per-cell runs, =2 the block-major copy (PCP_TERRAIN_FINE=0:
    2x2x2 blocks, F > 0: windows of fine cells c / F) from the first query on (the default, 1,
    switches at the second query): all bit-exact on the fan and the reference-mode scoring."""
    monkeypatch.setenv("PCP_TERRAIN_BLOCKS", mode)
    monkeypatch.setenv("PCP_TERRAIN_FINE", fine)
    monkeypatch.setenv("PCP_FINE_TILE", tile.rstrip("u"))
    monkeypatch.setenv("PCP_FINE_PACK", "0" if tile.endswith("u") else "1")
    ctx = _abi.Context(0)
    try:
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.set_aux_cloud(aux, point_step=32)
        ctx.set_cells(cells.xyz, cells.normals)
        T, A = oracle.Cloud(scene.terrain), oracle.Cloud(aux)
        params = _abi.default_vl_params()
        poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
        fan = _abi.fan_params(n_az=128, n_el=48)
        _, _, fh, _ = ctx.raycast_fan(poses[:5], fan, want_first_hit=True)
        assert ctx.terrain_info()["scan_layout"] == layout
        _, _, r_fh = oracle.raycast_fan(T, poses[:5], 128, 48, fan.el_min, fan.el_max,
                                        fan.max_distance)
        np.testing.assert_array_equal(fh, r_fh)
        flags_g = np.zeros(cells.xyz.shape[0], np.uint8)
        flags_r = flags_g.copy()
        tot, cov, rep = ctx.score_poses(poses, scene.zx120_pose5, params, flags_g)
        r_tot, r_cov, r_rep = oracle.score_poses(T, A, cells.xyz, cells.normals, poses,
                                                 scene.zx120_pose5, oracle.vl_params(), flags_r)
        np.testing.assert_array_equal(flags_g, flags_r)
        np.testing.assert_array_equal(cov, r_cov)
        assert _rel_close(tot, r_tot)
        assert rep.best_idx == r_rep.best_idx
    finally:
        ctx.close()


@pytest.mark.parametrize("mode,fine,tile,layout", LAYOUTS)
def test_terrain_block_copy_dense_and_tiny(oracle, mode, fine, tile, layout, monkeypatch):
    """Block-major copies on awkward terrains: 20 k points packed into a 0.3 m cube (blocks of
    thousands of points, ties in z) next to a sparse plane, and a one-point terrain."""
    monkeypatch.setenv("PCP_TERRAIN_BLOCKS", mode)
    monkeypatch.setenv("PCP_TERRAIN_FINE", fine)
    monkeypatch.setenv("PCP_FINE_TILE", tile.rstrip("u"))
    monkeypatch.setenv("PCP_FINE_PACK", "0" if tile.endswith("u") else "1")
    rng = np.random.default_rng(11)
    dense = np.column_stack([rng.uniform(2.0, 2.3, 20_000), rng.uniform(-0.15, 0.15, 20_000),
                             np.round(rng.uniform(0.0, 0.3, 20_000), 2)])
    gx, gy = np.meshgrid(np.arange(-3.0, 6.0, 0.07), np.arange(-3.0, 3.0, 0.07))
    plane = np.column_stack([gx.ravel(), gy.ravel(), rng.normal(-0.5, 0.01, gx.size)])
    poses = np.array([[0.0, 0.0, 1.0, -0.3, 0.0], [4.5, 0.5, 0.8, 0.0, np.pi],
                      [2.15, 0.0, 0.15, 0.0, 0.3], [-2.0, -2.0, 2.5, -0.8, 0.7]])
    fan = _abi.fan_params(n_az=96, n_el=40, el_min_deg=-80.0, el_max_deg=60.0, max_distance=9.0)
    for pts in (np.vstack([dense, plane]), np.array([[1.0, 0.2, 0.4]])):
        cloud = np.zeros((pts.shape[0], 8), np.float32)
        cloud[:, :3] = pts
        ctx = _abi.Context(0)
        try:
            ctx.set_terrain(cloud, point_step=32)
            for _ in range(2):   # mode 1 would switch paths between these two calls
                blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
                r_blocked, r_units, r_fh = oracle.raycast_fan(oracle.Cloud(cloud), poses, 96, 40,
                                                              fan.el_min, fan.el_max, 9.0)
                np.testing.assert_array_equal(fh, r_fh)
                np.testing.assert_array_equal(blocked, r_blocked)
                np.testing.assert_array_equal(units, r_units)
                assert ctx.terrain_info()["scan_layout"] == layout
        finally:
            ctx.close()


@pytest.mark.parametrize("skip", ["1", "2"])
def test_fine_copy_dense_window(oracle, monkeypatch, skip):
    """70,000 points in a 5 cm cube: fine windows of 70 k points (the walks end at the first
    point r below or at the window's sentinel, no stored count; the skip counts at their caps),
    bit-exact."""
    monkeypatch.setenv("PCP_TERRAIN_BLOCKS", "2")
    monkeypatch.setenv("PCP_FINE_SKIP", skip)
    rng = np.random.default_rng(5)
    n = 70_000
    cube = np.column_stack([rng.uniform(1.0, 1.05, n), rng.uniform(0.0, 0.05, n),
                            rng.uniform(0.0, 0.05, n)])
    cloud = np.zeros((n, 8), np.float32)
    cloud[:, :3] = cube
    poses = np.array([[0.0, 0.0, 0.3, -0.2, 0.0]])
    fan = _abi.fan_params(n_az=64, n_el=8, el_min_deg=-30.0, el_max_deg=10.0, max_distance=3.0)
    with _abi.Context(0) as ctx:
        ctx.set_terrain(cloud, point_step=32)
        blocked, units, fh, _ = ctx.raycast_fan(poses, fan, want_first_hit=True)
        assert ctx.terrain_info()["scan_layout"] == "fine"
        r_blocked, r_units, r_fh = oracle.raycast_fan(oracle.Cloud(cloud), poses, 64, 8,
                                                      fan.el_min, fan.el_max, 3.0)
        np.testing.assert_array_equal(fh, r_fh)
        np.testing.assert_array_equal(blocked, r_blocked)
        np.testing.assert_array_equal(units, r_units)
        assert blocked[0] > 0


# ---------------------------------------------------------------------------------- multi-GPU
_DEVICE_KEYS_CHECK = r"""
import sys
import numpy as np
import torch
torch.cuda.init()                      # torch's HIP runtime first, as in bench.py
sys.path.insert(0, sys.argv[1])
import bench
from pointcloud_processor_amd import _abi, synth
from pointcloud_processor_amd import dist as pd
scene = synth.terrain_scene()
gpu = _abi.Context(0)
gpu.set_terrain(scene.terrain, point_step=32)
poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, 96)
fan = _abi.fan_params(n_az=256, n_el=64)
b1, u1, _, _ = gpu.raycast_fan(poses, fan)
P, world = poses.shape[0], 4
ref_keys, ref_best = pd.reduce_fan(b1, 0, P, P)
dev = torch.device("cuda", 0)
units = torch.zeros(P, dtype=torch.int64, device=dev)
red = None
for r in range(world):
    lo, hi = pd.shard(P, world, r)
    k = torch.empty(P, dtype=torch.int64, device=dev)
    # no stream handle: torch's runtime is not libpcp's (the call returns with the keys written)
    gpu.raycast_fan_keys(np.ascontiguousarray(poses[lo:hi]), fan, lo, P, k.data_ptr(),
                         units.data_ptr() + 8 * lo, None)
    red = k if red is None else torch.minimum(red, k)
kh = red.cpu().numpy()
assert np.array_equal(kh >> 32, ref_keys)
assert np.array_equal(kh & 0xFFFFFFFF, np.arange(P))
assert int(kh.min()) & 0xFFFFFFFF == ref_best
assert np.array_equal(units.cpu().numpy().astype(np.uint64), u1)
k = torch.zeros(P, dtype=torch.int64, device=dev)
gpu.raycast_fan_keys(poses[:0].copy(), fan, P, P, k.data_ptr(), None, None)
assert bool((k == np.iinfo(np.int64).max).all())
print("device keys ok", P, ref_best)
"""


def test_fan_device_keys_match_reduce_fan():
    """bench.py --gpus N over RCCL: pcp_raycast_fan_keys writes each rank's keys into a torch
    device vector (no host copy), the collective is an int64 MIN.  Four ranks' shards on one
    device, their vectors combined by torch.minimum (the all-reduce's arithmetic): blocked
    counts, units and the argmin bit-identical to the host path (raycast_fan ->
    dist.reduce_fan).  In its own process, torch's HIP runtime initialised first as in
    bench.py (torch bundles its own ROCm runtime beside the one libpcp links)."""
    import subprocess
    import sys
    from pathlib import Path

    root = str(Path(__file__).resolve().parents[1])
    r = subprocess.run([sys.executable, "-c", _DEVICE_KEYS_CHECK, root], capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "device keys ok" in r.stdout


def test_fan_allreduce_own_communicator(gpu, loaded, scene):
    """bench.py --gpus N with libpcp's OWN RCCL communicator (one HIP runtime in the process):
    pcp_comm_init_rank over one rank, then pcp_raycast_fan_allreduce -- keys on the context's
    device vector, ncclAllReduce(MIN) on its stream, the reduced vector back once -- bit-identical
    to the host path (raycast_fan -> dist.reduce_fan): every blocked count, the units, the argmin.
    A shard that leaves poses unwritten is refused (PCP_E_STATE), an empty shard is not."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench
    from pointcloud_processor_amd import dist as pd

    poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, 96)
    fan = _abi.fan_params(n_az=256, n_el=64)
    b1, u1, _, _ = gpu.raycast_fan(poses, fan)
    P = poses.shape[0]
    ref_keys, ref_best = pd.reduce_fan(b1, 0, P, P)
    with _abi.Context(0) as ctx:
        assert ctx.comm_info() == (0, 0)
        with pytest.raises(_abi.PcpError):          # no communicator yet
            ctx.raycast_fan_allreduce(poses, fan, 0, P)
        ctx.comm_init_rank(1, _abi.comm_unique_id(), 0)
        assert ctx.comm_info() == (1, 0)
        ctx.set_terrain(scene.terrain, point_step=32)
        for rep in range(3):                         # steady state: same answer every query
            blocked = np.zeros(P, np.uint32)
            units = np.zeros(P, np.uint64)
            best, ms = ctx.raycast_fan_allreduce(poses, fan, 0, P, blocked, units, timed=rep == 2)
            np.testing.assert_array_equal(blocked, ref_keys)
            np.testing.assert_array_equal(units, u1)
            assert best == ref_best == int(np.argmin(b1))
        assert ms is not None and ms >= 0.0
        with pytest.raises(_abi.PcpError):           # poses [P/2, P) written by no rank
            ctx.raycast_fan_allreduce(np.ascontiguousarray(poses[:P // 2]), fan, 0, P)
        best, _ = ctx.raycast_fan_allreduce(poses[:0].copy(), fan, 0, 0)
        assert best == -1


def test_score_allreduce_own_communicator(oracle, loaded, scene, cells, aux):
    """runOptimization's scoring for N processes in ONE RCCL collective
    (pcp_score_poses_allreduce: [P totals | P covered | 3 x C newest-pose flag keys | health],
    ncclAllReduce(MAX) on the context's stream).  At N = 1 it is bit-identical to
    pcp_score_poses on the same context: every total's bits, the covered counts, the stale flags
    of two ticks (the second from the first's flags, poses reversed), the report; the oracle
    agrees on the flags and the best index.  A rank whose arguments fail before the collective
    still runs it with a poisoned health word: it reports its own error, and the communicator
    stays usable (the next query is exact again); poses that no rank scored are reported."""
    T, A = loaded
    params = _abi.default_vl_params()
    zx = np.ascontiguousarray(scene.zx120_pose5, np.float64)
    with _abi.Context(0) as ctx:
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.set_aux_cloud(aux, point_step=32)
        ctx.set_cells(cells.xyz, cells.normals)
        poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
        P, C = poses.shape[0], cells.xyz.shape[0]
        rep = _abi.VlReport()
        fl = np.zeros(C, np.uint8)
        with pytest.raises(_abi.PcpError):          # no communicator yet
            ctx.score_poses_allreduce(poses, zx, params, 0, P, fl, None, None, rep)
        ctx.comm_init_rank(1, _abi.comm_unique_id(), 0)
        f1, f2, fr = np.zeros(C, np.uint8), np.zeros(C, np.uint8), np.zeros(C, np.uint8)
        for tick, pz in enumerate((poses, poses[::-1].copy())):
            t1, c1, r1 = ctx.score_poses(pz, zx, params, f1)
            t2, c2 = np.zeros(P, np.float64), np.zeros(P, np.int32)
            rep2 = _abi.VlReport()
            ms = ctx.score_poses_allreduce(pz, zx, params, 0, P, f2, t2, c2, rep2, timed=True)
            assert ms is not None and ms >= 0.0
            np.testing.assert_array_equal(t2.view(np.uint64), t1.view(np.uint64))
            np.testing.assert_array_equal(c2, c1)
            np.testing.assert_array_equal(f2, f1)
            assert rep2.as_dict() == r1.as_dict(), tick
            _, _, rr = oracle.score_poses(T, A, cells.xyz, cells.normals, pz, scene.zx120_pose5,
                                          oracle.vl_params(), fr)
            np.testing.assert_array_equal(f2, fr)
            assert rep2.best_idx == rr.best_idx
        # a bad shard fails on this rank only; the collective still ran (health word poisoned)
        with pytest.raises(_abi.PcpError):
            ctx.score_poses_allreduce(poses, zx, params, 5, P, f2.copy(), None, None, rep)
        assert ctx.comm_info() == (1, 0)
        f3 = np.zeros(C, np.uint8)
        t3 = np.zeros(P, np.float64)
        ctx.score_poses_allreduce(poses, zx, params, 0, P, f3, t3, None, rep)
        t4, _, r4 = ctx.score_poses(poses, zx, params, np.zeros(C, np.uint8))
        np.testing.assert_array_equal(t3.view(np.uint64), t4.view(np.uint64))
        assert rep.best_idx == r4.best_idx
        # poses no rank scored (here: [0, 3) of a one-rank communicator) are an error, as the
        # fan's unwritten keys are -- not zero totals; the caller's flags stay as they were
        f5 = np.full(C, 0x5A, np.uint8)
        with pytest.raises(_abi.PcpError, match="scored by no rank"):
            ctx.score_poses_allreduce(poses[3:], zx, params, 3, P, f5, None, None, rep)
        assert (f5 == 0x5A).all()
        ctx.score_poses_allreduce(poses, zx, params, 0, P, f3 * 0, t3, None, rep)
        np.testing.assert_array_equal(t3.view(np.uint64), t4.view(np.uint64))
        # the fan's collective carries the same health word: a bad shard, then an exact query
        fan = _abi.fan_params(n_az=128, n_el=32)
        with pytest.raises(_abi.PcpError):
            ctx.raycast_fan_allreduce(poses, fan, 3, P)
        bl = np.zeros(P, np.uint32)
        best, _ = ctx.raycast_fan_allreduce(poses, fan, 0, P, bl)
        b_ref, _, _, best_ref = ctx.raycast_fan(poses, fan)
        np.testing.assert_array_equal(bl, b_ref[:P])
        assert best == best_ref


@pytest.mark.parametrize("onepass", ["1", "0"])
def test_exclusive_scan_tile_boundaries(onepass, monkeypatch):
    """the index builds' device scan on its own.  Back-to-back scans sized to 1, 2,
    63, 64 (the one-pass look-back's largest) and 65 (three launches) tiles of 2,048, growing
    and shrinking (the look-back state regrows, the epoch and ticket advance), each equal to
    numpy's, with PCP_SCAN_ONEPASS=1 (default) and 0."""
    monkeypatch.setenv("PCP_SCAN_ONEPASS", onepass)
    rng = np.random.default_rng(11)
    with _abi.Context(0) as ctx:
        for tiles in (1, 2, 63, 64, 65, 2, 64, 3, 200, 64, 1):
            for n in (tiles * 2048, tiles * 2048 - 5):
                if n <= 0:
                    continue
                a = rng.integers(0, 1000, n, dtype=np.uint32)
                ref = np.zeros(n + 1, np.uint64)
                ref[1:] = np.cumsum(a, dtype=np.uint64)
                got = ctx.debug_exclusive_scan(a)
                np.testing.assert_array_equal(got, ref.astype(np.uint32)), (tiles, n)


def _cell_census(got_sm, got_sz, ref_sm, ref_sz):
    """Per-cell comparison of evaluateCellScore values: cells whose score differs, by how many
    ulps, and the signed balance of the differences (a systematic drift leans one way)."""
    g = np.concatenate([got_sm.ravel(), got_sz])
    r = np.concatenate([ref_sm.ravel(), ref_sz])
    d = parity.ulps(g, r)
    pos = r > 0
    up = int(((g > r) & (d > 0)).sum())
    return {"cells": int(g.size), "positive": int(pos.sum()), "differ": int((d > 0).sum()),
            "up": up, "down": int((d > 0).sum()) - up, "max_ulps": float(d.max(initial=0)),
            "zero_mismatch": int(((g > 0) != pos).sum())}


def test_parity_bar_per_cell(oracle, loaded, scene, cells, aux):
    """VERDICT r5 item 5, at the cells: evaluateCellScore per (pose, cell) on the device
    (pcp_score_matrix) against the oracle's (orc_score_matrix) on the 91-candidate tick.  The
    production build rounds acos / sin correctly (pcp_crmath.h), as glibc does but for its rare
    near ties: 0.16 % of the positive cell scores differ, by 1-4 ulps (ocml's own functions
    left 9 %, up to 8 ulps); the `make perturb` (every cell) and `make perturb8` (every 8th cell)
    builds fail the per-cell bar (tests/parity.py: cell_bar)."""
    T, A = loaded
    params = _abi.default_vl_params()
    zx = np.ascontiguousarray(scene.zx120_pose5, np.float64)
    res = {}
    for tag, path in (("prod", None), ("perturbed", str(PERTURB_LIB)),
                      ("perturbed8", str(PERTURB8_LIB))):
        with _abi.Context(0, lib_path=path) as ctx:
            ctx.set_terrain(scene.terrain, point_step=32)
            ctx.set_aux_cloud(aux, point_step=32)
            ctx.set_cells(cells.xyz, cells.normals)
            poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
            res[tag] = (poses, ctx.score_matrix(poses, zx, params))
    poses = res["prod"][0]
    r_sm, r_sz = oracle.score_matrix(T, A, cells.xyz, cells.normals, poses, scene.zx120_pose5,
                                     oracle.vl_params())
    for tag in res:
        np.testing.assert_array_equal(res[tag][0], poses)
        cen = _cell_census(*res[tag][1], r_sm, r_sz)
        print("cell census", tag, cen, parity.cell_bar(cen))
        assert cen["zero_mismatch"] == 0
        assert parity.cell_bar(cen) == (tag == "prod"), (tag, cen)


def test_score_stats_and_burst(loaded, scene, cells, aux):
    """The reference-mode roofline's inputs: pcp_score_poses_stats counts
    the visibility rays' gather lane-loads with a twin of k_score_cells -- deterministic, every
    walk start follows a probe, the fine-window copy needs no directory loads -- and
    pcp_score_poses_burst times the production launch; neither touches the caller's flags nor
    changes the next query's results."""
    params = _abi.default_vl_params()
    zx = np.ascontiguousarray(scene.zx120_pose5, np.float64)
    with _abi.Context(0) as ctx:
        ctx.set_terrain(scene.terrain, point_step=32)
        ctx.set_aux_cloud(aux, point_step=32)
        ctx.set_cells(cells.xyz, cells.normals)
        poses = ctx.generate_candidates(cells.grid_bbox, params, scene.zx120_pose5)
        C = cells.xyz.shape[0]
        t0, c0, r0 = ctx.score_poses(poses, zx, params, np.zeros(C, np.uint8))
        st = ctx.score_poses_stats(poses, zx, params)
        assert st == ctx.score_poses_stats(poses, zx, params)
        assert st["probes"] >= st["walk_starts"] > 0 and st["point_tests"] > 0
        assert st["directory_loads"] == 0
        # more poses, more rays: the counts grow
        st2 = ctx.score_poses_stats(np.concatenate([poses, poses]), zx, params)
        assert st2["probes"] > st["probes"]
        ms = ctx.score_poses_burst(poses, zx, params, reps=5)
        assert ms > 0.0
        t1, c1, r1 = ctx.score_poses(poses, zx, params, np.zeros(C, np.uint8))
        np.testing.assert_array_equal(t1.view(np.uint64), t0.view(np.uint64))
        np.testing.assert_array_equal(c1, c0)
        assert r1.as_dict() == r0.as_dict()


def test_fan_keys_wait_stream_then_fan(gpu, loaded, scene, oracle):
    """a keys query handed to a libpcp wait_stream returns before its pose upload
    has read the pinned staging; the next fan query on the context (other poses) must not
    overwrite that staging first.  Keys of the first query == the oracle's blocked counts of its
    poses, the second query's counts == its own."""
    fan = _abi.fan_params(n_az=128, n_el=32)
    sc = scene
    rng = np.random.default_rng(7)
    a = np.column_stack([rng.uniform(-5, 5, 48), rng.uniform(-5, 5, 48), rng.uniform(0.5, 2.0, 48),
                         rng.uniform(-0.6, 0.0, 48), rng.uniform(-3, 3, 48)])
    b = a.copy()
    b[:, 4] += 1.0
    b[:, 2] += 0.7
    T = oracle.Cloud(sc.terrain)
    ra, _, _ = oracle.raycast_fan(T, a, 128, 32, fan.el_min, fan.el_max, fan.max_distance,
                                  want_first_hit=False)
    rb, _, _ = oracle.raycast_fan(T, b, 128, 32, fan.el_min, fan.el_max, fan.max_distance,
                                  want_first_hit=False)
    assert not np.array_equal(ra, rb)
    with _abi.Context(0) as ctx:
        ctx.set_terrain(sc.terrain, point_step=32)
        st = ctx.stream_create()
        try:
            keys = ctx.dev_alloc(8 * a.shape[0])
            for _ in range(3):
                ctx.raycast_fan_keys(np.ascontiguousarray(a), fan, 0, a.shape[0], keys, None, st)
                got_b, _, _, _ = ctx.raycast_fan(b, fan)      # rewrites the pinned pose staging
                kh = np.zeros(a.shape[0], np.int64)
                ctx.synchronize()
                ctx.d2h(kh, keys)
                np.testing.assert_array_equal((kh >> 32).astype(np.uint32), ra)
                np.testing.assert_array_equal(got_b, rb)
            ctx.dev_free(keys)
        finally:
            ctx.stream_destroy(st)


def _need_devices(devices):
    if len(set(devices)) > 1 and _abi.device_count() < len(set(devices)):
        pytest.skip(f"needs {len(set(devices))} GPUs (RCCL over distinct devices); "
                    f"{_abi.device_count()} visible")


def test_multi_rejects_mixed_device_lists(gpu):
    """Devices all distinct (RCCL) or all the same (on-device combine); a mixed list such as
    {0, 0, 1} would combine buffers across devices without peer access: refused."""
    with pytest.raises(_abi.PcpError):
        _abi.Multi([0, 0, 1])
    with pytest.raises(_abi.PcpError):
        _abi.Multi([0, 1, 1])


@pytest.mark.parametrize("devices", [[0], [0, 0, 0], [0, 1], [0, 1, 2, 3]])
def test_multi_fan_matches_single_context(gpu, loaded, scene, devices):
    """pcp_multi: the C2 poses sharded over the ranks, ONE all-reduce(MIN) over
    the (blocked << 32) | pose keys -- RCCL over one device, or three ranks sharing device 0
    (keys combined on the device) -- bit-identical to one context over all poses."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    _need_devices(devices)
    poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, 256)
    fan = _abi.fan_params()
    b1, u1, _, best1 = gpu.raycast_fan(poses, fan)
    with _abi.Multi(devices) as m:
        assert m.n == len(devices) and m.uses_rccl == (len(set(devices)) == len(devices))
        m.set_terrain(scene.terrain, point_step=32)
        for sel in (poses, poses[:5], poses[:1]):        # ranks with 0 poses too
            b, u, best = m.raycast_fan(sel, fan)
            n = sel.shape[0]
            np.testing.assert_array_equal(b, b1[:n])
            np.testing.assert_array_equal(u, u1[:n])
            assert best == int(np.argmin(b1[:n]))
        b, u, best = m.raycast_fan(poses[:0], fan)
        assert b.size == 0 and best == -1
    assert best1 == int(np.argmin(b1))


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 1]])
def test_multi_score_matches_single_context(gpu, loaded, scene, cells, aux, devices):
    """pcp_multi_score_poses: totals, covered counts, strict-'>' best index, stale flags and the
    colour report over two ticks (the second starting from the first's flags), identical to
    pcp_score_poses on one context."""
    _need_devices(devices)
    params = _abi.default_vl_params()
    poses = gpu.generate_candidates(cells.grid_bbox, _abi.default_vl_params(num_candidates=400),
                                    scene.zx120_pose5)
    with _abi.Multi(devices) as m:
        m.set_terrain(scene.terrain, point_step=32)
        m.set_aux_cloud(aux, point_step=32)
        m.set_cells(cells.xyz, cells.normals)
        f1 = np.zeros(cells.xyz.shape[0], np.uint8)
        fm = f1.copy()
        for sel in (poses, poses[::7][:3], poses[:0]):
            t1, c1, r1 = gpu.score_poses(sel, scene.zx120_pose5, params, f1)
            tm, cm, rm = m.score_poses(sel, scene.zx120_pose5, params, fm)
            np.testing.assert_array_equal(tm, t1)
            np.testing.assert_array_equal(cm, c1)
            np.testing.assert_array_equal(fm, f1)
            assert rm.as_dict() == r1.as_dict()


def test_gpu_matches_flann_restatement(gpu, oracle, loaded, scene):
    """The GPU's first hits against the oracle in FLANN mode (oracle/pcp_flann.c: the
    KdTreeFLANN search the reference runs, float pruning included) on 8 of the C2 poses,
    every sample query also cross-checked against the exact grid count."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    import bench

    poses, _ = bench._poses_for(gpu, bench._grid_bbox(scene.area), scene.zx120_pose5, 256)
    sel = poses[::32]
    fan = _abi.fan_params()
    blocked, units, fh, _ = gpu.raycast_fan(sel, fan, want_first_hit=True)
    T, _ = loaded
    tree = oracle.KdTree(scene.terrain)
    oracle.set_threads(16)
    try:
        rb, ru, rfh, st = oracle.raycast_fan_kd(tree, T, sel, 1024, 256, fan.el_min, fan.el_max,
                                                fan.max_distance)
    finally:
        oracle.set_threads(1)
    assert st["count_mismatch"] == 0 and st["any_mismatch"] == 0, st
    assert st["queries"] == int(ru.sum())
    np.testing.assert_array_equal(fh, rfh)
    np.testing.assert_array_equal(blocked, rb)
    np.testing.assert_array_equal(units, ru)
