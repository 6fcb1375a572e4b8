"""ctypes binding of oracle/liboracle.so -- the CPU restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / timed CPU baseline.  Never a product path.
Parity unpinned (see pcp_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


class VlParams(C.Structure):
    _fields_ = [("grid_resolution", C.c_double), ("sensor_height", C.c_double),
                ("search_radius", C.c_double), ("max_distance", C.c_double),
                ("num_candidates", C.c_int32), ("vertical_layers", C.c_int32)]


class VlReport(C.Structure):
    _fields_ = [("best_idx", C.c_int64), ("best_score", C.c_double),
                ("zx120_total_score", C.c_double),
                ("zx120_range_ok", C.c_int32), ("zx120_fov_ok", C.c_int32),
                ("zx120_visible_ok", C.c_int32), ("total_cells", C.c_int32),
                ("zx120_green", C.c_int32), ("zx120_red", C.c_int32),
                ("zx120_blue", C.c_int32), ("zx120_yellow", C.c_int32),
                ("green", C.c_int32), ("red", C.c_int32), ("blue", C.c_int32),
                ("yellow", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = C.c_void_p
_SIGS = [
    ("orc_set_threads", None, [C.c_int]),
    ("orc_get_threads", C.c_int, []),
    ("orc_crop_box", C.c_int64, [_P, C.c_int64, C.c_int64, _P, _P]),
    ("orc_voxel_grid", C.c_int64, [_P, C.c_int64, C.c_int64, C.c_float, _P, _P, _P,
                                   C.POINTER(C.c_int)]),
    ("orc_transform_rgb", None, [_P, C.c_int64, C.c_int64, _P, _P, C.c_uint8, C.c_uint8,
                                 C.c_uint8, _P]),
    ("orc_cloud_build", _P, [_P, C.c_int64, C.c_int64]),
    ("orc_cloud_free", None, [_P]),
    ("orc_cloud_any_within", C.c_int, [_P, C.c_float, C.c_float, C.c_float, C.c_double]),
    ("orc_ground_height", C.c_double, [_P, C.c_double, C.c_double]),
    ("orc_generate_candidates", C.c_int64, [_P, C.c_int, _P, C.POINTER(VlParams), _P, _P,
                                            C.c_int64]),
    ("orc_score_poses", None, [_P, _P, C.c_int64, _P, _P, C.c_int64, _P, C.c_int64, _P,
                               C.POINTER(VlParams), _P, _P, _P, C.POINTER(VlReport)]),
    ("orc_score_totals", None, [_P, _P, C.c_int64, _P, _P, C.c_int64, _P, C.c_int64, _P,
                                C.POINTER(VlParams), _P, _P]),
    ("orc_score_matrix", None, [_P, _P, C.c_int64, _P, _P, C.c_int64, _P, C.c_int64, _P,
                                C.POINTER(VlParams), _P, _P]),
    ("orc_raycast_fan", None, [_P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_double, C.c_double,
                               C.c_double, _P, _P, _P]),
    ("orc_cloud_use_kdtree", None, [_P, _P]),
    ("orc_cloud_count_within", C.c_int64, [_P, C.c_float, C.c_float, C.c_float, C.c_double]),
    ("orc_kd_build", _P, [_P, C.c_int64, C.c_int64, C.c_int]),
    ("orc_kd_free", None, [_P]),
    ("orc_kd_size", C.c_int64, [_P]),
    ("orc_kd_radius", C.c_int64, [_P, C.c_float, C.c_float, C.c_float, C.c_float, _P,
                                  C.c_int64]),
    ("orc_kd_check_queries", None, [_P, _P, _P, C.c_int64, C.c_double, _P]),
    ("orc_kd_raycast_fan", None, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_double,
                                  C.c_double, C.c_double, _P, _P, _P, _P]),
    ("orc_fan_tables", None, [C.c_int32, C.c_int32, C.c_double, C.c_double, _P, _P, _P, _P]),
    ("orc_area_normals", None, [_P, C.c_int64, C.c_int64, C.c_double, _P]),
    ("orc_terrain_height", C.c_double, [_P, C.c_int64, C.c_int64, C.c_double, C.c_double,
                                        C.c_double]),
    ("orc_drivable_area", None, [_P, C.c_int64, C.c_int64, _P, _P, C.c_double, C.c_double,
                                 C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                 C.c_double, C.c_int32, C.c_double, _P, _P, _P]),
    ("orc_excavate", None, [_P, C.c_int64, C.c_int64, _P, _P, _P, _P, _P, C.c_int64, _P, _P,
                            C.c_int64, _P, _P]),
    ("orc_excavation_grid", C.c_int64, [_P, C.c_int64, C.c_int64, C.c_double, C.c_int32, _P, _P,
                                        _P, C.c_int64, _P, _P]),
    ("orc_filter_frame_mt", C.c_int64, [C.c_int, _P, _P, _P, _P, C.c_float, _P, _P, _P,
                                        C.c_int64, _P, C.c_int]),
]

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        l = C.CDLL(str(LIB))
        for name, res, args in _SIGS:
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f32(a):
    a = np.ascontiguousarray(a, np.float32)
    if a.ndim != 2 or a.shape[1] < 3:
        raise ValueError("expected (N, k>=3) float32")
    return a


def set_threads(n: int):
    lib().orc_set_threads(int(n))


def crop_box(pts, box):
    a = _f32(pts)
    kept = np.empty(max(a.shape[0], 1), np.uint32)
    box = np.ascontiguousarray(box, np.float64)
    m = lib().orc_crop_box(_p(a), a.shape[0], a.shape[1], _p(box), _p(kept))
    return kept[:m].copy()


def voxel_grid(pts, leaf):
    a = _f32(pts)
    n = max(a.shape[0], 1)
    out = np.empty((n, 3), np.float32)
    idx = np.empty(n, np.uint32)
    cnt = np.empty(n, np.uint32)
    pt = C.c_int()
    k = lib().orc_voxel_grid(_p(a), a.shape[0], a.shape[1], C.c_float(leaf), _p(out), _p(idx),
                             _p(cnt), C.byref(pt))
    return out[:k].copy(), idx[:k].copy(), cnt[:k].copy(), bool(pt.value)


def transform_rgb(pts, t, q, rgb):
    a = _f32(pts)
    out = np.empty((max(a.shape[0], 1), 8), np.float32)
    t = np.ascontiguousarray(t, np.float64)
    q = np.ascontiguousarray(q, np.float64)
    lib().orc_transform_rgb(_p(a), a.shape[0], a.shape[1], _p(t), _p(q), int(rgb[0]),
                            int(rgb[1]), int(rgb[2]), _p(out))
    return out[: a.shape[0]].copy()


def filter_frame_mt(clouds, boxes, leaf, tfs, rgbs, threads):
    """The C3 frame on `threads` OpenMP threads (pcp_oracle_mt.c): per cloud crop ->
    VoxelGrid -> transform + colour, concatenated -> (N, 8) float32 records, per-cloud counts."""
    arrs = [_f32(c) for c in clouds]
    k = len(arrs)
    ptrs = (C.c_void_p * k)(*[a.ctypes.data for a in arrs])
    n = np.array([a.shape[0] for a in arrs], np.int64)
    stride = np.array([a.shape[1] for a in arrs], np.int64)
    bx = np.ascontiguousarray(np.asarray(boxes, np.float64).reshape(k, 6))
    tq = np.ascontiguousarray([list(t) + list(q) for t, q in tfs], np.float64)
    rgb = np.ascontiguousarray(np.asarray(rgbs, np.uint8).reshape(k, 3))
    cap = int(n.sum())
    out = np.empty((max(cap, 1), 8), np.float32)
    per = np.zeros(k, np.int64)
    m = lib().orc_filter_frame_mt(k, ptrs, _p(n), _p(stride), _p(bx), C.c_float(leaf), _p(tq),
                                  _p(rgb), _p(out), cap, _p(per), int(threads))
    if m < 0:
        raise ValueError("orc_filter_frame_mt failed")
    return out[:m].copy(), per


class Cloud:
    """Exact radius-search structure over a point array (replaces KdTreeFLANN).

    flann=True: every radius query the oracle makes on this cloud (ray march, relaxed zx120
    check, getGroundHeight) is answered by the restated KdTreeFLANN of pcp_flann.c instead of
    the exact grid scan -- the reference's own search, float pruning included."""

    def __init__(self, pts, flann=False):
        a = _f32(pts)
        self.n = a.shape[0]
        self.h = lib().orc_cloud_build(_p(a), a.shape[0], a.shape[1])
        self.kd = None
        if flann:
            self.kd = KdTree(a)
            lib().orc_cloud_use_kdtree(self.h, self.kd.h)

    def __del__(self):
        try:
            if self.h:
                lib().orc_cloud_free(self.h)
        except Exception:
            pass

    def any_within(self, q, radius):
        return bool(lib().orc_cloud_any_within(self.h, C.c_float(q[0]), C.c_float(q[1]),
                                               C.c_float(q[2]), radius))

    def ground_height(self, x, y):
        return lib().orc_ground_height(self.h, x, y)

    def count_within(self, q, radius):
        return int(lib().orc_cloud_count_within(self.h, C.c_float(q[0]), C.c_float(q[1]),
                                                C.c_float(q[2]), radius))


class KdTree:
    """FLANN 1.9.1 KDTreeSingleIndex as PCL 1.12.1 KdTreeFLANN builds and queries it
    (oracle/pcp_flann.c): the reference's own radius search, float pruning included."""

    def __init__(self, pts, leaf_max=15):
        a = _f32(pts)
        self.n = a.shape[0]
        self.h = lib().orc_kd_build(_p(a), a.shape[0], a.shape[1], int(leaf_max))

    def __del__(self):
        try:
            if self.h:
                lib().orc_kd_free(self.h)
        except Exception:
            pass

    def radius_search(self, q, radius, want_idx=False):
        """-> neighbour count (and their cloud indices, sorted) with dist < float(r*r)."""
        r2 = C.c_float(float(np.float32(radius * radius)))
        q = [C.c_float(float(v)) for v in q[:3]]
        n = lib().orc_kd_radius(self.h, *q, r2, None, 0)
        if not want_idx:
            return int(n)
        idx = np.empty(max(n, 1), np.int64)
        lib().orc_kd_radius(self.h, *q, r2, _p(idx), n)
        return int(n), np.sort(idx[:n])

    def check_queries(self, grid: "Cloud", queries, radius):
        """Tree count vs the exact grid count for every query (float xyz rows) ->
        {queries, count_mismatch, any_mismatch, neighbours}."""
        q = np.ascontiguousarray(np.asarray(queries, np.float32)[:, :3])
        st = np.zeros(4, np.uint64)
        lib().orc_kd_check_queries(self.h, grid.h, _p(q), q.shape[0], float(radius), _p(st))
        return dict(zip(("queries", "count_mismatch", "any_mismatch", "neighbours"),
                        (int(x) for x in st)))


def raycast_fan_kd(tree: KdTree, grid: "Cloud | None", poses5, n_az, n_el, el_min, el_max,
                   max_distance, want_first_hit=True):
    """The fan march with every sample answered by the restated KdTreeFLANN, each sample
    cross-checked against the exact grid count -> (blocked, units, first_hit, stats)."""
    poses = np.ascontiguousarray(poses5, np.float64).reshape(-1, 5)
    P = poses.shape[0]
    fh = np.empty((P, n_el, n_az), np.int16) if want_first_hit else None
    blocked = np.zeros(max(P, 1), np.uint32)
    units = np.zeros(max(P, 1), np.uint64)
    st = np.zeros(4, np.uint64)
    lib().orc_kd_raycast_fan(tree.h, grid.h if grid else None, _p(poses), P, n_az, n_el,
                             el_min, el_max, max_distance, _p(fh), _p(blocked), _p(units),
                             _p(st))
    stats = dict(zip(("queries", "count_mismatch", "any_mismatch", "neighbours"),
                     (int(x) for x in st)))
    return blocked[:P].copy(), units[:P].copy(), fh, stats


def vl_params(**kw):
    p = VlParams(0.1, 1.1, 3.0, 15.0, 100, 10)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def generate_candidates(terrain: Cloud | None, grid_bbox, params, zx120_pose5, terrain_empty=False):
    bb = np.ascontiguousarray(grid_bbox, np.float64)
    zx = np.ascontiguousarray(zx120_pose5, np.float64)
    gs = int(np.ceil(np.sqrt(float(params.num_candidates))))
    cap = max(gs * gs, 1)
    out = np.empty((cap, 5), np.float64)
    n = lib().orc_generate_candidates(terrain.h if terrain else None, int(terrain_empty), _p(bb),
                                      C.byref(params), _p(zx), _p(out), cap)
    return out[:n].copy()


def score_poses(terrain: Cloud | None, aux: Cloud | None, cells_xyz, cells_nrm, poses5,
                zx120_pose5, params, cell_flags):
    cx = np.ascontiguousarray(cells_xyz, np.float64).reshape(-1, 3)
    cn = np.ascontiguousarray(cells_nrm, np.float32).reshape(-1, 3)
    poses = np.ascontiguousarray(poses5, np.float64).reshape(-1, 5)
    zx = np.ascontiguousarray(zx120_pose5, np.float64)
    P = poses.shape[0]
    tot = np.empty(max(P, 1), np.float64)
    cov = np.empty(max(P, 1), np.int32)
    rep = VlReport()
    assert cell_flags.dtype == np.uint8
    lib().orc_score_poses(terrain.h if terrain else None, aux.h if aux else None,
                          aux.n if aux else 0, _p(cx), _p(cn), cx.shape[0], _p(poses), P, _p(zx),
                          C.byref(params), _p(cell_flags), _p(tot), _p(cov), C.byref(rep))
    return tot[:P].copy(), cov[:P].copy(), rep


def score_matrix(terrain: Cloud | None, aux: Cloud | None, cells_xyz, cells_nrm, poses5,
                 zx120_pose5, params):
    """evaluateCellScore per (pose, cell) -> (score_mobile [P, C], score_zx120 [C]) (OpenMP
    over poses; the per-cell parity bar)."""
    cx = np.ascontiguousarray(cells_xyz, np.float64).reshape(-1, 3)
    cn = np.ascontiguousarray(cells_nrm, np.float32).reshape(-1, 3)
    poses = np.ascontiguousarray(poses5, np.float64).reshape(-1, 5)
    zx = np.ascontiguousarray(zx120_pose5, np.float64)
    P, nc = poses.shape[0], cx.shape[0]
    sm = np.zeros((max(P, 1), max(nc, 1)), np.float64)
    sz = np.zeros(max(nc, 1), np.float64)
    lib().orc_score_matrix(terrain.h if terrain else None, aux.h if aux else None,
                           aux.n if aux else 0, _p(cx), _p(cn), nc, _p(poses), P, _p(zx),
                           C.byref(params), _p(sm), _p(sz))
    return sm[:P, :nc].copy(), sz[:nc].copy()


def score_totals(terrain: Cloud | None, aux: Cloud | None, cells_xyz, cells_nrm, poses5,
                 zx120_pose5, params):
    """Per-pose total_score / covered of the candidate loop (no flags), OpenMP over poses."""
    cx = np.ascontiguousarray(cells_xyz, np.float64).reshape(-1, 3)
    cn = np.ascontiguousarray(cells_nrm, np.float32).reshape(-1, 3)
    poses = np.ascontiguousarray(poses5, np.float64).reshape(-1, 5)
    zx = np.ascontiguousarray(zx120_pose5, np.float64)
    P = poses.shape[0]
    tot = np.empty(max(P, 1), np.float64)
    cov = np.empty(max(P, 1), np.int32)
    lib().orc_score_totals(terrain.h if terrain else None, aux.h if aux else None,
                           aux.n if aux else 0, _p(cx), _p(cn), cx.shape[0], _p(poses), P,
                           _p(zx), C.byref(params), _p(tot), _p(cov))
    return tot[:P].copy(), cov[:P].copy()


def raycast_fan(terrain: Cloud, poses5, n_az, n_el, el_min, el_max, max_distance,
                want_first_hit=True):
    poses = np.ascontiguousarray(poses5, np.float64).reshape(-1, 5)
    P = poses.shape[0]
    fh = np.empty((P, n_el, n_az), np.int16) if want_first_hit else None
    blocked = np.zeros(max(P, 1), np.uint32)
    units = np.zeros(max(P, 1), np.uint64)
    lib().orc_raycast_fan(terrain.h, _p(poses), P, n_az, n_el, el_min, el_max, max_distance,
                          _p(fh), _p(blocked), _p(units))
    return blocked[:P].copy(), units[:P].copy(), fh


def fan_tables(n_az, n_el, el_min, el_max):
    ca = np.empty(n_az); sa = np.empty(n_az); ce = np.empty(n_el); se = np.empty(n_el)
    lib().orc_fan_tables(n_az, n_el, el_min, el_max, _p(ca), _p(sa), _p(ce), _p(se))
    return ca, sa, ce, se


def area_normals(pts, radius=1.5):
    """computeTerrainNormals: (N, 3) float32, NaN where < 3 neighbours."""
    a = _f32(pts)
    out = np.empty((a.shape[0], 3), np.float32)
    lib().orc_area_normals(_p(a), a.shape[0], a.shape[1], float(radius), _p(out))
    return out


def excavation_grid(pts, grid_resolution=0.1, vertical_layers=10, normals=None):
    """generateExcavationGrid3D + computeCellSurfaceNormal -> (cells_xyz f64 (M,3),
    cells_nrm f32 (M,3), grid_bbox f64 (6,), dims (gh, gw, layers))."""
    a = _f32(pts)
    nrm = None if normals is None else np.ascontiguousarray(normals, np.float32)
    bbox = np.zeros(6, np.float64)
    dims = np.zeros(3, np.int32)
    n = lib().orc_excavation_grid(_p(a), a.shape[0], a.shape[1], float(grid_resolution),
                                  int(vertical_layers), _p(nrm), None, None, 0, _p(bbox), _p(dims))
    xyz = np.empty((max(n, 1), 3), np.float64)
    cn = np.empty((max(n, 1), 3), np.float32)
    lib().orc_excavation_grid(_p(a), a.shape[0], a.shape[1], float(grid_resolution),
                              int(vertical_layers), _p(nrm), _p(xyz), _p(cn), n, _p(bbox),
                              _p(dims))
    return xyz[:n], cn[:n], bbox, tuple(int(d) for d in dims)


class ExcParams(C.Structure):
    _fields_ = [("depth", C.c_double), ("slope_angle_deg", C.c_double),
                ("offset_x", C.c_double), ("offset_y", C.c_double),
                ("point_density", C.c_double), ("terrain_search_radius", C.c_double),
                ("l_shape_enabled", C.c_int32), ("arm1_length", C.c_double),
                ("arm1_width", C.c_double), ("arm2_length", C.c_double),
                ("arm2_width", C.c_double), ("width", C.c_double), ("length", C.c_double)]


def exc_params(**kw):
    """excavated_surface_generator.cpp:29-51 defaults."""
    p = ExcParams(1.0, 75.0, 4.0, 1.0, 0.05, 0.5, 1, 2.0, 1.2, 2.0, 1.2, 1.2, 1.8)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def terrain_height(pts, x, y, radius=0.5):
    a = _f32(pts)
    return lib().orc_terrain_height(_p(a), a.shape[0], a.shape[1], float(x), float(y),
                                    float(radius))


def excavate(pts, t, q, params=None):
    """-> keep (N,) bool, surf (S, 4) f32 rows x,y,z,rgb, area (A, 4), pose (cx, cy, cz, yaw)."""
    a = _f32(pts)
    p = params or exc_params()
    t = np.ascontiguousarray(t, np.float64)
    q = np.ascontiguousarray(q, np.float64)
    keep = np.empty(max(a.shape[0], 1), np.uint8)
    ns, na = C.c_int64(), C.c_int64()
    pose = np.zeros(4, np.float64)
    lib().orc_excavate(_p(a), a.shape[0], a.shape[1], C.byref(p), _p(t), _p(q), _p(keep), None,
                       0, C.byref(ns), None, 0, C.byref(na), _p(pose))
    surf = np.empty((max(ns.value, 1), 4), np.float32)
    area = np.empty((max(na.value, 1), 4), np.float32)
    lib().orc_excavate(_p(a), a.shape[0], a.shape[1], C.byref(p), _p(t), _p(q), _p(keep),
                       _p(surf), ns.value, C.byref(ns), _p(area), na.value, C.byref(na),
                       _p(pose))
    return keep[:a.shape[0]].astype(bool), surf[:ns.value], area[:na.value], pose


def drivable_area(pts, t, q, robot_xy, start_xy, res=1.0, map_w=100.0, map_h=100.0,
                  max_gradient=0.3, min_points=10, clear_r=3.0):
    """calc_drivable_area: -> grid (gh, gw) int8, origin (2,)."""
    a = _f32(pts)
    gw, gh = int(map_w / res), int(map_h / res)
    grid = np.zeros((max(gh, 1), max(gw, 1)), np.int8)
    dims = np.zeros(2, np.int32)
    origin = np.zeros(2, np.float64)
    lib().orc_drivable_area(_p(a), a.shape[0], a.shape[1], _p(np.asarray(t, np.float64)),
                            _p(np.asarray(q, np.float64)), float(robot_xy[0]),
                            float(robot_xy[1]), float(start_xy[0]), float(start_xy[1]),
                            float(res), float(map_w), float(map_h), float(max_gradient),
                            int(min_points), float(clear_r), _p(grid), _p(dims), _p(origin))
    return grid[:gh, :gw], origin
