"""Synthetic inputs for the hot path, seeded with 20260227.

The reference ships no data (no rosbag, no fixtures), so benchmarks and tests run on
synthetic scenes of the documented shape.  The geometry restates the excavation generator
(`excavated_surface_generator.cpp`) only as a data source: it is input generation, not the
product path, and it uses numpy/scipy approximations where exactness does not matter
(e.g. getTerrainHeight as a disk mean on the ground lattice).

Scenes:
  * terrain_scene()  -- T1M: 1000 x 1000 ground lattice at 0.05 m, z ~ N(0, 0.01), L-pit
                        carved (processExcavation :457-485) and its surface added
                        (generateExcavatedSurface :487-584) -> /excavated_terrain;
                        generateExcavationArea (:350-455) -> /excavation_area.
  * excavation_cells() -- virtual_lidar.cpp:209-340 grid cells + PCA normals.
  * lidar_cloud()     -- 64-ring LiDAR-like cloud with a ground plane (C3).
  * zx120_scan()      -- HDL-64-like scan from the zx120 sensor (aux cloud, C1/C5).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

SEED = 20260227


# ----------------------------------------------------------------------------------------
# excavation geometry (excavated_surface_generator.cpp:28-47 defaults, :138-181 boxes)
# ----------------------------------------------------------------------------------------
@dataclass
class ExcavationParams:
    depth: float = 1.0
    slope_angle: float = 75.0
    offset_x: float = 4.0
    offset_y: float = 1.0
    point_density: float = 0.05
    l_shape_enabled: bool = True
    arm1_length: float = 2.0
    arm1_width: float = 1.2
    arm2_length: float = 2.0
    arm2_width: float = 1.2
    width: float = 1.2
    length: float = 1.8


def excavation_boxes(p: ExcavationParams):
    """getExcavationBoxes (:138-181): list of (cx, cy, length, width, minx, maxx, miny, maxy)."""
    if p.l_shape_enabled:
        boxes = []
        cx, cy, ln, wd = 0.0, -p.arm1_length / 2.0, p.arm1_width, p.arm1_length
        boxes.append((cx, cy, ln, wd, cx - ln / 2.0, cx + ln / 2.0, cy - wd / 2.0, cy + wd / 2.0))
        cx, cy = p.arm2_length / 2.0, -p.arm1_length + p.arm2_width / 2.0
        ln, wd = p.arm2_length, p.arm2_width
        boxes.append((cx, cy, ln, wd, cx - ln / 2.0, cx + ln / 2.0, cy - wd / 2.0, cy + wd / 2.0))
        return boxes
    return [(0.0, 0.0, p.length, p.width, -p.length / 2.0, p.length / 2.0,
             -p.width / 2.0, p.width / 2.0)]


def _inside_any(xl, yl, boxes):
    out = np.zeros(np.broadcast(xl, yl).shape, bool)
    for b in boxes:
        out |= (xl >= b[4]) & (xl <= b[5]) & (yl >= b[6]) & (yl <= b[7])
    return out


def _outer_edge(xl, yl, boxes, tol):
    """isOuterEdge (:240-261)."""
    ins = _inside_any(xl, yl, boxes)
    nb = (~_inside_any(xl + tol, yl, boxes)) | (~_inside_any(xl - tol, yl, boxes)) | \
         (~_inside_any(xl, yl + tol, boxes)) | (~_inside_any(xl, yl - tol, boxes))
    return ins & nb


def _inside_excavation(xl, yl, zrel, boxes, p: ExcavationParams):
    """isInsideExcavationArea (:327-348), vectorised."""
    slope_offset = p.depth / math.tan(p.slope_angle * math.pi / 180.0)
    ok = (zrel >= -p.depth) & (zrel <= 0)
    cur = slope_offset * ((p.depth + zrel) / p.depth)
    inside = np.zeros(xl.shape, bool)
    for b in boxes:
        inside |= (np.abs(xl - b[0]) <= b[2] / 2.0 + cur) & (np.abs(yl - b[1]) <= b[3] / 2.0 + cur)
    return ok & inside


@dataclass
class TerrainScene:
    terrain: np.ndarray          # (N, 8) float32 PointXYZRGB image: x,y,z,1,rgb,0,0,0
    area: np.ndarray             # (M, 8) float32 /excavation_area
    center: tuple                # excavation centre (x, y, z)
    zx120_pose5: np.ndarray      # getZX120Position result for base_link at the origin
    info: dict = field(default_factory=dict)


def _pack(xyz: np.ndarray, rgb) -> np.ndarray:
    out = np.zeros((xyz.shape[0], 8), np.float32)
    out[:, :3] = xyz
    out[:, 3] = 1.0
    r, g, b = rgb if np.ndim(rgb) == 1 else (None, None, None)
    if r is None:
        rgba = (rgb[:, 2].astype(np.uint32) | (rgb[:, 1].astype(np.uint32) << 8) |
                (rgb[:, 0].astype(np.uint32) << 16) | np.uint32(255 << 24))
    else:
        rgba = np.full(xyz.shape[0], (b | (g << 8) | (r << 16) | (255 << 24)), np.uint32)
    out[:, 4] = rgba.view(np.float32)
    return out


def terrain_scene(n_side: int = 1000, spacing: float = 0.05, x0: float = -20.0,
                  y0: float = -25.0, sigma: float = 0.01, seed: int = SEED,
                  params: ExcavationParams | None = None) -> TerrainScene:
    """T1M terrain with the L-pit carved at zx120 + (4.0, 1.0)."""
    from scipy.signal import fftconvolve

    p = params or ExcavationParams()
    rng = np.random.default_rng(seed)
    xs = x0 + spacing * np.arange(n_side)
    ys = y0 + spacing * np.arange(n_side)
    Z = rng.normal(0.0, sigma, size=(n_side, n_side))           # Z[iy, ix]
    # getTerrainHeight (:183-226) ~ mean z over the 2-D disk of terrain_search_radius 0.5
    rc = int(round(0.5 / spacing))
    yy, xx = np.mgrid[-rc:rc + 1, -rc:rc + 1]
    disk = ((xx * spacing) ** 2 + (yy * spacing) ** 2 <= 0.5 ** 2 + 1e-12).astype(np.float64)
    num = fftconvolve(Z, disk, mode="same")
    den = fftconvolve(np.ones_like(Z), disk, mode="same")
    H = num / den

    def height_at(x, y):
        ix = np.clip(np.rint((np.asarray(x) - x0) / spacing).astype(np.int64), 0, n_side - 1)
        iy = np.clip(np.rint((np.asarray(y) - y0) / spacing).astype(np.int64), 0, n_side - 1)
        return H[iy, ix]

    boxes = excavation_boxes(p)
    cx, cy = p.offset_x, p.offset_y                      # zx120 at the map origin, yaw 0
    cz = float(height_at(cx, cy))
    # processExcavation (:457-485): keep ground points outside the excavation volume
    X, Y = np.meshgrid(xs, ys)
    xl, yl = X - cx, Y - cy
    inside = _inside_excavation(xl, yl, Z - H, boxes, p)
    keep = ~inside
    ground = np.stack([X[keep], Y[keep], Z[keep]], 1)
    # generateExcavatedSurface (:487-584)
    d = p.point_density
    omin_x = min(b[4] for b in boxes); omax_x = max(b[5] for b in boxes)
    omin_y = min(b[6] for b in boxes); omax_y = max(b[7] for b in boxes)
    n_x = int((omax_x - omin_x) / d) + 1
    n_y = int((omax_y - omin_y) / d) + 1
    I, J = np.meshgrid(np.arange(n_x + 1), np.arange(n_y + 1), indexing="ij")
    lx = omin_x + I.ravel() * d
    ly = omin_y + J.ravel() * d
    ins = _inside_any(lx, ly, boxes)
    bx, by = cx + lx[ins], cy + ly[ins]
    bottom = np.stack([bx, by, height_at(bx, by) - p.depth], 1)
    slope_offset = p.depth / math.tan(p.slope_angle * math.pi / 180.0)
    n_slope = int(slope_offset / d) + 1
    edge = _outer_edge(lx, ly, boxes, d)
    ex, ey = lx[edge], ly[edge]
    sx_pos = ~_inside_any(ex + d, ey, boxes)
    sx_neg = (~sx_pos) & (~_inside_any(ex - d, ey, boxes))
    sy_pos = ~_inside_any(ex, ey + d, boxes)
    sy_neg = (~sy_pos) & (~_inside_any(ex, ey - d, boxes))
    slopes = []
    for k in range(n_slope + 1):
        zr = k / n_slope
        off = slope_offset * zr
        xsl = ex + np.where(sx_pos, off, np.where(sx_neg, -off, 0.0))
        ysl = ey + np.where(sy_pos, off, np.where(sy_neg, -off, 0.0))
        gx, gy = cx + xsl, cy + ysl
        slopes.append(np.stack([gx, gy, height_at(gx, gy) - p.depth * (1.0 - zr)], 1))
    surface = np.concatenate([bottom] + slopes, 0)
    terr_xyz = np.concatenate([ground, surface], 0).astype(np.float32)
    n_ground = ground.shape[0]
    rgb = np.zeros((terr_xyz.shape[0], 3), np.uint8)
    rgb[:n_ground] = (255, 0, 0)
    rgb[n_ground:n_ground + bottom.shape[0]] = (0, 139, 0)
    rgb[n_ground + bottom.shape[0]:] = (144, 238, 144)
    terrain = _pack(terr_xyz, rgb)
    # generateExcavationArea (:350-455): bottom + slope k = 1 .. n_depth-1
    n_depth = int(p.depth / d)
    area_pts = [np.stack([bx, by, height_at(bx, by) - p.depth], 1)]
    for k in range(1, n_depth):
        zr = k / n_depth
        off = slope_offset * zr
        xsl = ex + np.where(sx_pos, off, np.where(sx_neg, -off, 0.0))
        ysl = ey + np.where(sy_pos, off, np.where(sy_neg, -off, 0.0))
        gx, gy = cx + xsl, cy + ysl
        # z uses the un-offset (x_global, y_global) terrain height (:389, :426)
        hz = height_at(cx + ex, cy + ey)
        area_pts.append(np.stack([gx, gy, hz - p.depth + k * d], 1))
    # the reference interleaves bottom/slope per lattice node; order does not matter for the
    # cells (radius queries), but keep bottom-first deterministic order
    area_xyz = np.concatenate(area_pts, 0).astype(np.float32)
    area = _pack(area_xyz, (255, 255, 0))
    zx = np.array([0.0 + 0.4, 0.0 + 0.5, 0.0 + 3.5, -math.pi / 6, 0.0])   # :348-352
    return TerrainScene(terrain, area, (cx, cy, cz), zx,
                        {"n_ground": n_ground, "n_surface": surface.shape[0],
                         "n_area": area_xyz.shape[0]})


# ----------------------------------------------------------------------------------------
# virtual_lidar setup (virtual_lidar.cpp:209-340): cells + normals
# ----------------------------------------------------------------------------------------
@dataclass
class Cells:
    xyz: np.ndarray       # (C, 3) float64
    normals: np.ndarray   # (C, 3) float32
    grid_bbox: np.ndarray  # grid_min_x, grid_max_x, grid_min_y, grid_max_y, ex_min_z, ex_max_z
    dims: tuple


def _pca_normals(pts: np.ndarray, radius: float) -> np.ndarray:
    """NormalEstimation (radius, PCA smallest eigenvector), flipped towards +z (:223-229)."""
    from scipy.spatial import cKDTree

    tree = cKDTree(pts)
    nb = tree.query_ball_point(pts, radius)
    out = np.full((pts.shape[0], 3), np.nan, np.float64)
    for i, idx in enumerate(nb):
        if len(idx) < 3:
            continue
        q = pts[idx]
        cov = np.cov(q.T, bias=True)
        w, v = np.linalg.eigh(cov)
        n = v[:, 0]
        # flipNormalTowardsViewpoint(0,0,0) then the reference's flip to +z
        if np.dot(-pts[i], n) < 0:
            n = -n
        if n[2] < 0:
            n = -n
        out[i] = n
    return out.astype(np.float32)


def excavation_cells(area: np.ndarray, grid_resolution: float = 0.1,
                     vertical_layers: int = 10) -> Cells:
    """generateExcavationGrid3D (:236-287) + computeCellSurfaceNormal (:301-340)."""
    from scipy.spatial import cKDTree

    pts = area[:, :3].astype(np.float64)
    gminx, gmaxx = pts[:, 0].min() - grid_resolution, pts[:, 0].max() + grid_resolution
    gminy, gmaxy = pts[:, 1].min() - grid_resolution, pts[:, 1].max() + grid_resolution
    zmin, zmax = pts[:, 2].min() - grid_resolution, pts[:, 2].max() + grid_resolution
    gw = int(math.ceil((gmaxx - gminx) / grid_resolution)) + 1
    gh = int(math.ceil((gmaxy - gminy) / grid_resolution)) + 1
    z_step = (zmax - zmin) / max(1, vertical_layers)
    tree = cKDTree(pts)
    I, J, K = np.meshgrid(np.arange(gh), np.arange(gw), np.arange(vertical_layers), indexing="ij")
    x = gminx + J.ravel() * grid_resolution
    y = gminy + I.ravel() * grid_resolution
    z = zmin + K.ravel() * z_step + z_step / 2.0
    q = np.stack([x, y, z], 1)
    qf = q.astype(np.float32).astype(np.float64)
    cnt = tree.query_ball_point(qf, grid_resolution * 1.5, return_length=True)
    valid = cnt > 0
    cells = q[valid]
    normals_pt = _pca_normals(pts, 1.5)
    nb = tree.query_ball_point(cells.astype(np.float32).astype(np.float64), 1.5)
    cn = np.zeros((cells.shape[0], 3), np.float64)
    cn[:, 2] = 1.0
    for i, idx in enumerate(nb):
        if not idx:
            continue
        v = normals_pt[idx].astype(np.float64)
        v = v[np.isfinite(v).all(1)]
        if v.shape[0] == 0:
            continue
        s = v.sum(0)
        nrm = math.sqrt(float(s @ s))
        if nrm > 1e-6:
            cn[i] = s / nrm
    return Cells(cells, cn.astype(np.float32),
                 np.array([gminx, gmaxx, gminy, gmaxy, zmin, zmax], np.float64), (gh, gw, vertical_layers))


# ----------------------------------------------------------------------------------------
# LiDAR-like clouds (C3) and the zx120 scan (aux cloud)
# ----------------------------------------------------------------------------------------
def lidar_cloud(n: int, sensor_height: float = 2.0, seed: int = SEED, rings: int = 64,
                el_lo_deg: float = -24.9, el_hi_deg: float = 2.0, r_lo: float = 1.0,
                r_hi: float = 40.0) -> np.ndarray:
    """(n, 4) float32 x, y, z, intensity (point_step 16) in the sensor frame."""
    rng = np.random.default_rng(seed)
    ring = rng.integers(0, rings, n)
    el = np.deg2rad(el_lo_deg + (el_hi_deg - el_lo_deg) * ring / (rings - 1))
    az = rng.uniform(-math.pi, math.pi, n)
    r = rng.uniform(r_lo, r_hi, n)
    down = el < 0
    r_ground = np.where(down, sensor_height / np.maximum(np.sin(-el), 1e-9), np.inf)
    r = np.minimum(r, r_ground)
    ce = np.cos(el)
    out = np.empty((n, 4), np.float32)
    out[:, 0] = r * ce * np.cos(az)
    out[:, 1] = r * ce * np.sin(az)
    out[:, 2] = r * np.sin(el)
    out[:, 3] = rng.uniform(0, 255, n)
    return out


def zx120_scan(scene: TerrainScene | None = None, seed: int = SEED, n_az: int = 938,
               rings: int = 64, noise: float = 0.02, max_range: float = 60.0) -> np.ndarray:
    """HDL-64-like scan (64 x 938) from the zx120 velodyne, sensor frame, (n, 4) float32.

    Extrinsic tf_zx120.launch.xml:3-4: (0.55, 0.4, 3.5), pitch 0.4363 rad; ray-cast
    analytically against the ground plane z = 0 and the pit bottom z = -depth."""
    rng = np.random.default_rng(seed + 1)
    p = ExcavationParams()
    boxes = excavation_boxes(p)
    el = np.deg2rad(np.linspace(-24.9, 2.0, rings))
    az = np.linspace(-math.pi, math.pi, n_az, endpoint=False)
    E, A = np.meshgrid(el, az, indexing="ij")
    d_s = np.stack([np.cos(E) * np.cos(A), np.cos(E) * np.sin(A), np.sin(E)], -1).reshape(-1, 3)
    pitch = 0.4363
    cp, sp = math.cos(pitch), math.sin(pitch)
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    d_m = d_s @ Ry.T
    o = np.array([0.55, 0.4, 3.5])
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.where(d_m[:, 2] < -1e-9, -o[2] / d_m[:, 2], np.inf)
        hit = o + t[:, None] * d_m
        inpit = _inside_any(hit[:, 0] - p.offset_x, hit[:, 1] - p.offset_y, boxes)
        t2 = np.where(d_m[:, 2] < -1e-9, (-p.depth - o[2]) / d_m[:, 2], np.inf)
    t = np.where(inpit, t2, t)
    ok = np.isfinite(t) & (t < max_range)
    r = t[ok] + rng.normal(0, noise, ok.sum())
    pts = d_s[ok] * r[:, None]
    out = np.zeros((pts.shape[0], 4), np.float32)
    out[:, :3] = pts
    out[:, 3] = 100.0
    return out


def numpy_voxel_mean(xyz: np.ndarray, leaf: float) -> np.ndarray:
    """Plain voxel mean for synthetic-input preparation only (not the product voxel)."""
    k = np.floor(xyz[:, :3] / leaf).astype(np.int64)
    _, inv = np.unique(k, axis=0, return_inverse=True)
    inv = inv.ravel()
    cnt = np.bincount(inv)
    out = np.stack([np.bincount(inv, xyz[:, a]) / cnt for a in range(3)], 1)
    return out.astype(np.float32)


def aux_cloud(seed: int = SEED) -> np.ndarray:
    """/zx120/filtered_points stand-in: zx120 scan cropped (15/10/10) and voxelised 0.2."""
    s = zx120_scan(seed=seed)
    m = (s[:, 0] > 0) & (s[:, 0] < 15) & (s[:, 1] > -10) & (s[:, 1] < 10) & (s[:, 2] > -1.5) & \
        (s[:, 2] < 10)
    v = numpy_voxel_mean(s[m], 0.2)
    out = np.zeros((v.shape[0], 8), np.float32)
    out[:, :3] = v
    out[:, 3] = 1.0
    return out


def candidate_lattice_size(target: int) -> int:
    """num_candidates giving a lattice with >= target survivors is found by the caller."""
    return int(math.ceil(math.sqrt(target))) ** 2
