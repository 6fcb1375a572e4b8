/* pcp_oracle_setup.c -- CPU restatement of virtual_lidar.cpp's excavation-area setup
 * (excavationAreaCallback :164-178 -> computeTerrainNormals :209-234 +
 * generateExcavationGrid3D :236-287 + isPointNearExcavation :289-299 +
 * computeCellSurfaceNormal :301-340).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).
 * PARITY UNPINNED: pcl::NormalEstimation / pcl::eigen33 / FLANN are absent from this image;
 * their published algorithms are restated here (PCL 1.12.1, FLANN 1.9.1):
 *  - KdTreeFLANN::radiusSearch: neighbours are the points with the L2_Simple<float> distance
 *    ((0 + dx^2) + dy^2) + dz^2 < (float)(r*r), query rounded to float, returned sorted by
 *    (distance, index) ascending (FLANN RadiusResultSet, sorted = true).
 *  - NormalEstimation::computePointNormal: < 3 neighbours -> NaN normal; else
 *    computeMeanAndCovarianceMatrix in float with the shifted accumulation (K = the first
 *    neighbour), covariance = E[xx] - E[x]E[x] per entry; solvePlaneParameters ->
 *    eigen33 (scale by max |entry|, computeRoots closed form, smallest root, largest of the
 *    three row cross products); flipNormalTowardsViewpoint with viewpoint (0, 0, 0).
 *  - then the reference's own flip to normal_z >= 0 (:223-229).
 */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pcp_oracle.h"

typedef struct {
    float d;
    int64_t i;
} nb_t;

static int nb_cmp(const void *a, const void *b) {
    const nb_t *x = (const nb_t *)a, *y = (const nb_t *)b;
    if (x->d < y->d) return -1;
    if (x->d > y->d) return 1;
    return (x->i > y->i) - (x->i < y->i);
}

/* brute-force radius search with FLANN's predicate and result order */
static int64_t radius_search(const float *pts, int64_t n, int64_t stride, float qx, float qy,
                             float qz, double radius, nb_t *out) {
    const float r2 = (float)(radius * radius);
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        const float d0 = qx - p[0], d1 = qy - p[1], d2 = qz - p[2];
        float acc = 0.0f;
        acc = acc + d0 * d0;
        acc = acc + d1 * d1;
        acc = acc + d2 * d2;
        if (acc < r2) {
            out[m].d = acc;
            out[m].i = i;
            ++m;
        }
    }
    qsort(out, (size_t)m, sizeof(nb_t), nb_cmp);
    return m;
}

/* pcl::computeRoots2 */
static void roots2(float b, float c, float r[3]) {
    r[0] = 0.0f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0f) d = 0.0f;
    const float sd = sqrtf(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}

/* pcl::computeRoots (symmetric 3x3, float) */
static void roots3(const float m[3][3], float r[3]) {
    const float c0 = m[0][0] * m[1][1] * m[2][2] + 2.0f * m[0][1] * m[0][2] * m[1][2] -
                     m[0][0] * m[1][2] * m[1][2] - m[1][1] * m[0][2] * m[0][2] -
                     m[2][2] * m[0][1] * m[0][1];
    const float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] -
                     m[0][2] * m[0][2] + m[1][1] * m[2][2] - m[1][2] * m[1][2];
    const float c2 = m[0][0] + m[1][1] + m[2][2];
    if (fabsf(c0) < FLT_EPSILON) {
        roots2(c2, c1, r);
        return;
    }
    const float s_inv3 = (float)(1.0 / 3.0);
    const float s_sqrt3 = sqrtf(3.0f);
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    const float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.0f) q = 0.0f;
    const float rho = sqrtf(-a_over_3);
    const float theta = atan2f(sqrtf(-q), half_b) * s_inv3;
    const float ct = cosf(theta), st = sinf(theta);
    r[0] = c2_over_3 + 2.0f * rho * ct;
    r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
    r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
    float t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
    if (r[1] >= r[2]) {
        t = r[1]; r[1] = r[2]; r[2] = t;
        if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
    }
    if (r[0] <= 0.0f) roots2(c2, c1, r);
}

static void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* pcl::eigen33 (smallest eigenvalue's eigenvector) */
static void eigen33_min(const float cov[3][3], float ev[3]) {
    float scale = 0.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale = fmaxf(scale, fabsf(cov[i][j]));
    if (scale <= FLT_MIN) scale = 1.0f;
    float m[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i][j] = cov[i][j] / scale;
    float r[3];
    roots3(m, r);
    for (int i = 0; i < 3; ++i) m[i][i] -= r[0];
    float v1[3], v2[3], v3[3];
    cross3(m[0], m[1], v1);
    cross3(m[0], m[2], v2);
    cross3(m[1], m[2], v3);
    const float l1 = v1[0] * v1[0] + v1[1] * v1[1] + v1[2] * v1[2];
    const float l2 = v2[0] * v2[0] + v2[1] * v2[1] + v2[2] * v2[2];
    const float l3 = v3[0] * v3[0] + v3[1] * v3[1] + v3[2] * v3[2];
    const float *v;
    float l;
    if (l1 >= l2 && l1 >= l3) { v = v1; l = l1; }
    else if (l2 >= l1 && l2 >= l3) { v = v2; l = l2; }
    else { v = v3; l = l3; }
    const float s = sqrtf(l);
    for (int a = 0; a < 3; ++a) ev[a] = v[a] / s;
}

void orc_area_normals(const float *pts, int64_t n, int64_t stride_floats, double radius,
                      float *normals3) {
    nb_t *nb = (nb_t *)malloc(sizeof(nb_t) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) {
        const float *q = pts + i * stride_floats;
        float *o = normals3 + 3 * i;
        const int64_t m = radius_search(pts, n, stride_floats, q[0], q[1], q[2], radius, nb);
        if (m < 3) {
            o[0] = o[1] = o[2] = NAN;
            continue;
        }
        const float *k0 = pts + nb[0].i * stride_floats;
        const float kx = k0[0], ky = k0[1], kz = k0[2];
        float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t t = 0; t < m; ++t) {
            const float *p = pts + nb[t].i * stride_floats;
            const float x = p[0] - kx, y = p[1] - ky, z = p[2] - kz;
            acc[0] += x * x;
            acc[1] += x * y;
            acc[2] += x * z;
            acc[3] += y * y;
            acc[4] += y * z;
            acc[5] += z * z;
            acc[6] += x;
            acc[7] += y;
            acc[8] += z;
        }
        for (int a = 0; a < 9; ++a) acc[a] /= (float)m;
        float cov[3][3];
        cov[0][0] = acc[0] - acc[6] * acc[6];
        cov[0][1] = acc[1] - acc[6] * acc[7];
        cov[0][2] = acc[2] - acc[6] * acc[8];
        cov[1][1] = acc[3] - acc[7] * acc[7];
        cov[1][2] = acc[4] - acc[7] * acc[8];
        cov[2][2] = acc[5] - acc[8] * acc[8];
        cov[1][0] = cov[0][1];
        cov[2][0] = cov[0][2];
        cov[2][1] = cov[1][2];
        float ev[3];
        eigen33_min(cov, ev);
        /* flipNormalTowardsViewpoint, viewpoint (0,0,0) */
        const float ct = (0.0f - q[0]) * ev[0] + (0.0f - q[1]) * ev[1] + (0.0f - q[2]) * ev[2];
        if (ct < 0.0f)
            for (int a = 0; a < 3; ++a) ev[a] = -ev[a];
        /* computeTerrainNormals: normal_z >= 0 */
        if (ev[2] < 0.0f)
            for (int a = 0; a < 3; ++a) ev[a] = -ev[a];
        o[0] = ev[0];
        o[1] = ev[1];
        o[2] = ev[2];
    }
    free(nb);
}

int64_t orc_excavation_grid(const float *pts, int64_t n, int64_t stride_floats,
                            double grid_resolution, int32_t vertical_layers,
                            const float *area_normals3, double *cells_xyz, float *cells_nrm,
                            int64_t cap, double grid_bbox[6], int32_t dims[3]) {
    if (n <= 0) return 0;
    double gx0 = DBL_MAX, gy0 = DBL_MAX, gz0 = DBL_MAX;
    double gx1 = -DBL_MAX, gy1 = -DBL_MAX, gz1 = -DBL_MAX;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride_floats;
        gx0 = fmin(gx0, (double)p[0]);
        gx1 = fmax(gx1, (double)p[0]);
        gy0 = fmin(gy0, (double)p[1]);
        gy1 = fmax(gy1, (double)p[1]);
        gz0 = fmin(gz0, (double)p[2]);
        gz1 = fmax(gz1, (double)p[2]);
    }
    const double margin = grid_resolution;
    gx0 -= margin; gx1 += margin;
    gy0 -= margin; gy1 += margin;
    gz0 -= margin; gz1 += margin;
    const int gw = (int)ceil((gx1 - gx0) / grid_resolution) + 1;
    const int gh = (int)ceil((gy1 - gy0) / grid_resolution) + 1;
    const double z_range = gz1 - gz0;
    const double z_step = z_range / (vertical_layers > 1 ? vertical_layers : 1);
    grid_bbox[0] = gx0; grid_bbox[1] = gx1;
    grid_bbox[2] = gy0; grid_bbox[3] = gy1;
    grid_bbox[4] = gz0; grid_bbox[5] = gz1;
    dims[0] = gh; dims[1] = gw; dims[2] = vertical_layers;
    nb_t *nb = (nb_t *)malloc(sizeof(nb_t) * (size_t)n);
    int64_t nc = 0;
    for (int i = 0; i < gh; ++i)
        for (int j = 0; j < gw; ++j)
            for (int k = 0; k < vertical_layers; ++k) {
                const double x = gx0 + j * grid_resolution;
                const double y = gy0 + i * grid_resolution;
                const double z = gz0 + k * z_step + z_step / 2.0;
                const float qx = (float)x, qy = (float)y, qz = (float)z;
                if (radius_search(pts, n, stride_floats, qx, qy, qz, grid_resolution * 1.5, nb) <= 0)
                    continue;
                /* GridCell default normal (0, 0, 1); computeCellSurfaceNormal */
                double nx = 0.0, ny = 0.0, nz = 1.0;
                if (area_normals3) {
                    const int64_t m = radius_search(pts, n, stride_floats, qx, qy, qz, 1.5, nb);
                    double sx = 0.0, sy = 0.0, sz = 0.0;
                    int valid = 0;
                    for (int64_t t = 0; t < m; ++t) {
                        const float *v = area_normals3 + 3 * nb[t].i;
                        if (isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2])) {
                            sx += v[0];
                            sy += v[1];
                            sz += v[2];
                            ++valid;
                        }
                    }
                    if (valid > 0) {
                        const double norm = sqrt(sx * sx + sy * sy + sz * sz);
                        if (norm > 1e-6) {
                            nx = sx / norm;
                            ny = sy / norm;
                            nz = sz / norm;
                        }
                    }
                }
                if (nc < cap) {
                    cells_xyz[3 * nc + 0] = x;
                    cells_xyz[3 * nc + 1] = y;
                    cells_xyz[3 * nc + 2] = z;
                    cells_nrm[3 * nc + 0] = (float)nx;
                    cells_nrm[3 * nc + 1] = (float)ny;
                    cells_nrm[3 * nc + 2] = (float)nz;
                }
                ++nc;
            }
    free(nb);
    return nc;
}

/* ==========================================================================================
 * excavated_surface_generator.cpp (ExcavationTerrainGenerator) -- the carve in front of the
 * ray-trace.  getTerrainHeight (:183-226) here is a brute-force restatement of the KdTreeFLANN
 * it rebuilds per call: 3-D radius search from (x, y, 0) with FLANN's float predicate (non-
 * finite points are not in the tree), a 2-D distance filter in double, the mean z summed in
 * the distance-sorted result order; else the nearest point's z (nearestKSearch k = 1: smallest
 * float distance, lowest index on a tie); else 0.
 * ========================================================================================== */
double orc_terrain_height(const float *pts, int64_t n, int64_t stride_floats, double x, double y,
                          double radius) {
    if (n <= 0) return 0.0;
    const float qx = (float)x, qy = (float)y, qz = 0.0f;
    nb_t *nb = (nb_t *)malloc(sizeof(nb_t) * (size_t)n);
    const float r2 = (float)(radius * radius);
    int64_t m = 0, best = -1;
    float bestd = INFINITY;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride_floats;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        const float d0 = qx - p[0], d1 = qy - p[1], d2 = qz - p[2];
        float acc = 0.0f;
        acc = acc + d0 * d0;
        acc = acc + d1 * d1;
        acc = acc + d2 * d2;
        if (acc < r2) {
            nb[m].d = acc;
            nb[m].i = i;
            ++m;
        }
        if (acc < bestd) {
            bestd = acc;
            best = i;
        }
    }
    qsort(nb, (size_t)m, sizeof(nb_t), nb_cmp);
    double sum_z = 0.0;
    int valid = 0;
    for (int64_t t = 0; t < m; ++t) {
        const float *p = pts + nb[t].i * stride_floats;
        const double dx = p[0] - x, dy = p[1] - y;
        if (sqrt(dx * dx + dy * dy) <= radius) {
            sum_z += p[2];
            ++valid;
        }
    }
    free(nb);
    if (valid > 0) return sum_z / valid;
    if (best >= 0) return pts[best * stride_floats + 2];
    return 0.0;
}

typedef struct {
    double cx, cy, len, wid, min_x, max_x, min_y, max_y;
} exc_box;

/* getExcavationBoxes (:138-181) */
static int exc_boxes(const orc_exc_params *p, exc_box b[2]) {
    if (p->l_shape_enabled) {
        b[0].cx = 0.0;
        b[0].cy = -p->arm1_length / 2.0;
        b[0].len = p->arm1_width;
        b[0].wid = p->arm1_length;
        b[1].cx = p->arm2_length / 2.0;
        b[1].cy = -p->arm1_length + p->arm2_width / 2.0;
        b[1].len = p->arm2_length;
        b[1].wid = p->arm2_width;
        for (int k = 0; k < 2; ++k) {
            b[k].min_x = b[k].cx - b[k].len / 2.0;
            b[k].max_x = b[k].cx + b[k].len / 2.0;
            b[k].min_y = b[k].cy - b[k].wid / 2.0;
            b[k].max_y = b[k].cy + b[k].wid / 2.0;
        }
        return 2;
    }
    b[0].cx = 0.0;
    b[0].cy = 0.0;
    b[0].len = p->length;
    b[0].wid = p->width;
    b[0].min_x = -p->length / 2.0;
    b[0].max_x = p->length / 2.0;
    b[0].min_y = -p->width / 2.0;
    b[0].max_y = p->width / 2.0;
    return 1;
}

/* isInsideAnyBox (:229-237) */
static int inside_any(double x, double y, const exc_box *b, int nb) {
    for (int k = 0; k < nb; ++k)
        if (x >= b[k].min_x && x <= b[k].max_x && y >= b[k].min_y && y <= b[k].max_y) return 1;
    return 0;
}

/* isOuterEdge (:240-258) */
static int outer_edge(double x, double y, const exc_box *b, int nb, double tol) {
    if (!inside_any(x, y, b, nb)) return 0;
    int out = 0;
    if (!inside_any(x + tol, y, b, nb)) out = 1;
    if (!inside_any(x - tol, y, b, nb)) out = 1;
    if (!inside_any(x, y + tol, b, nb)) out = 1;
    if (!inside_any(x, y - tol, b, nb)) out = 1;
    return out;
}

/* isInsideExcavationArea (:328-348) */
static int inside_exc(double xl, double yl, double zrel, const exc_box *b, int nb,
                      const orc_exc_params *p, double slope_rad) {
    if (zrel < -p->depth || zrel > 0) return 0;
    const double slope_offset = p->depth / tan(slope_rad);
    const double slope_factor = (p->depth + zrel) / p->depth;
    const double cur = slope_offset * slope_factor;
    for (int k = 0; k < nb; ++k) {
        const double dx = xl - b[k].cx, dy = yl - b[k].cy;
        const double hl = b[k].len / 2.0 + cur, hw = b[k].wid / 2.0 + cur;
        if (fabs(dx) <= hl && fabs(dy) <= hw) return 1;
    }
    return 0;
}

/* PointXYZRGB rgb float of (r, g, b), alpha 255 */
static float pack_rgb(unsigned r, unsigned g, unsigned b) {
    const uint32_t v = b | (g << 8) | (r << 16) | (255u << 24);
    float f;
    memcpy(&f, &v, 4);
    return f;
}

static void put4(float *o, int64_t i, int64_t cap, double x, double y, double z, float rgb) {
    if (i >= cap) return;
    o[4 * i + 0] = (float)x;
    o[4 * i + 1] = (float)y;
    o[4 * i + 2] = (float)z;
    o[4 * i + 3] = rgb;
}

void orc_excavate(const float *pts, int64_t n, int64_t stride_floats, const orc_exc_params *p,
                  const double t[3], const double q[4], uint8_t *keep, float *surf,
                  int64_t cap_surf, int64_t *n_surf, float *area, int64_t cap_area,
                  int64_t *n_area, double pose_out[4]) {
    /* tf2::Matrix3x3::setRotation (quaternion x, y, z, w) and Transform * (ox, oy, 0) */
    const double qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    const double d = qx * qx + qy * qy + qz * qz + qw * qw;
    const double s = 2.0 / d;
    const double xs = qx * s, ys = qy * s, zs = qz * s;
    const double wx = qw * xs, wy = qw * ys, wz = qw * zs;
    const double xx = qx * xs, xy = qx * ys, xz = qx * zs;
    const double yy = qy * ys, yz = qy * zs, zz = qz * zs;
    const double m[3][3] = {{1.0 - (yy + zz), xy - wz, xz + wy},
                            {xy + wz, 1.0 - (xx + zz), yz - wx},
                            {xz - wy, yz + wx, 1.0 - (xx + yy)}};
    const double ox = p->offset_x, oy = p->offset_y, oz = 0.0;
    const double cx = (m[0][0] * ox + m[0][1] * oy + m[0][2] * oz) + t[0];
    const double cy = (m[1][0] * ox + m[1][1] * oy + m[1][2] * oz) + t[1];
    const double r = p->terrain_search_radius;
    const double cz = orc_terrain_height(pts, n, stride_floats, cx, cy, r);
    /* Matrix3x3::getRPY -> getEulerYPR, solution 1 */
    double yaw;
    if (fabs(m[2][0]) >= 1) {
        yaw = 0.0;
    } else {
        const double pitch = -asin(m[2][0]);
        yaw = atan2(m[1][0] / cos(pitch), m[0][0] / cos(pitch));
    }
    if (pose_out) {
        pose_out[0] = cx;
        pose_out[1] = cy;
        pose_out[2] = cz;
        pose_out[3] = yaw;
    }
    exc_box b[2];
    const int nb = exc_boxes(p, b);
    const double slope_rad = p->slope_angle_deg * M_PI / 180.0;
    const double slope_offset = p->depth / tan(slope_rad);
    /* processExcavation (:451-485): points provably outside every widened box keep without a
     * terrain-height query (inside needs |dx| <= half + offset with offset <= slope_offset) */
    const double cyw = cos(-yaw), syw = sin(-yaw);
    for (int64_t i = 0; i < n; ++i) {
        const float *pt = pts + i * stride_floats;
        const double dx = pt[0] - cx, dy = pt[1] - cy;
        const double xl = dx * cyw - dy * syw;
        const double yl = dx * syw + dy * cyw;
        int maybe = 0;
        for (int k = 0; k < nb; ++k)
            if (fabs(xl - b[k].cx) <= b[k].len / 2.0 + slope_offset &&
                fabs(yl - b[k].cy) <= b[k].wid / 2.0 + slope_offset)
                maybe = 1;
        int inside = 0;
        if (maybe) {
            const double h = orc_terrain_height(pts, n, stride_floats, pt[0], pt[1], r);
            inside = inside_exc(xl, yl, pt[2] - h, b, nb, p, slope_rad);
        }
        keep[i] = inside ? 0 : 1;
    }
    double mnx = DBL_MAX, mxx = -DBL_MAX, mny = DBL_MAX, mxy = -DBL_MAX;
    for (int k = 0; k < nb; ++k) {
        mnx = fmin(mnx, b[k].min_x);
        mxx = fmax(mxx, b[k].max_x);
        mny = fmin(mny, b[k].min_y);
        mxy = fmax(mxy, b[k].max_y);
    }
    const double dens = p->point_density;
    const int n_x = (int)((mxx - mnx) / dens) + 1;
    const int n_y = (int)((mxy - mny) / dens) + 1;
    const double cyaw = cos(yaw), syaw = sin(yaw);
    /* generateExcavatedSurface (:487-584): bottom, then the outer-wall slopes */
    int64_t ns = 0;
    const float rgb_bottom = pack_rgb(0, 139, 0), rgb_slope = pack_rgb(144, 238, 144);
    for (int i = 0; i <= n_x; ++i)
        for (int j = 0; j <= n_y; ++j) {
            const double xl = mnx + i * dens, yl = mny + j * dens;
            if (!inside_any(xl, yl, b, nb)) continue;
            const double xg = cx + xl * cyaw - yl * syaw;
            const double yg = cy + xl * syaw + yl * cyaw;
            const double h = orc_terrain_height(pts, n, stride_floats, xg, yg, r);
            put4(surf, ns++, cap_surf, xg, yg, h - p->depth, rgb_bottom);
        }
    const int n_slope = (int)(slope_offset / dens) + 1;
    for (int i = 0; i <= n_x; ++i)
        for (int j = 0; j <= n_y; ++j) {
            const double xl = mnx + i * dens, yl = mny + j * dens;
            if (!outer_edge(xl, yl, b, nb, dens)) continue;
            for (int k = 0; k <= n_slope; ++k) {
                const double z_ratio = (double)k / n_slope;
                const double off = slope_offset * z_ratio;
                double ofx = 0.0, ofy = 0.0;
                if (!inside_any(xl + dens, yl, b, nb)) ofx = off;
                else if (!inside_any(xl - dens, yl, b, nb)) ofx = -off;
                if (!inside_any(xl, yl + dens, b, nb)) ofy = off;
                else if (!inside_any(xl, yl - dens, b, nb)) ofy = -off;
                const double xs2 = xl + ofx, ys2 = yl + ofy;
                const double xg = cx + xs2 * cyaw - ys2 * syaw;
                const double yg = cy + xs2 * syaw + ys2 * cyaw;
                const double h = orc_terrain_height(pts, n, stride_floats, xg, yg, r);
                put4(surf, ns++, cap_surf, xg, yg, h - p->depth * (1.0 - z_ratio), rgb_slope);
            }
        }
    *n_surf = ns;
    /* generateExcavationArea (:350-455) */
    int64_t na = 0;
    const int n_depth = (int)(p->depth / dens);
    const float rgb_abot = pack_rgb(255, 255, 0), rgb_aslope = pack_rgb(200, 200, 0);
    for (int i = 0; i <= n_x; ++i)
        for (int j = 0; j <= n_y; ++j) {
            const double xl = mnx + i * dens, yl = mny + j * dens;
            if (!inside_any(xl, yl, b, nb)) continue;
            const double xg = cx + xl * cyaw - yl * syaw;
            const double yg = cy + xl * syaw + yl * cyaw;
            const double h = orc_terrain_height(pts, n, stride_floats, xg, yg, r);
            put4(area, na++, cap_area, xg, yg, h - p->depth, rgb_abot);
            if (!outer_edge(xl, yl, b, nb, dens)) continue;
            for (int k = 1; k < n_depth; ++k) {
                const double z_ratio = (double)k / n_depth;
                const double off = slope_offset * z_ratio;
                double ofx = 0.0, ofy = 0.0;
                if (!inside_any(xl + dens, yl, b, nb)) ofx = off;
                else if (!inside_any(xl - dens, yl, b, nb)) ofx = -off;
                if (!inside_any(xl, yl + dens, b, nb)) ofy = off;
                else if (!inside_any(xl, yl - dens, b, nb)) ofy = -off;
                const double xs2 = xl + ofx, ys2 = yl + ofy;
                const double xg2 = cx + xs2 * cyaw - ys2 * syaw;
                const double yg2 = cy + xs2 * syaw + ys2 * cyaw;
                put4(area, na++, cap_area, xg2, yg2, h - p->depth + k * dens, rgb_aslope);
            }
        }
    *n_area = na;
}

/* ==========================================================================================
 * calc_drivable_area.cpp robotCloudCallback (:67-226): tf2::doTransform (Eigen float, the
 * order of orc_transform_rgb), (int) truncating bins, per-cell z lists, then the rules.
 * ========================================================================================== */
void orc_drivable_area(const float *pts, int64_t n, int64_t stride_floats, const double t[3],
                       const double q[4], double robot_x, double robot_y, double start_x,
                       double start_y, double res, double map_w, double map_h,
                       double max_gradient, int32_t min_points, double clear_r, int8_t *grid,
                       int32_t dims[2], double origin[2]) {
    const int gw = (int)(map_w / res), gh = (int)(map_h / res);
    dims[0] = gw;
    dims[1] = gh;
    const double ox = robot_x - map_w / 2.0, oy = robot_y - map_h / 2.0;
    origin[0] = ox;
    origin[1] = oy;
    if (n <= 0 || gw <= 0 || gh <= 0) return;
    const int64_t nc = (int64_t)gw * gh;
    int64_t *cnt = (int64_t *)calloc((size_t)nc, sizeof(int64_t));
    float *zmin = (float *)malloc(sizeof(float) * (size_t)nc);
    float *zmax = (float *)malloc(sizeof(float) * (size_t)nc);
    /* Eigen::Quaternionf(w,x,y,z).toRotationMatrix() + translation, in float */
    const float qx = (float)q[0], qy = (float)q[1], qz = (float)q[2], qw = (float)q[3];
    const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
    const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
    const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const float m[3][3] = {{1.0f - (tyy + tzz), txy - twz, txz + twy},
                           {txy + twz, 1.0f - (txx + tzz), tyz - twx},
                           {txz - twy, tyz + twx, 1.0f - (txx + tyy)}};
    const float T[3] = {(float)t[0], (float)t[1], (float)t[2]};
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride_floats;
        float o[3];
        for (int a = 0; a < 3; ++a) o[a] = ((m[a][0] * p[0] + m[a][1] * p[1]) + m[a][2] * p[2]) + T[a];
        if (!isfinite(o[0]) || !isfinite(o[1]) || !isfinite(o[2])) continue;
        const int gx = (int)((o[0] - ox) / res), gy = (int)((o[1] - oy) / res);
        if (gx >= 0 && gx < gw && gy >= 0 && gy < gh) {
            const int64_t c = (int64_t)gy * gw + gx;
            if (cnt[c] == 0) {
                zmin[c] = zmax[c] = o[2];
            } else {
                if (o[2] < zmin[c]) zmin[c] = o[2];   /* std::min_element: first smallest */
                if (zmax[c] < o[2]) zmax[c] = o[2];   /* std::max_element: first largest */
            }
            ++cnt[c];
        }
    }
    for (int y = 0; y < gh; ++y)
        for (int x = 0; x < gw; ++x) {
            const int64_t c = (int64_t)y * gw + x;
            const double cx = ox + (x + 0.5) * res, cy = oy + (y + 0.5) * res;
            const double dist = sqrt(pow(cx - start_x, 2) + pow(cy - start_y, 2));
            if (dist <= clear_r) {
                grid[c] = 0;
            } else if (cnt[c] == 0 || (size_t)cnt[c] < (size_t)min_points) {
                grid[c] = -1;
            } else {
                float g = 0.0f;
                if (cnt[c] >= 2) g = (zmax[c] - zmin[c]) / res;
                grid[c] = g > max_gradient ? 100 : 0;
            }
        }
    free(cnt);
    free(zmin);
    free(zmax);
}
