/*
 * pcp_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (see pcp_oracle.h for the rules, and for why parity is unpinned).
 *
 * Every function cites the reference lines it restates.  Third-party semantics:
 *  - FLANN 1.9.1 KDTreeSingleIndex + L2_Simple<float> behind PCL 1.12.1
 *    KdTreeFLANN::radiusSearch: a point is returned iff
 *        ((0 + dx*dx) + dy*dy) + dz*dz  <  (float)(radius*radius)      (all float, dx = q - p)
 *    with the query point already rounded to float (PointXYZRGB fields).  Any exact
 *    spatial structure returns the same set, so this file uses a plain uniform grid.
 *  - PCL 1.12.1 VoxelGrid<PointXYZ>::applyFilter with downsample_all_data_=true and
 *    min_points_per_voxel_=0 (keying, overflow guard, ascending-index output).
 *  - Eigen 3.4: Quaternionf::toRotationMatrix and Affine3f * Vector3f evaluated as the
 *    homogeneous 4x4 product ((m0*x + m1*y) + m2*z) + t  (column-major packet product,
 *    no FMA), as called by tf2_sensor_msgs::doTransform(PointCloud2).
 */
#include "pcp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* virtual_lidar.cpp:100-114 */
#define VL_MIN_ELEVATION (-85.0 * M_PI / 180.0)
#define VL_MAX_ELEVATION (85.0 * M_PI / 180.0)

static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n > 0 ? n : 1; }
int orc_get_threads(void) { return g_threads; }

/* ================================================================================ */
/* pointcloud_filter.cpp:106-116 (cropFrontArea hot loop)                           */
/* ================================================================================ */
int64_t orc_crop_box(const float *pts, int64_t n, int64_t stride, const double box[6],
                     uint32_t *kept)
{
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        /* float promoted to double, compared with the double parameters (:111-113) */
        if ((double)p[0] > box[0] && (double)p[0] < box[1] &&
            (double)p[1] > box[2] && (double)p[1] < box[3] &&
            (double)p[2] > box[4] && (double)p[2] < box[5]) {
            kept[m++] = (uint32_t)i;
        }
    }
    return m;
}

/* ================================================================================ */
/* pointcloud_filter.cpp:122-139 -> pcl::VoxelGrid<PointXYZ>::applyFilter [upstream] */
/* ================================================================================ */
typedef struct { uint32_t idx; uint32_t cloud_index; } vg_pair;

static int vg_cmp(const void *a, const void *b)
{
    const vg_pair *x = (const vg_pair *)a, *y = (const vg_pair *)b;
    if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
    /* PCL's spreadsort is not stable; the in-voxel order only moves the float centroid
     * by rounding (tolerance 1e-5 m in tests).  We fix input order. */
    return x->cloud_index < y->cloud_index ? -1 : (x->cloud_index > y->cloud_index);
}

int64_t orc_voxel_grid(const float *pts, int64_t n, int64_t stride, float leaf,
                       float *out_xyz, uint32_t *out_idx, uint32_t *out_count,
                       int *passthrough)
{
    *passthrough = 0;
    if (n <= 0) return 0;   /* downsampleCloud returns the empty input (:125-127) */
    /* setLeafSize(float,float,float): the double parameter is narrowed; inverse is 1/leaf
     * in float (Eigen::Array4f::Ones() / leaf_size_). */
    const float inv = 1.0f / leaf;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    int64_t nfin = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        ++nfin;
        for (int a = 0; a < 3; ++a) {
            if (p[a] < mn[a]) mn[a] = p[a];
            if (p[a] > mx[a]) mx[a] = p[a];
        }
    }
    if (nfin == 0) return 0;
    /* overflow guard: int64 of float product, +1 */
    int64_t dxl = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    int64_t dyl = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    int64_t dzl = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dxl * dyl * dzl > (int64_t)INT32_MAX) {
        *passthrough = 1;             /* output = *input_ */
        for (int64_t i = 0; i < n; ++i) {
            out_xyz[3 * i + 0] = pts[i * stride + 0];
            out_xyz[3 * i + 1] = pts[i * stride + 1];
            out_xyz[3 * i + 2] = pts[i * stride + 2];
        }
        return n;
    }
    int min_b[3], max_b[3], div_b[3];
    for (int a = 0; a < 3; ++a) {
        min_b[a] = (int)floorf(mn[a] * inv);
        max_b[a] = (int)floorf(mx[a] * inv);
        div_b[a] = max_b[a] - min_b[a] + 1;
    }
    const int mul1 = div_b[0], mul2 = div_b[0] * div_b[1];
    vg_pair *iv = (vg_pair *)malloc((size_t)nfin * sizeof(vg_pair));
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        int ijk0 = (int)(floorf(p[0] * inv) - (float)min_b[0]);
        int ijk1 = (int)(floorf(p[1] * inv) - (float)min_b[1]);
        int ijk2 = (int)(floorf(p[2] * inv) - (float)min_b[2]);
        int idx = ijk0 + ijk1 * mul1 + ijk2 * mul2;
        iv[m].idx = (uint32_t)idx;
        iv[m].cloud_index = (uint32_t)i;
        ++m;
    }
    qsort(iv, (size_t)m, sizeof(vg_pair), vg_cmp);
    int64_t total = 0, index = 0;
    while (index < m) {
        int64_t j = index + 1;
        while (j < m && iv[j].idx == iv[index].idx) ++j;
        /* CentroidPoint<PointXYZ>: float accumulation of x,y,z, then / (float)n */
        float sx = 0.f, sy = 0.f, sz = 0.f;
        for (int64_t l = index; l < j; ++l) {
            const float *p = pts + (int64_t)iv[l].cloud_index * stride;
            sx += p[0]; sy += p[1]; sz += p[2];
        }
        const float cnt = (float)(j - index);
        out_xyz[3 * total + 0] = sx / cnt;
        out_xyz[3 * total + 1] = sy / cnt;
        out_xyz[3 * total + 2] = sz / cnt;
        out_idx[total] = iv[index].idx;
        out_count[total] = (uint32_t)(j - index);
        ++total;
        index = j;
    }
    free(iv);
    return total;
}

/* ================================================================================ */
/* pointcloud_merger.cpp:354-394 (processRobotCloud): tf2::doTransform + colour        */
/* ================================================================================ */
void orc_transform_rgb(const float *pts, int64_t n, int64_t stride, const double t[3],
                       const double q[4], uint8_t r, uint8_t g, uint8_t b, float *out8)
{
    /* Eigen::Quaternion<float>(w,x,y,z) from the double message fields */
    const float qx = (float)q[0], qy = (float)q[1], qz = (float)q[2], qw = (float)q[3];
    const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
    const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
    const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const float m00 = 1.0f - (tyy + tzz), m01 = txy - twz, m02 = txz + twy;
    const float m10 = txy + twz, m11 = 1.0f - (txx + tzz), m12 = tyz - twx;
    const float m20 = txz - twy, m21 = tyz + twx, m22 = 1.0f - (txx + tyy);
    const float Tx = (float)t[0], Ty = (float)t[1], Tz = (float)t[2];
    /* PointXYZRGB rgba word: b | g<<8 | r<<16 | a<<24, a = 255 (default ctor) */
    const uint32_t rgba = (uint32_t)b | ((uint32_t)g << 8) | ((uint32_t)r << 16) | (255u << 24);
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        const float x = p[0], y = p[1], z = p[2];
        float *o = out8 + 8 * i;
        o[0] = ((m00 * x + m01 * y) + m02 * z) + Tx;
        o[1] = ((m10 * x + m11 * y) + m12 * z) + Ty;
        o[2] = ((m20 * x + m21 * y) + m22 * z) + Tz;
        o[3] = 1.0f;
        memcpy(&o[4], &rgba, 4);
        o[5] = 0.f; o[6] = 0.f; o[7] = 0.f;
    }
}

/* ================================================================================ */
/* Exact radius search (replaces KdTreeFLANN for the checker)                       */
/* ================================================================================ */
struct orc_cloud {
    const orc_kdtree *kd;   /* non-NULL: radius queries answered by the restated KdTreeFLANN
                               (pcp_flann.c) instead of the exact grid scan */
    int64_t n;              /* finite points kept */
    float *p;               /* 3 floats per point, sorted by cell */
    uint32_t *start;        /* ncell + 1 */
    double ox, oy, oz, g;
    int64_t nx, ny, nz;
};

orc_cloud *orc_cloud_build(const float *pts, int64_t n, int64_t stride)
{
    orc_cloud *c = (orc_cloud *)calloc(1, sizeof(orc_cloud));
    double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    int64_t nf = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;  /* PCL drops NaN */
        ++nf;
        for (int a = 0; a < 3; ++a) {
            if (p[a] < mn[a]) mn[a] = p[a];
            if (p[a] > mx[a]) mx[a] = p[a];
        }
    }
    c->n = nf;
    if (nf == 0) { c->nx = c->ny = c->nz = 1; c->g = 1.0;
        c->start = (uint32_t *)calloc(2, sizeof(uint32_t)); c->p = NULL; return c; }
    double g = 0.25;
    for (;;) {
        c->nx = (int64_t)floor((mx[0] - mn[0]) / g) + 1;
        c->ny = (int64_t)floor((mx[1] - mn[1]) / g) + 1;
        c->nz = (int64_t)floor((mx[2] - mn[2]) / g) + 1;
        if (c->nx * c->ny * c->nz <= ((int64_t)1 << 26)) break;
        g *= 2.0;
    }
    c->g = g; c->ox = mn[0]; c->oy = mn[1]; c->oz = mn[2];
    const int64_t ncell = c->nx * c->ny * c->nz;
    c->start = (uint32_t *)calloc((size_t)ncell + 1, sizeof(uint32_t));
    uint32_t *cid = (uint32_t *)malloc((size_t)nf * sizeof(uint32_t));
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        int64_t ix = (int64_t)floor(((double)p[0] - c->ox) / g);
        int64_t iy = (int64_t)floor(((double)p[1] - c->oy) / g);
        int64_t iz = (int64_t)floor(((double)p[2] - c->oz) / g);
        if (ix >= c->nx) ix = c->nx - 1;
        if (iy >= c->ny) iy = c->ny - 1;
        if (iz >= c->nz) iz = c->nz - 1;
        cid[k] = (uint32_t)(ix + c->nx * (iy + c->ny * iz));
        c->start[cid[k] + 1]++;
        ++k;
    }
    for (int64_t i = 0; i < ncell; ++i) c->start[i + 1] += c->start[i];
    uint32_t *cur = (uint32_t *)malloc((size_t)ncell * sizeof(uint32_t));
    memcpy(cur, c->start, (size_t)ncell * sizeof(uint32_t));
    c->p = (float *)malloc((size_t)nf * 3 * sizeof(float));
    k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        uint32_t d = cur[cid[k]]++;
        c->p[3 * d + 0] = p[0]; c->p[3 * d + 1] = p[1]; c->p[3 * d + 2] = p[2];
        ++k;
    }
    free(cur); free(cid);
    return c;
}

void orc_cloud_free(orc_cloud *c)
{
    if (!c) return;
    free(c->p); free(c->start); free(c);
}

/* FLANN L2_Simple<float>: result += diff*diff over x,y,z, strict < against float(r^2). */
static inline int flann_within(float qx, float qy, float qz, const float *p, float r2)
{
    float d0 = qx - p[0], d1 = qy - p[1], d2 = qz - p[2];
    float acc = 0.0f;
    acc += d0 * d0;
    acc += d1 * d1;
    acc += d2 * d2;
    return acc < r2;
}

/* cells overlapping [q - r - m, q + r + m] (double, conservative margin) */
static inline void cell_range(const orc_cloud *c, double lo, double hi, double o, int64_t nax,
                              int64_t *a, int64_t *b)
{
    int64_t i0 = (int64_t)floor((lo - o) / c->g), i1 = (int64_t)floor((hi - o) / c->g);
    if (i0 < 0) i0 = 0;
    if (i1 > nax - 1) i1 = nax - 1;
    *a = i0; *b = i1;
}

static int any_within_r2(const orc_cloud *c, float qx, float qy, float qz, double radius, float r2)
{
    if (c->kd) return orc_kd_radius(c->kd, qx, qy, qz, r2, NULL, 0) > 0;
    if (c->n == 0) return 0;
    const double m = radius + 1e-3;
    int64_t x0, x1, y0, y1, z0, z1;
    cell_range(c, (double)qx - m, (double)qx + m, c->ox, c->nx, &x0, &x1);
    cell_range(c, (double)qy - m, (double)qy + m, c->oy, c->ny, &y0, &y1);
    cell_range(c, (double)qz - m, (double)qz + m, c->oz, c->nz, &z0, &z1);
    if (x0 > x1 || y0 > y1 || z0 > z1) return 0;
    for (int64_t iz = z0; iz <= z1; ++iz)
        for (int64_t iy = y0; iy <= y1; ++iy) {
            const int64_t row = c->nx * (iy + c->ny * iz);
            const uint32_t s = c->start[row + x0], e = c->start[row + x1 + 1];
            for (uint32_t k = s; k < e; ++k)
                if (flann_within(qx, qy, qz, c->p + 3 * (int64_t)k, r2)) return 1;
        }
    return 0;
}

void orc_cloud_use_kdtree(orc_cloud *c, const orc_kdtree *kd) { c->kd = kd; }

/* exact grid count (never the attached tree: this is what the tree is checked against) */
int64_t orc_cloud_count_within(const orc_cloud *c, float qx, float qy, float qz, double radius)
{
    if (c->n == 0) return 0;
    const float r2 = (float)(radius * radius);
    const double m = radius + 1e-3;
    int64_t x0, x1, y0, y1, z0, z1, cnt = 0;
    cell_range(c, (double)qx - m, (double)qx + m, c->ox, c->nx, &x0, &x1);
    cell_range(c, (double)qy - m, (double)qy + m, c->oy, c->ny, &y0, &y1);
    cell_range(c, (double)qz - m, (double)qz + m, c->oz, c->nz, &z0, &z1);
    if (x0 > x1 || y0 > y1 || z0 > z1) return 0;
    for (int64_t iz = z0; iz <= z1; ++iz)
        for (int64_t iy = y0; iy <= y1; ++iy) {
            const int64_t row = c->nx * (iy + c->ny * iz);
            const uint32_t s = c->start[row + x0], e = c->start[row + x1 + 1];
            for (uint32_t k = s; k < e; ++k)
                cnt += flann_within(qx, qy, qz, c->p + 3 * (int64_t)k, r2);
        }
    return cnt;
}

int orc_cloud_any_within(const orc_cloud *c, float qx, float qy, float qz, double radius)
{
    /* KdTreeFLANN::radiusSearch: static_cast<float>(radius * radius) */
    return any_within_r2(c, qx, qy, qz, radius, (float)(radius * radius));
}

/* virtual_lidar.cpp:600-625 getGroundHeight.  The caller handles the empty-cloud early
 * return (:601). */
double orc_ground_height(const orc_cloud *c, double x, double y)
{
    const float qx = (float)x, qy = (float)y, qz = 0.0f;   /* PointXYZRGB search_point */
    const double radius = 2.0;
    const float r2 = (float)(radius * radius);
    if (c->kd) {   /* the tree's neighbour list (:611), then the 2-D filter (:613-620) */
        const int64_t nn = orc_kd_radius(c->kd, qx, qy, qz, r2, NULL, 0);
        if (nn == 0) return 0.0;
        int64_t *idx = (int64_t *)malloc((size_t)nn * sizeof(int64_t));
        orc_kd_radius(c->kd, qx, qy, qz, r2, idx, nn);
        double max_z = -DBL_MAX;
        for (int64_t k = 0; k < nn; ++k) {
            const float *p = orc_kd_point(c->kd, idx[k]);
            const double dx = (double)p[0] - x, dy = (double)p[1] - y;
            if (sqrt(dx * dx + dy * dy) < 1.0 && (double)p[2] > max_z) max_z = (double)p[2];
        }
        free(idx);
        return max_z != -DBL_MAX ? max_z : 0.0;
    }
    if (c->n == 0) return 0.0;
    const double m = radius + 1e-3;
    int64_t x0, x1, y0, y1, z0, z1;
    cell_range(c, (double)qx - m, (double)qx + m, c->ox, c->nx, &x0, &x1);
    cell_range(c, (double)qy - m, (double)qy + m, c->oy, c->ny, &y0, &y1);
    cell_range(c, -m, m, c->oz, c->nz, &z0, &z1);
    double max_z = -DBL_MAX;   /* std::numeric_limits<double>::lowest() */
    if (x0 <= x1 && y0 <= y1 && z0 <= z1) {
        for (int64_t iz = z0; iz <= z1; ++iz)
            for (int64_t iy = y0; iy <= y1; ++iy) {
                const int64_t row = c->nx * (iy + c->ny * iz);
                const uint32_t s = c->start[row + x0], e = c->start[row + x1 + 1];
                for (uint32_t k = s; k < e; ++k) {
                    const float *p = c->p + 3 * (int64_t)k;
                    if (!flann_within(qx, qy, qz, p, r2)) continue;
                    const double dx = (double)p[0] - x, dy = (double)p[1] - y;  /* :615-616 */
                    if (sqrt(dx * dx + dy * dy) < 1.0) {
                        if ((double)p[2] > max_z) max_z = (double)p[2];
                    }
                }
            }
    }
    if (max_z != -DBL_MAX) return max_z;
    return 0.0;
}

/* ================================================================================ */
/* virtual_lidar.cpp:550-598 generateCandidatePositions                              */
/* ================================================================================ */
int64_t orc_generate_candidates(const orc_cloud *terrain, int terrain_empty, const double bb[6],
                                const orc_vl_params *p, const double zx[5], double *out,
                                int64_t cap)
{
    const double gminx = bb[0], gmaxx = bb[1], gminy = bb[2], gmaxy = bb[3];
    const double ezmin = bb[4], ezmax = bb[5];
    const double exminx = gminx - p->search_radius, exmaxx = gmaxx + p->search_radius;
    const double exminy = gminy - p->search_radius, exmaxy = gmaxy + p->search_radius;
    const double cx = (gminx + gmaxx) / 2.0, cy = (gminy + gmaxy) / 2.0;
    const double cz = (ezmin + ezmax) / 2.0;
    const int gs = (int)ceil(sqrt((double)p->num_candidates));
    const double xs = (exmaxx - exminx) / (gs - 1);
    const double ys = (exmaxy - exminy) / (gs - 1);
    int64_t n = 0;
    for (int i = 0; i < gs; ++i)
        for (int j = 0; j < gs; ++j) {
            const double x = exminx + i * xs;
            const double y = exminy + j * ys;
            const double ddx = x - zx[0], ddy = y - zx[1];
            if (sqrt(ddx * ddx + ddy * ddy) < 0.5) continue;          /* pow(.,2) == x*x */
            if (x >= gminx && x <= gmaxx && y >= gminy && y <= gmaxy) continue;
            const double ground = (terrain_empty || !terrain) ? 0.0 : orc_ground_height(terrain, x, y);
            const double z = ground + p->sensor_height;
            const double dx = cx - x, dy = cy - y, dz = cz - z;
            const double hd = sqrt(dx * dx + dy * dy);
            if (hd < 0.1) continue;
            const double elev = atan2(-dz, hd);
            if (elev >= VL_MIN_ELEVATION && elev <= VL_MAX_ELEVATION) {
                if (n < cap) {
                    double *o = out + 5 * n;
                    o[0] = x; o[1] = y; o[2] = z;
                    o[3] = -M_PI / 2 + elev;
                    o[4] = atan2(dy, dx);
                }
                ++n;
            }
        }
    return n;
}

/* ================================================================================ */
/* virtual_lidar.cpp:754-800 checkVisibilityWithRaycasting                           */
/* ================================================================================ */
static int raycast_visible(const orc_cloud *t, const double pos[3], double cx, double cy, double cz)
{
    const double dx = cx - pos[0], dy = cy - pos[1], dz = cz - pos[2];
    const double distance = sqrt(dx * dx + dy * dy + dz * dz);
    const double ndx = dx / distance, ndy = dy / distance, ndz = dz / distance;
    const double radius = VL_VISIBILITY_RADIUS * 0.7;
    const float r2 = (float)(radius * radius);
    double step = 0.5;
    const double end = distance - VL_VISIBILITY_RADIUS;
    while (step < end) {
        const float qx = (float)(pos[0] + ndx * step);
        const float qy = (float)(pos[1] + ndy * step);
        const float qz = (float)(pos[2] + ndz * step);
        /* radiusSearch(.., 0.056) > 0 and any d2 < VISIBILITY_RADIUS*0.5 (always true for a
         * returned squared distance < 0.003136) -> blocked */
        if (any_within_r2(t, qx, qy, qz, radius, r2)) return 0;
        step += VL_RAY_STEP_SIZE;
    }
    return 1;
}

typedef struct {
    const orc_cloud *terrain;   /* NULL: no terrain KD-tree */
    const orc_cloud *aux;       /* NULL or empty: no zx120 cloud */
    int64_t aux_n;
    double max_distance;
} vl_env;

/* virtual_lidar.cpp:716-752 checkVisibility / checkVisibilityWithPointCloudRelaxed */
static int check_visibility(const vl_env *E, const double pos[3], const double c[3], int is_zx120)
{
    if (is_zx120) {
        if (!E->aux || E->aux_n == 0) {
            if (!E->terrain) return 1;
            return raycast_visible(E->terrain, pos, c[0], c[1], c[2]);
        }
        if (any_within_r2(E->aux, (float)c[0], (float)c[1], (float)c[2],
                          VL_VISIBILITY_RADIUS * 3.0,
                          (float)((VL_VISIBILITY_RADIUS * 3.0) * (VL_VISIBILITY_RADIUS * 3.0))))
            return 1;
        if (!E->terrain) return 1;
        return raycast_visible(E->terrain, pos, c[0], c[1], c[2]);
    }
    if (!E->terrain) return 1;
    return raycast_visible(E->terrain, pos, c[0], c[1], c[2]);
}

/* virtual_lidar.cpp:656-701 evaluateCellScore (+ isInFieldOfView :703-714) */
static double eval_cell(const vl_env *E, const double pose[5], const double c[3], const float n[3],
                        uint8_t *flags, int is_zx120)
{
    const double dx = c[0] - pose[0], dy = c[1] - pose[1], dz = c[2] - pose[2];
    const double L = sqrt(dx * dx + dy * dy + dz * dz);
    const int in_range = (L >= VL_MIN_DISTANCE && L <= E->max_distance);
    const uint8_t fr = is_zx120 ? ORC_F_RANGE_Z : ORC_F_RANGE_M;
    const uint8_t ff = is_zx120 ? ORC_F_FOV_Z : ORC_F_FOV_M;
    const uint8_t fv = is_zx120 ? ORC_F_VIS_Z : ORC_F_VIS_M;
    *flags = in_range ? (uint8_t)(*flags | fr) : (uint8_t)(*flags & ~fr);
    if (!in_range) return 0.0;
    const double elevation = atan2(dz, sqrt(dx * dx + dy * dy));
    const double elevation_diff = elevation - pose[3];
    const double FOV_VERTICAL_LOCAL = 180.0 * M_PI / 180.0;
    const int in_fov = fabs(elevation_diff) <= FOV_VERTICAL_LOCAL / 2.0;
    *flags = in_fov ? (uint8_t)(*flags | ff) : (uint8_t)(*flags & ~ff);
    if (!in_fov) return 0.0;
    const int visible = check_visibility(E, pose, c, is_zx120);
    *flags = visible ? (uint8_t)(*flags | fv) : (uint8_t)(*flags & ~fv);
    if (!visible) return 0.0;
    const double bx = dx / L, by = dy / L, bz = dz / L;
    const double dot = bx * (double)n[0] + by * (double)n[1] + bz * (double)n[2];
    const double theta = acos(fmax(0.0, fmin(1.0, fabs(dot))));
    const double score = 1.0 * sin(M_PI / 2 - theta) + 1.0 * (1.0 / L);
    return fmax(0.0, score);
}

void orc_score_poses(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                     const double *cxyz, const float *cn, int64_t C,
                     const double *poses5, int64_t P, const double zx120[5],
                     const orc_vl_params *p, uint8_t *flags,
                     double *total_score, int32_t *covered, orc_vl_report *rep)
{
    vl_env E = {terrain, aux, aux_n, p->max_distance};
    memset(rep, 0, sizeof(*rep));
    /* evaluateZX120Only (:360-452) */
    double tz = 0.0;
    for (int64_t i = 0; i < C; ++i) {
        rep->total_cells++;
        const double s = eval_cell(&E, zx120, cxyz + 3 * i, cn + 3 * i, &flags[i], 1);
        if (flags[i] & ORC_F_RANGE_Z) rep->zx120_range_ok++;
        if (flags[i] & ORC_F_FOV_Z) rep->zx120_fov_ok++;
        if (flags[i] & ORC_F_VIS_Z) rep->zx120_visible_ok++;
        if (s > 0) tz += s;
        if (!(flags[i] & ORC_F_RANGE_Z)) rep->zx120_blue++;
        else if (!(flags[i] & ORC_F_FOV_Z)) rep->zx120_yellow++;
        else if (!(flags[i] & ORC_F_VIS_Z)) rep->zx120_red++;
        else rep->zx120_green++;
    }
    rep->zx120_total_score = tz;
    /* candidate loop (:464-475) */
    double best = -INFINITY;
    int64_t best_idx = -1;
    for (int64_t k = 0; k < P; ++k) {
        const double *pose = poses5 + 5 * k;
        double total = 0.0;
        int32_t cov = 0;
        for (int64_t i = 0; i < C; ++i) {   /* evaluatePosition (:634-645) */
            const double sz = eval_cell(&E, zx120, cxyz + 3 * i, cn + 3 * i, &flags[i], 1);
            const double sm = eval_cell(&E, pose, cxyz + 3 * i, cn + 3 * i, &flags[i], 0);
            const double comb = sz > sm ? sz : sm;   /* std::max */
            if (comb > 0) { cov++; total += comb; }
        }
        total_score[k] = total;
        covered[k] = cov;
        if (total > best) { best = total; best_idx = k; }
    }
    rep->best_idx = best_idx;
    rep->best_score = best;
    /* colour statistics from the (stale) flags (:487-501) */
    for (int64_t i = 0; i < C; ++i) {
        const uint8_t f = flags[i];
        if (!(f & ORC_F_RANGE_Z) && !(f & ORC_F_RANGE_M)) rep->blue++;
        else if (!(f & ORC_F_FOV_Z) && !(f & ORC_F_FOV_M)) rep->yellow++;
        else if (!(f & ORC_F_VIS_Z) && !(f & ORC_F_VIS_M)) rep->red++;
        else rep->green++;
    }
}

/* evaluateCellScore's value for every (pose, cell) and for the zx120 pose (test
 * infrastructure: the per-cell parity bar): sm[k * C + i] = the pose's score_mobile of cell i,
 * sz[i] = score_zx120 (evaluatePosition :634-645 before the std::max).  Flags are scratch. */
void orc_score_matrix(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                      const double *cxyz, const float *cn, int64_t C,
                      const double *poses5, int64_t P, const double zx120[5],
                      const orc_vl_params *p, double *sm, double *sz)
{
    vl_env E = {terrain, aux, aux_n, p->max_distance};
    uint8_t *fl = (uint8_t *)calloc((size_t)(C > 0 ? C : 1), 1);
    for (int64_t i = 0; i < C; ++i) sz[i] = eval_cell(&E, zx120, cxyz + 3 * i, cn + 3 * i, &fl[i], 1);
#ifdef _OPENMP
#pragma omp parallel for num_threads(g_threads) schedule(dynamic, 1)
#endif
    for (int64_t k = 0; k < P; ++k) {
        uint8_t f = 0;
        for (int64_t i = 0; i < C; ++i)
            sm[k * C + i] = eval_cell(&E, poses5 + 5 * k, cxyz + 3 * i, cn + 3 * i, &f, 0);
    }
    free(fl);
}

/* The candidate loop's per-pose totals alone (evaluatePosition :627-654 for every pose),
 * OpenMP over poses -- the CPU baseline's multi-threaded variant.  The flags a pose writes
 * never feed a score, so each thread keeps its own scratch flags; totals and covered counts
 * are those of orc_score_poses. */
void orc_score_totals(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                      const double *cxyz, const float *cn, int64_t C,
                      const double *poses5, int64_t P, const double zx120[5],
                      const orc_vl_params *p, double *total_score, int32_t *covered)
{
    vl_env E = {terrain, aux, aux_n, p->max_distance};
#ifdef _OPENMP
#pragma omp parallel num_threads(g_threads)
#endif
    {
        uint8_t *fl = (uint8_t *)calloc((size_t)(C > 0 ? C : 1), 1);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = 0; k < P; ++k) {
            const double *pose = poses5 + 5 * k;
            double total = 0.0;
            int32_t cov = 0;
            for (int64_t i = 0; i < C; ++i) {
                const double sz = eval_cell(&E, zx120, cxyz + 3 * i, cn + 3 * i, &fl[i], 1);
                const double sm = eval_cell(&E, pose, cxyz + 3 * i, cn + 3 * i, &fl[i], 0);
                const double comb = sz > sm ? sz : sm;
                if (comb > 0) { cov++; total += comb; }
            }
            total_score[k] = total;
            covered[k] = cov;
        }
        free(fl);
    }
}

/* ================================================================================ */
/* Fan raycast (BASELINE configs[1]) using the :765-797 march rule                   */
/* ================================================================================ */
void orc_fan_tables(int32_t n_az, int32_t n_el, double el_min, double el_max,
                    double *ca, double *sa, double *ce, double *se)
{
    for (int32_t i = 0; i < n_az; ++i) {
        const double a = 2.0 * M_PI * (double)i / (double)n_az;
        ca[i] = cos(a); sa[i] = sin(a);
    }
    for (int32_t j = 0; j < n_el; ++j) {
        const double e = el_min + (el_max - el_min) * ((double)j + 0.5) / (double)n_el;
        ce[j] = cos(e); se[j] = sin(e);
    }
}

void orc_raycast_fan(const orc_cloud *t, const double *poses5, int64_t P, int32_t n_az,
                     int32_t n_el, double el_min, double el_max, double max_distance,
                     int16_t *first_hit, uint32_t *blocked, uint64_t *units)
{
    double *ca = (double *)malloc(sizeof(double) * (size_t)n_az);
    double *sa = (double *)malloc(sizeof(double) * (size_t)n_az);
    double *ce = (double *)malloc(sizeof(double) * (size_t)n_el);
    double *se = (double *)malloc(sizeof(double) * (size_t)n_el);
    orc_fan_tables(n_az, n_el, el_min, el_max, ca, sa, ce, se);
    const double radius = VL_VISIBILITY_RADIUS * 0.7;
    const float r2 = (float)(radius * radius);
    const double end = max_distance - VL_VISIBILITY_RADIUS;
    int32_t K = 0;
    for (double s = 0.5; s < end; s += VL_RAY_STEP_SIZE) ++K;
    for (int64_t p = 0; p < P; ++p) { blocked[p] = 0; units[p] = 0; }
    const int64_t jobs = P * (int64_t)n_el;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_threads)
#endif
    for (int64_t job = 0; job < jobs; ++job) {
        const int64_t p = job / n_el;
        const int32_t j = (int32_t)(job % n_el);
        const double *pose = poses5 + 5 * p;
        const double cyw = cos(pose[4]), syw = sin(pose[4]);
        uint32_t nb = 0;
        uint64_t nu = 0;
        for (int32_t i = 0; i < n_az; ++i) {
            const double lx = ce[j] * ca[i], ly = ce[j] * sa[i], lz = se[j];
            const double dx = cyw * lx - syw * ly;
            const double dy = syw * lx + cyw * ly;
            const double dz = lz;
            int32_t hit = -1, k = 0;
            double step = 0.5;
            while (step < end) {
                const float qx = (float)(pose[0] + dx * step);
                const float qy = (float)(pose[1] + dy * step);
                const float qz = (float)(pose[2] + dz * step);
                if (any_within_r2(t, qx, qy, qz, radius, r2)) { hit = k; break; }
                step += VL_RAY_STEP_SIZE;
                ++k;
            }
            if (first_hit) first_hit[(p * n_el + j) * (int64_t)n_az + i] = (int16_t)hit;
            if (hit >= 0) { nb++; nu += (uint64_t)hit + 1; }
            else nu += (uint64_t)K;
        }
#ifdef _OPENMP
#pragma omp atomic
#endif
        blocked[p] += nb;
#ifdef _OPENMP
#pragma omp atomic
#endif
        units[p] += nu;
    }
    free(ca); free(sa); free(ce); free(se);
}
