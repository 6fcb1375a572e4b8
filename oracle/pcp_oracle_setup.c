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
