/* pcp_flann.c -- TEST INFRASTRUCTURE ONLY (the second, independent checker of the radius
 * predicate; never a product path).
 *
 * The reference answers every radius query through pcl::KdTreeFLANN<PointXYZRGB>
 * (virtual_lidar.cpp:185-187 setInputCloud, :782 radiusSearch in the ray march, :298, :312,
 * :611, :745).  That class is a thin wrapper over FLANN's KDTreeSingleIndex, a third-party
 * dependency absent from /root/reference (no lockfile; ROS 2 Humble on Ubuntu 22.04 ships
 * PCL 1.12.1 + FLANN 1.9.1).  This file restates the published FLANN 1.9.1
 * algorithm as PCL 1.12.1 configures it, so that the grid-based oracle (pcp_oracle.c) and the
 * GPU -- both "exact" uniform-grid searches -- can be checked against the tree whose float
 * pruning the reference actually runs:
 *
 *   PCL KdTreeFLANN::setInputCloud: non-finite points dropped (index mapping), 3 floats per
 *     point (PointRepresentation xyz), flann::KDTreeSingleIndexParams(leaf_max_size = 15),
 *     reorder = true.
 *   PCL KdTreeFLANN::radiusSearch(p, radius, ..., max_nn = 0): query = float xyz of p,
 *     radius passed as static_cast<float>(radius * radius), SearchParams(checks = -1 /
 *     unlimited, eps = 0, sorted), max_neighbors = -1 -> RadiusResultSet.
 *   FLANN KDTreeSingleIndex::buildIndexImpl: vind = 0..n-1, computeBoundingBox (float),
 *     divideTree(0, n, root_bbox) with middleSplit_ (EPS = 1e-5f, widest-span axes within
 *     (1 - EPS) * max_span, largest spread wins, cut at the split-box midpoint clamped to the
 *     points' [min, max], planeSplit's two partition passes, index = lim1 / lim2 / count / 2),
 *     leaves of <= 15 points with their tight bbox, divlow / divhigh = the children's tight
 *     bounds along divfeat.
 *   FLANN findNeighbors / searchLevel: computeInitialDistances against the root bbox, then
 *     the recursive descent with the incrementally updated float mindistsq
 *     (mindistsq + cut_dist - dists[idx]) and the prune test mindistsq * (1 + eps) <=
 *     worstDist(); leaf points tested with L2_Simple<float> (((0 + dx^2) + dy^2) + dz^2) and
 *     kept iff dist < radius (strict).
 *
 * Built with -ffp-contract=off: every float operation rounds as in the SSE2 build.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pcp_oracle.h"

typedef struct {
    int32_t child1, child2;   /* -1: leaf */
    int32_t left, right;      /* leaf: [left, right) of vind */
    int32_t divfeat;
    float divlow, divhigh;
} kd_node;

struct orc_kdtree {
    int64_t n;
    int leaf_max;
    float *pts;        /* finite points, 3 floats each, in input order (FLANN's dataset) */
    int32_t *vind;     /* permutation built by divideTree */
    float *data;       /* reorder_: data[i] = pts[vind[i]] */
    int64_t *orig;     /* finite point k -> index in the caller's cloud (PCL index mapping) */
    kd_node *nodes;
    int64_t nn, cap;
    float root_bbox[3][2];
    int32_t root;
};

static int32_t new_node(orc_kdtree *t)
{
    if (t->nn == t->cap) {
        t->cap = t->cap ? 2 * t->cap : 1024;
        t->nodes = (kd_node *)realloc(t->nodes, (size_t)t->cap * sizeof(kd_node));
    }
    kd_node *nd = &t->nodes[t->nn];
    nd->child1 = nd->child2 = -1;
    nd->left = nd->right = 0;
    nd->divfeat = 0;
    nd->divlow = nd->divhigh = 0.0f;
    return (int32_t)t->nn++;
}

/* computeMinMax */
static void min_max(const orc_kdtree *t, const int32_t *ind, int count, int dim, float *mn,
                    float *mx)
{
    *mn = t->pts[3 * (int64_t)ind[0] + dim];
    *mx = *mn;
    for (int i = 1; i < count; ++i) {
        const float v = t->pts[3 * (int64_t)ind[i] + dim];
        if (v < *mn) *mn = v;
        if (v > *mx) *mx = v;
    }
}

/* planeSplit */
static void plane_split(const orc_kdtree *t, int32_t *ind, int count, int cutfeat, float cutval,
                        int *lim1, int *lim2)
{
#define V(i) (t->pts[3 * (int64_t)ind[i] + cutfeat])
    int left = 0, right = count - 1;
    for (;;) {
        while (left <= right && V(left) < cutval) ++left;
        while (left <= right && V(right) >= cutval) --right;
        if (left > right) break;
        int32_t tmp = ind[left]; ind[left] = ind[right]; ind[right] = tmp;
        ++left; --right;
    }
    *lim1 = left;
    right = count - 1;
    for (;;) {
        while (left <= right && V(left) <= cutval) ++left;
        while (left <= right && V(right) > cutval) --right;
        if (left > right) break;
        int32_t tmp = ind[left]; ind[left] = ind[right]; ind[right] = tmp;
        ++left; --right;
    }
    *lim2 = left;
#undef V
}

/* middleSplit_ */
static void middle_split(const orc_kdtree *t, int32_t *ind, int count, int *index, int *cutfeat,
                         float *cutval, float bbox[3][2])
{
    const float EPS = 0.00001f;
    float max_span = bbox[0][1] - bbox[0][0];
    for (int i = 1; i < 3; ++i) {
        const float span = bbox[i][1] - bbox[i][0];
        if (span > max_span) max_span = span;
    }
    float max_spread = -1.0f;
    *cutfeat = 0;
    for (int i = 0; i < 3; ++i) {
        const float span = bbox[i][1] - bbox[i][0];
        if (span > (1.0f - EPS) * max_span) {
            float mn, mx;
            min_max(t, ind, count, i, &mn, &mx);
            const float spread = mx - mn;
            if (spread > max_spread) {
                *cutfeat = i;
                max_spread = spread;
            }
        }
    }
    const float split_val = (bbox[*cutfeat][0] + bbox[*cutfeat][1]) / 2.0f;
    float mn, mx;
    min_max(t, ind, count, *cutfeat, &mn, &mx);
    if (split_val < mn) *cutval = mn;
    else if (split_val > mx) *cutval = mx;
    else *cutval = split_val;
    int lim1, lim2;
    plane_split(t, ind, count, *cutfeat, *cutval, &lim1, &lim2);
    if (lim1 > count / 2) *index = lim1;
    else if (lim2 < count / 2) *index = lim2;
    else *index = count / 2;
}

/* divideTree: bbox is in/out (the split box in, the tight box of the subtree out) */
static int32_t divide_tree(orc_kdtree *t, int left, int right, float bbox[3][2])
{
    const int32_t id = new_node(t);
    if (right - left <= t->leaf_max) {
        kd_node *nd = &t->nodes[id];
        nd->left = left;
        nd->right = right;
        for (int i = 0; i < 3; ++i) {
            bbox[i][0] = t->pts[3 * (int64_t)t->vind[left] + i];
            bbox[i][1] = bbox[i][0];
        }
        for (int k = left + 1; k < right; ++k)
            for (int i = 0; i < 3; ++i) {
                const float v = t->pts[3 * (int64_t)t->vind[k] + i];
                if (bbox[i][0] > v) bbox[i][0] = v;
                if (bbox[i][1] < v) bbox[i][1] = v;
            }
        return id;
    }
    int idx, cutfeat;
    float cutval;
    middle_split(t, t->vind + left, right - left, &idx, &cutfeat, &cutval, bbox);
    t->nodes[id].divfeat = cutfeat;
    float lb[3][2], rb[3][2];
    memcpy(lb, bbox, sizeof(lb));
    lb[cutfeat][1] = cutval;
    const int32_t c1 = divide_tree(t, left, left + idx, lb);
    memcpy(rb, bbox, sizeof(rb));
    rb[cutfeat][0] = cutval;
    const int32_t c2 = divide_tree(t, left + idx, right, rb);
    kd_node *nd = &t->nodes[id];   /* (nodes may have moved) */
    nd->child1 = c1;
    nd->child2 = c2;
    nd->divlow = lb[cutfeat][1];
    nd->divhigh = rb[cutfeat][0];
    for (int i = 0; i < 3; ++i) {
        bbox[i][0] = lb[i][0] < rb[i][0] ? lb[i][0] : rb[i][0];   /* std::min */
        bbox[i][1] = lb[i][1] > rb[i][1] ? lb[i][1] : rb[i][1];   /* std::max */
    }
    return id;
}

orc_kdtree *orc_kd_build(const float *pts, int64_t n, int64_t stride, int leaf_max)
{
    orc_kdtree *t = (orc_kdtree *)calloc(1, sizeof(orc_kdtree));
    t->leaf_max = leaf_max > 0 ? leaf_max : 15;
    t->pts = (float *)malloc((size_t)(n > 0 ? n : 1) * 3 * sizeof(float));
    t->orig = (int64_t *)malloc((size_t)(n > 0 ? n : 1) * sizeof(int64_t));
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * stride;
        if (!(isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2]))) continue;
        t->pts[3 * k] = p[0];
        t->pts[3 * k + 1] = p[1];
        t->pts[3 * k + 2] = p[2];
        t->orig[k] = i;
        ++k;
    }
    t->n = k;
    t->root = -1;
    if (k == 0) return t;
    t->vind = (int32_t *)malloc((size_t)k * sizeof(int32_t));
    for (int64_t i = 0; i < k; ++i) t->vind[i] = (int32_t)i;
    /* computeBoundingBox */
    for (int i = 0; i < 3; ++i) t->root_bbox[i][0] = t->root_bbox[i][1] = t->pts[i];
    for (int64_t j = 1; j < k; ++j)
        for (int i = 0; i < 3; ++i) {
            const float v = t->pts[3 * j + i];
            if (v < t->root_bbox[i][0]) t->root_bbox[i][0] = v;
            if (v > t->root_bbox[i][1]) t->root_bbox[i][1] = v;
        }
    t->root = divide_tree(t, 0, (int)k, t->root_bbox);
    t->data = (float *)malloc((size_t)k * 3 * sizeof(float));
    for (int64_t i = 0; i < k; ++i) memcpy(t->data + 3 * i, t->pts + 3 * (int64_t)t->vind[i], 12);
    return t;
}

void orc_kd_free(orc_kdtree *t)
{
    if (!t) return;
    free(t->pts); free(t->vind); free(t->data); free(t->orig); free(t->nodes); free(t);
}

int64_t orc_kd_size(const orc_kdtree *t) { return t ? t->n : 0; }

/* the point behind a neighbour index returned by orc_kd_radius (an index of the caller's
 * cloud): the finite points keep their input order, so a binary search over orig finds it */
const float *orc_kd_point(const orc_kdtree *t, int64_t cloud_idx)
{
    int64_t lo = 0, hi = t->n - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (t->orig[mid] < cloud_idx) lo = mid + 1;
        else hi = mid;
    }
    return t->pts + 3 * lo;
}

typedef struct {
    float radius;     /* RadiusResultSet: worstDist() == radius, addPoint iff dist < radius */
    int64_t count;
    int64_t *idx;     /* nullable: neighbours' indices in the caller's cloud */
    int64_t cap;
} radius_set;

static void search_level(const orc_kdtree *t, radius_set *rs, const float q[3], int32_t id,
                         float mindistsq, float dists[3])
{
    const kd_node *nd = &t->nodes[id];
    if (nd->child1 < 0 && nd->child2 < 0) {
        const float worst = rs->radius;
        for (int i = nd->left; i < nd->right; ++i) {
            const float *p = t->data + 3 * (int64_t)i;
            float result = 0.0f, diff;
            diff = q[0] - p[0]; result += diff * diff;
            diff = q[1] - p[1]; result += diff * diff;
            diff = q[2] - p[2]; result += diff * diff;
            if (result < worst && result < rs->radius) {
                if (rs->idx && rs->count < rs->cap) rs->idx[rs->count] = t->orig[t->vind[i]];
                rs->count++;
            }
        }
        return;
    }
    const int f = nd->divfeat;
    const float val = q[f];
    const float diff1 = val - nd->divlow;
    const float diff2 = val - nd->divhigh;
    int32_t best, other;
    float cut_dist;
    if ((diff1 + diff2) < 0.0f) {
        best = nd->child1;
        other = nd->child2;
        cut_dist = (val - nd->divhigh) * (val - nd->divhigh);
    } else {
        best = nd->child2;
        other = nd->child1;
        cut_dist = (val - nd->divlow) * (val - nd->divlow);
    }
    search_level(t, rs, q, best, mindistsq, dists);
    const float dst = dists[f];
    mindistsq = mindistsq + cut_dist - dst;
    dists[f] = cut_dist;
    if (mindistsq * 1.0f <= rs->radius)   /* epsError = 1 + eps = 1 */
        search_level(t, rs, q, other, mindistsq, dists);
    dists[f] = dst;
}

int64_t orc_kd_radius(const orc_kdtree *t, float qx, float qy, float qz, float r2,
                      int64_t *idx, int64_t cap)
{
    if (!t || t->n == 0) return 0;
    const float q[3] = {qx, qy, qz};
    float dists[3] = {0.0f, 0.0f, 0.0f};
    float distsq = 0.0f;   /* computeInitialDistances */
    for (int i = 0; i < 3; ++i) {
        if (q[i] < t->root_bbox[i][0]) {
            dists[i] = (q[i] - t->root_bbox[i][0]) * (q[i] - t->root_bbox[i][0]);
            distsq += dists[i];
        }
        if (q[i] > t->root_bbox[i][1]) {
            dists[i] = (q[i] - t->root_bbox[i][1]) * (q[i] - t->root_bbox[i][1]);
            distsq += dists[i];
        }
    }
    radius_set rs = {r2, 0, idx, cap};
    search_level(t, &rs, q, t->root, distsq, dists);
    return rs.count;
}

int64_t orc_kd_radius_search(const orc_kdtree *t, float qx, float qy, float qz, double radius)
{
    return orc_kd_radius(t, qx, qy, qz, (float)(radius * radius), NULL, 0);
}

/* Every query (xyz float triples): the tree's neighbour count against the exact grid scan of
 * pcp_oracle.c (same float predicate, no pruning).  stats: [0] queries, [1] queries whose
 * counts differ, [2] queries whose "any neighbour" differs, [3] neighbours (grid). */
void orc_kd_check_queries(const orc_kdtree *t, const orc_cloud *g, const float *q, int64_t nq,
                          double radius, uint64_t stats[4])
{
    const float r2 = (float)(radius * radius);
    uint64_t s1 = 0, s2 = 0, s3 = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4096) reduction(+ : s1, s2, s3) num_threads(orc_get_threads())
#endif
    for (int64_t i = 0; i < nq; ++i) {
        const float *p = q + 3 * i;
        const int64_t a = orc_kd_radius(t, p[0], p[1], p[2], r2, NULL, 0);
        const int64_t b = orc_cloud_count_within(g, p[0], p[1], p[2], radius);
        s1 += (a != b);
        s2 += ((a > 0) != (b > 0));
        s3 += (uint64_t)b;
    }
    stats[0] = (uint64_t)nq;
    stats[1] = s1;
    stats[2] = s2;
    stats[3] = s3;
}

/* The fan march of orc_raycast_fan (virtual_lidar.cpp:765-797 rule) with every sample query
 * answered by the restated KdTreeFLANN (radiusSearch(q, 0.056) > 0 => blocked), and every
 * sample cross-checked against the exact grid count.  Outputs as orc_raycast_fan (first hit
 * per ray: the reference's own predicate); stats as orc_kd_check_queries over the sample
 * queries the reference executes. */
void orc_kd_raycast_fan(const orc_kdtree *t, const orc_cloud *g, const double *poses5, int64_t P,
                        int32_t n_az, int32_t n_el, double el_min, double el_max,
                        double max_distance, int16_t *first_hit, uint32_t *blocked,
                        uint64_t *units, uint64_t stats[4])
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
    uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    const int64_t jobs = P * (int64_t)n_el;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : s0, s1, s2, s3) num_threads(orc_get_threads())
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
                const int64_t a = orc_kd_radius(t, qx, qy, qz, r2, NULL, 0);
                const int64_t b = g ? orc_cloud_count_within(g, qx, qy, qz, radius) : a;
                s0 += 1;
                s1 += (a != b);
                s2 += ((a > 0) != (b > 0));
                s3 += (uint64_t)b;
                if (a > 0) { hit = k; break; }
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
    stats[0] = s0; stats[1] = s1; stats[2] = s2; stats[3] = s3;
    free(ca); free(sa); free(ce); free(se);
}
