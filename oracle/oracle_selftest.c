/* oracle_selftest.c -- TEST INFRASTRUCTURE ONLY: drives every entry point of the CPU
 * restatement (pcp_oracle.c, pcp_oracle_setup.c, pcp_flann.c) on small seeded inputs, for the
 * AddressSanitizer / UndefinedBehaviorSanitizer build (`make -C oracle asan`).
 * Inputs include NaN points, exact box faces, empty clouds, the voxel overflow passthrough,
 * duplicated points and degenerate (single-column) clouds.  Besides the sanitizers' own
 * reports, it checks the invariants that need no second implementation: the restated
 * KdTreeFLANN and the grid scan agree on every query, the fan in FLANN mode equals the fan
 * over the grid, and counts stay within their capacities.  Exit 0 = clean. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcp_oracle.h"

static uint64_t g_rng = 20260227u;
static double urand(void) {   /* splitmix64 -> [0, 1) */
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
}
static double unif(double a, double b) { return a + (b - a) * urand(); }

static int g_fail = 0;
#define CHECK(c, ...)                                \
    do {                                             \
        if (!(c)) {                                  \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);            \
            fprintf(stderr, "\n");                   \
            g_fail = 1;                              \
        }                                            \
    } while (0)

/* a 0.05 m lattice with noise, a pit and a wall, as float4 rows (x, y, z, rgb) */
static float *terrain(int side, int64_t *n_out) {
    const int64_t n = (int64_t)side * side + 400;
    float *t = (float *)calloc((size_t)n * 8, sizeof(float));
    int64_t k = 0;
    for (int i = 0; i < side; ++i)
        for (int j = 0; j < side; ++j, ++k) {
            const double x = -2.0 + 0.05 * i, y = -2.0 + 0.05 * j;
            double z = unif(-0.01, 0.01);
            if (x > 0.5 && x < 1.5 && y > -0.3 && y < 0.4) z -= 0.5;
            t[8 * k] = (float)x; t[8 * k + 1] = (float)y; t[8 * k + 2] = (float)z;
            t[8 * k + 3] = 1.0f;
        }
    for (int w = 0; w < 400; ++w, ++k) {   /* a wall at x = 2 */
        t[8 * k] = 2.0f; t[8 * k + 1] = (float)(-1.0 + 0.05 * (w % 40)); t[8 * k + 2] = (float)(0.05 * (w / 40));
        t[8 * k + 3] = 1.0f;
    }
    *n_out = n;
    return t;
}

static void test_filter(void) {
    const int64_t n = 20000;
    float *c = (float *)malloc((size_t)n * 4 * sizeof(float));
    for (int64_t i = 0; i < n; ++i) {
        c[4 * i] = (float)unif(-3, 18); c[4 * i + 1] = (float)unif(-12, 12);
        c[4 * i + 2] = (float)unif(-3, 12); c[4 * i + 3] = 0.0f;
    }
    for (int i = 0; i < 50; ++i) c[4 * i] = NAN;
    for (int i = 50; i < 70; ++i) c[4 * i] = 15.0f;       /* exact box faces */
    for (int i = 70; i < 90; ++i) c[4 * i + 2] = -1.5f;
    const double box[6] = {0.0, 15.0, -10.0, 10.0, -1.5, 10.0};
    uint32_t *kept = (uint32_t *)malloc((size_t)n * sizeof(uint32_t));
    const int64_t m = orc_crop_box(c, n, 4, box, kept);
    CHECK(m > 0 && m < n, "crop kept %lld", (long long)m);
    float *cr = (float *)malloc((size_t)(m > 0 ? m : 1) * 4 * sizeof(float));
    for (int64_t i = 0; i < m; ++i) memcpy(cr + 4 * i, c + 4 * (int64_t)kept[i], 16);
    float *vx = (float *)malloc((size_t)(m > 0 ? m : 1) * 3 * sizeof(float));
    uint32_t *vi = (uint32_t *)malloc((size_t)(m > 0 ? m : 1) * sizeof(uint32_t));
    uint32_t *vc = (uint32_t *)malloc((size_t)(m > 0 ? m : 1) * sizeof(uint32_t));
    int pt = 0;
    int64_t nv = orc_voxel_grid(cr, m, 4, 0.2f, vx, vi, vc, &pt);
    CHECK(nv > 0 && nv <= m && !pt, "voxel %lld pt %d", (long long)nv, pt);
    uint64_t tot = 0;
    for (int64_t v = 0; v < nv; ++v) tot += vc[v];
    CHECK(tot == (uint64_t)m, "voxel counts %llu vs %lld", (unsigned long long)tot, (long long)m);
    nv = orc_voxel_grid(cr, m, 4, 1e-4f, vx, vi, vc, &pt);   /* int32 overflow -> passthrough */
    CHECK(pt == 1 && nv == m, "overflow passthrough %d %lld", pt, (long long)nv);
    nv = orc_voxel_grid(cr, 0, 4, 0.2f, vx, vi, vc, &pt);
    CHECK(nv == 0, "empty voxel");
    float *o8 = (float *)malloc((size_t)(m > 0 ? m : 1) * 8 * sizeof(float));
    const double t[3] = {8.0, -3.0, 0.0}, q[4] = {0.0, 0.0, 0.2588190451025208, 0.9659258262890683};
    orc_transform_rgb(cr, m, 4, t, q, 255, 0, 0, o8);
    free(c); free(kept); free(cr); free(vx); free(vi); free(vc); free(o8);
}

static void test_search_and_fan(void) {
    int64_t n = 0;
    float *t = terrain(80, &n);
    t[8 * 3] = NAN;   /* a non-finite point: dropped by both structures */
    orc_cloud *g = orc_cloud_build(t, n, 8);
    orc_kdtree *kd = orc_kd_build(t, n, 8, 15);
    CHECK(orc_kd_size(kd) == n - 1, "kd size %lld", (long long)orc_kd_size(kd));
    const int64_t nq = 20000;
    float *q = (float *)malloc((size_t)nq * 3 * sizeof(float));
    for (int64_t i = 0; i < nq; ++i) {
        const int64_t p = (int64_t)(urand() * (double)n);
        const double r = (i & 1) ? 0.056 : 0.24;
        const double u = unif(-1, 1), v = unif(0, 2 * M_PI), w = sqrt(1 - u * u);
        q[3 * i] = (float)(t[8 * p] + r * w * cos(v));
        q[3 * i + 1] = (float)(t[8 * p + 1] + r * w * sin(v));
        q[3 * i + 2] = (float)(t[8 * p + 2] + r * u);
    }
    uint64_t st[4];
    orc_kd_check_queries(kd, g, q, nq, 0.056, st);
    CHECK(st[1] == 0 && st[2] == 0, "kd vs grid r=0.056: %llu %llu", (unsigned long long)st[1],
          (unsigned long long)st[2]);
    orc_kd_check_queries(kd, g, q, nq, 0.24, st);
    CHECK(st[1] == 0 && st[2] == 0, "kd vs grid r=0.24");
    const double poses[10] = {0.0, 0.0, 1.1, -0.5, 0.3, 1.8, 1.0, 0.6, -0.2, 2.5};
    const double el = 85.0 * M_PI / 180.0;
    int16_t *fh = (int16_t *)malloc(2 * 16 * 64 * sizeof(int16_t));
    int16_t *fk = (int16_t *)malloc(2 * 16 * 64 * sizeof(int16_t));
    uint32_t b[2], bk[2];
    uint64_t u[2], uk[2];
    orc_raycast_fan(g, poses, 2, 64, 16, -el, el, 15.0, fh, b, u);
    orc_kd_raycast_fan(kd, g, poses, 2, 64, 16, -el, el, 15.0, fk, bk, uk, st);
    CHECK(memcmp(fh, fk, 2 * 16 * 64 * sizeof(int16_t)) == 0 && b[0] == bk[0] && u[1] == uk[1],
          "fan grid vs kd");
    CHECK(st[1] == 0 && st[0] == u[0] + u[1], "fan sample checks");
    /* candidates + scoring over a few cells, grid mode then FLANN mode */
    double cells[3 * 40];
    float nrm[3 * 40];
    for (int i = 0; i < 40; ++i) {
        cells[3 * i] = 0.5 + 0.1 * (i % 10); cells[3 * i + 1] = -0.2 + 0.1 * (i / 10);
        cells[3 * i + 2] = -0.45;
        nrm[3 * i] = 0.0f; nrm[3 * i + 1] = 0.0f; nrm[3 * i + 2] = 1.0f;
    }
    const double bb[6] = {0.4, 1.6, -0.3, 0.5, -0.6, 0.1};
    const double zx[5] = {0.4, 0.5, 3.5, -M_PI / 6, 0.0};
    orc_vl_params prm = {0.1, 1.1, 3.0, 15.0, 49, 10};
    double cand[5 * 64];
    const int64_t nc = orc_generate_candidates(g, 0, bb, &prm, zx, cand, 64);
    CHECK(nc > 0 && nc <= 64, "candidates %lld", (long long)nc);
    uint8_t fl[40] = {0}, fl2[40] = {0};
    double tot[64], tot2[64];
    int32_t cov[64], cov2[64];
    orc_vl_report rep, rep2;
    orc_score_poses(g, g, n, cells, nrm, 40, cand, nc, zx, &prm, fl, tot, cov, &rep);
    orc_cloud_use_kdtree(g, kd);
    orc_score_poses(g, g, n, cells, nrm, 40, cand, nc, zx, &prm, fl2, tot2, cov2, &rep2);
    orc_cloud_use_kdtree(g, NULL);
    CHECK(memcmp(tot, tot2, (size_t)nc * sizeof(double)) == 0 && memcmp(fl, fl2, 40) == 0 &&
              rep.best_idx == rep2.best_idx,
          "score grid vs kd");
    orc_score_totals(g, NULL, 0, cells, nrm, 40, cand, nc, zx, &prm, tot2, cov2);
    orc_score_poses(NULL, NULL, 0, cells, nrm, 40, cand, 0, zx, &prm, fl, tot, cov, &rep);
    CHECK(rep.best_idx == -1, "no candidates");
    /* an empty cloud */
    orc_cloud *e = orc_cloud_build(t, 0, 8);
    orc_kdtree *ek = orc_kd_build(t, 0, 8, 15);
    CHECK(!orc_cloud_any_within(e, 0, 0, 0, 0.056) && orc_kd_radius_search(ek, 0, 0, 0, 0.056) == 0,
          "empty clouds");
    orc_cloud_free(e); orc_kd_free(ek);
    /* duplicates and a degenerate column */
    float *d = (float *)calloc(3000 * 4, sizeof(float));
    for (int i = 0; i < 3000; ++i) {
        d[4 * i] = (i < 1500) ? 0.25f : (float)(i % 7) * 0.01f;
        d[4 * i + 1] = (i < 1500) ? -0.5f : 0.0f;
        d[4 * i + 2] = (i < 1500) ? (float)(i % 300) * 0.003f : 0.1f;
    }
    orc_cloud *dg = orc_cloud_build(d, 3000, 4);
    orc_kdtree *dk = orc_kd_build(d, 3000, 4, 15);
    for (int i = 0; i < 4000; ++i) {
        q[3 * i] = (float)unif(-0.1, 0.4); q[3 * i + 1] = (float)unif(-0.6, 0.1);
        q[3 * i + 2] = (float)unif(-0.1, 1.0);
    }
    orc_kd_check_queries(dk, dg, q, 4000, 0.056, st);
    CHECK(st[1] == 0, "degenerate cloud kd vs grid");
    orc_cloud_free(dg); orc_kd_free(dk); free(d);
    free(fh); free(fk); free(q);
    orc_kd_free(kd);
    orc_cloud_free(g);
    free(t);
}

static void test_setup_chain(void) {
    int64_t n = 0;
    float *t = terrain(60, &n);
    float *nr = (float *)malloc((size_t)n * 3 * sizeof(float));
    orc_area_normals(t, n, 8, 0.3, nr);
    double bbox[6];
    int32_t dims[3];
    const int64_t nc = orc_excavation_grid(t, n, 8, 0.1, 4, nr, NULL, NULL, 0, bbox, dims);
    CHECK(nc > 0, "excavation grid %lld", (long long)nc);
    double *cx = (double *)malloc((size_t)nc * 3 * sizeof(double));
    float *cn = (float *)malloc((size_t)nc * 3 * sizeof(float));
    CHECK(orc_excavation_grid(t, n, 8, 0.1, 4, nr, cx, cn, nc, bbox, dims) == nc, "grid 2nd pass");
    const orc_exc_params p = {1.0, 75.0, 0.5, 0.2, 0.05, 0.5, 1, 0.6, 0.4, 0.6, 0.4, 0.4, 0.6};
    const double tt[3] = {0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 1.0};
    uint8_t *keep = (uint8_t *)malloc((size_t)n);
    int64_t ns = 0, na = 0;
    double pose[4];
    orc_excavate(t, n, 8, &p, tt, q, keep, NULL, 0, &ns, NULL, 0, &na, pose);
    float *surf = (float *)malloc((size_t)(ns + 1) * 4 * sizeof(float));
    float *area = (float *)malloc((size_t)(na + 1) * 4 * sizeof(float));
    int64_t ns2 = 0, na2 = 0;
    orc_excavate(t, n, 8, &p, tt, q, keep, surf, ns, &ns2, area, na, &na2, pose);
    CHECK(ns2 == ns && na2 == na, "excavate counts");
    CHECK(isfinite(orc_terrain_height(t, n, 8, 0.3, 0.1, 0.5)), "terrain height");
    int8_t grid[40 * 40];
    int32_t gd[2];
    double org[2];
    orc_drivable_area(t, n, 8, tt, q, 0.0, 0.0, 0.0, 0.0, 0.5, 20.0, 20.0, 0.3, 3, 1.0, grid, gd, org);
    CHECK(gd[0] == 40 && gd[1] == 40, "drivable dims %d %d", gd[0], gd[1]);
    free(nr); free(cx); free(cn); free(keep); free(surf); free(area); free(t);
}

int main(void) {
    orc_set_threads(2);
    test_filter();
    test_search_and_fan();
    test_setup_chain();
    if (g_fail) return 1;
    printf("oracle selftest ok\n");
    return 0;
}
