// mock_pcp.cpp -- a CPU test double of the libpcp C ABI for the shell-driver tests.
// Test infrastructure only: it lets tests/ros_stub/shell_driver.cpp run a node shell plus the
// real node core (pcp_nodes.cpp) on a machine without a GPU, so the CPU suite can observe what
// the shell publishes per message.  Its numbers are canned, not the reference's algorithm; the
// GPU variant of the same driver links the real libpcp.so (tests/test_ros_shells.py).
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "pcp_abi.h"

struct pcp_ctx {
    std::string err;
    std::vector<double> cells;   // xyz per cell
    uint64_t terrain_n = 0, aux_n = 0;
};
struct pcp_multi {
    pcp_ctx r0;
};

static int fail(pcp_ctx *c, const char *what) {
    c->err = std::string("mock libpcp: ") + what;
    return PCP_E_INVALID;
}

extern "C" {

int pcp_create(int, pcp_ctx **out) {
    *out = new pcp_ctx();
    return PCP_OK;
}
void pcp_destroy(pcp_ctx *c) { delete c; }
const char *pcp_last_error(const pcp_ctx *c) { return c ? c->err.c_str() : "null context"; }

int pcp_multi_create(int, const int *, pcp_multi **out) {
    *out = new pcp_multi();
    return PCP_OK;
}
void pcp_multi_destroy(pcp_multi *m) { delete m; }
const char *pcp_multi_last_error(const pcp_multi *m) { return m->r0.err.c_str(); }
int pcp_multi_info(const pcp_multi *, int *n, int *rccl) {
    *n = 2;
    *rccl = 0;
    return PCP_OK;
}
pcp_ctx *pcp_multi_ctx(pcp_multi *m, int) { return &m->r0; }

static void xyz_of(const pcp_cloud_view *v, uint64_t i, double p[3]) {
    const uint8_t *r = static_cast<const uint8_t *>(v->data) + i * v->point_step;
    float f[3];
    std::memcpy(&f[0], r + v->off_x, 4);
    std::memcpy(&f[1], r + v->off_y, 4);
    std::memcpy(&f[2], r + v->off_z, 4);
    for (int a = 0; a < 3; ++a) p[a] = f[a];
}

// cells: every 7th area point; a non-finite point is refused (the error path of :175-177)
int pcp_set_excavation_area(pcp_ctx *c, const pcp_cloud_view *area, double res, int32_t,
                            double bb[6], uint64_t *n_cells) {
    c->cells.clear();
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint64_t i = 0; i < area->n; ++i) {
        double p[3];
        xyz_of(area, i, p);
        for (int a = 0; a < 3; ++a) {
            if (!std::isfinite(p[a])) return fail(c, "non-finite excavation-area point");
            lo[a] = std::fmin(lo[a], p[a]);
            hi[a] = std::fmax(hi[a], p[a]);
        }
        if (i % 7 == 0) c->cells.insert(c->cells.end(), p, p + 3);
    }
    for (int a = 0; a < 3; ++a) {
        bb[2 * a] = lo[a] - res;
        bb[2 * a + 1] = hi[a] + res;
    }
    *n_cells = c->cells.size() / 3;
    return PCP_OK;
}
// the composed filter + merger (not used by the shells)
int pcp_filter_merge_nodes(pcp_ctx *c, int, const pcp_cloud_view *, const double *, float,
                           const pcp_rigid *, const uint8_t *, void *, uint64_t, uint64_t *,
                           uint64_t *, float *const *, uint64_t *) {
    return fail(c, "pcp_filter_merge_nodes: not in the test double");
}
// the double has nothing in flight: the deferred setup is the synchronous one
int pcp_set_excavation_area_async(pcp_ctx *c, const pcp_cloud_view *area, double res, int32_t l,
                                  double bb[6], uint64_t *cap) {
    return pcp_set_excavation_area(c, area, res, l, bb, cap);
}
int pcp_filter_merge_landed(pcp_ctx *c, int, const void **, const float **) {
    return fail(c, "pcp_filter_merge_landed: not in the test double");
}
// the composed carve + area + terrain (not used by the shells)
int pcp_excavate_area_async(pcp_ctx *c, const pcp_cloud_view *, const pcp_excavation_params *,
                            const pcp_rigid *, void *, uint64_t, uint64_t *, void *, uint64_t,
                            uint64_t *, double *, double, int32_t, double *, uint64_t *) {
    return fail(c, "pcp_excavate_area_async: not in the test double");
}
int pcp_excavate_landed(pcp_ctx *c, const void **, const void **) {
    return fail(c, "pcp_excavate_landed: not in the test double");
}
int pcp_cells_count(pcp_ctx *c, uint64_t *n) {
    *n = c->cells.size() / 3;
    return PCP_OK;
}
int pcp_get_cells(pcp_ctx *c, double *xyz, float *nrm, uint64_t cap, uint64_t *n) {
    *n = c->cells.size() / 3;
    if ((xyz || nrm) && *n > cap) return PCP_E_CAPACITY;
    for (uint64_t i = 0; i < *n && (xyz || nrm); ++i)
        for (int a = 0; a < 3; ++a) {
            if (xyz) xyz[3 * i + a] = c->cells[3 * i + a];
            if (nrm) nrm[3 * i + a] = a == 2 ? 1.0f : 0.0f;
        }
    return PCP_OK;
}
int pcp_set_cells(pcp_ctx *c, const double *xyz, const float *, uint64_t n) {
    c->cells.assign(xyz, xyz + 3 * n);
    return PCP_OK;
}
int pcp_multi_set_cells(pcp_multi *m, const double *xyz, const float *nrm, uint64_t n) {
    return pcp_set_cells(&m->r0, xyz, nrm, n);
}
int pcp_set_terrain(pcp_ctx *c, const pcp_cloud_view *v) {
    c->terrain_n = v->n;
    return PCP_OK;
}
int pcp_multi_set_terrain(pcp_multi *m, const pcp_cloud_view *v) { return pcp_set_terrain(&m->r0, v); }
int pcp_set_aux_cloud(pcp_ctx *c, const pcp_cloud_view *v) {
    c->aux_n = v->n;
    return PCP_OK;
}
int pcp_multi_set_aux_cloud(pcp_multi *m, const pcp_cloud_view *v) {
    return pcp_set_aux_cloud(&m->r0, v);
}

// three candidates on the bbox centre line
int pcp_generate_candidates(pcp_ctx *, const double bb[6], const pcp_vl_params *, const double *,
                            double *poses5, uint64_t cap, uint64_t *n) {
    *n = 3;
    if (cap < 3) return PCP_E_CAPACITY;
    for (int i = 0; i < 3; ++i) {
        const double p[5] = {bb[0] + (i + 1) * (bb[1] - bb[0]) / 4, 0.5 * (bb[2] + bb[3]),
                             bb[5] + 1.1, -0.5, 0.0};
        std::memcpy(poses5 + 5 * i, p, sizeof(p));
    }
    return PCP_OK;
}

// canned scores (candidate 1 best); cell i gets flag state i % 4: blue, yellow, red, green
int pcp_score_poses(pcp_ctx *c, const double *, uint64_t n, const double *, const pcp_vl_params *,
                    uint8_t *flags, double *total, int32_t *covered, pcp_vl_report *rep) {
    const uint64_t nc = c->cells.size() / 3;
    static const uint8_t state[4] = {0, PCP_F_RANGE_M, PCP_F_RANGE_M | PCP_F_FOV_M,
                                     PCP_F_RANGE_M | PCP_F_FOV_M | PCP_F_VIS_M};
    *rep = pcp_vl_report{};
    rep->best_idx = n ? 1 : -1;
    rep->best_score = n ? 3.0 : -INFINITY;
    rep->total_cells = (int32_t)nc;
    for (uint64_t i = 0; i < nc; ++i) {
        if (flags) flags[i] = state[i % 4];
        int32_t *cnt[4] = {&rep->blue, &rep->yellow, &rep->red, &rep->green};
        ++*cnt[i % 4];
    }
    rep->zx120_blue = rep->total_cells;
    for (uint64_t i = 0; i < n; ++i) {
        if (total) total[i] = i == 1 ? 3.0 : 1.0;
        if (covered) covered[i] = (int32_t)i;
    }
    return PCP_OK;
}
int pcp_generate_and_score(pcp_ctx *c, const double bb[6], const pcp_vl_params *pp,
                           const double *zx, double *poses5, uint64_t cap, uint64_t *n,
                           uint8_t *f, double *t, int32_t *cv, pcp_vl_report *r) {
    if (int rc = pcp_generate_candidates(c, bb, pp, zx, poses5, cap, n)) return rc;
    return pcp_score_poses(c, poses5, *n, zx, pp, f, t, cv, r);
}
int pcp_multi_score_poses(pcp_multi *m, const double *p, uint64_t n, const double *zx,
                          const pcp_vl_params *pp, uint8_t *f, double *t, int32_t *cv,
                          pcp_vl_report *r) {
    return pcp_score_poses(&m->r0, p, n, zx, pp, f, t, cv, r);
}

// the other nodes' entry points link but are not exercised by the driver
int pcp_crop_voxel(pcp_ctx *c, const pcp_cloud_view *, const double *, float, float *, uint64_t,
                   uint64_t *, uint64_t *) {
    return fail(c, "pcp_crop_voxel");
}
int pcp_transform_concat(pcp_ctx *c, int, const pcp_cloud_view *, const pcp_rigid *,
                         const uint8_t *, void *, uint64_t, uint64_t *) {
    return fail(c, "pcp_transform_concat");
}
int pcp_excavate_bounds(const pcp_excavation_params *, uint64_t, uint64_t *t, uint64_t *a) {
    *t = *a = 0;
    return PCP_E_INVALID;
}
int pcp_excavate(pcp_ctx *c, const pcp_cloud_view *, const pcp_excavation_params *,
                 const pcp_rigid *, void *, uint64_t, uint64_t *, void *, uint64_t, uint64_t *,
                 double *) {
    return fail(c, "pcp_excavate");
}
int pcp_drivable_area(pcp_ctx *c, const pcp_cloud_view *, const pcp_rigid *, double, double,
                      double, double, const pcp_drivable_params *, int8_t *, uint64_t, int32_t *,
                      double *) {
    return fail(c, "pcp_drivable_area");
}

}  // extern "C"
