// pcp_drivable.hip -- calc_drivable_area.cpp (the occupancy-grid node, robotCloudCallback
// :67-226) on gfx950: tf2::doTransform of the robot's filtered cloud into map (Eigen float),
// binning into the robot-centred grid with the reference's truncating (int) cast, per-cell count
// and z range (order-free integer atomics on order-preserving float keys), then the per-cell
// rule: start-clear disc -> 0, fewer than min_points -> -1, (max z - min z) / resolution >
// max_gradient -> 100, else 0.
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>

#include "pcp_internal.hpp"
#include "pcp_rigid.hpp"

namespace pcp {

constexpr int kDT = 256;

struct DrivArgs {
    const unsigned char *raw;
    uint64_t n;
    uint32_t step, ox, oy, oz;
    Rigid r;
    double origin_x, origin_y, res;
    int32_t gw, gh;
};

// float -> int32 with the same order (non-NaN): atomicMin / atomicMax on the key
__device__ __forceinline__ int32_t fkey(float f) {
    const int32_t b = __float_as_int(f);
    return b >= 0 ? b : (int32_t)(b ^ 0x7FFFFFFF);
}
__device__ __forceinline__ float fkey_inv(int32_t k) {
    return __int_as_float(k >= 0 ? k : (int32_t)(k ^ 0x7FFFFFFF));
}

__global__ void __launch_bounds__(kDT)
k_driv_bin(DrivArgs a, uint32_t *__restrict__ cnt, int32_t *__restrict__ zlo,
           int32_t *__restrict__ zhi) {
    const uint64_t i = (uint64_t)blockIdx.x * kDT + threadIdx.x;
    if (i >= a.n) return;
    const unsigned char *p = a.raw + i * a.step;
    const float x = *reinterpret_cast<const float *>(p + a.ox);
    const float y = *reinterpret_cast<const float *>(p + a.oy);
    const float z = *reinterpret_cast<const float *>(p + a.oz);
    float X, Y, Z;
    xform_pt(a.r, x, y, z, X, Y, Z);
    if (!(isfinite(X) && isfinite(Y) && isfinite(Z))) return;
    const int gx = (int)(((double)X - a.origin_x) / a.res);   // truncation, as the reference
    const int gy = (int)(((double)Y - a.origin_y) / a.res);
    if (gx < 0 || gx >= a.gw || gy < 0 || gy >= a.gh) return;
    const uint32_t c = (uint32_t)gy * (uint32_t)a.gw + (uint32_t)gx;
    atomicAdd(&cnt[c], 1u);
    const int32_t k = fkey(Z);
    atomicMin(&zlo[c], k);
    atomicMax(&zhi[c], k);
}

__global__ void __launch_bounds__(kDT)
k_driv_init(uint32_t ncell, uint32_t *__restrict__ cnt, int32_t *__restrict__ zlo,
            int32_t *__restrict__ zhi) {
    const uint32_t c = blockIdx.x * kDT + threadIdx.x;
    if (c >= ncell) return;
    cnt[c] = 0;
    zlo[c] = INT32_MAX;
    zhi[c] = INT32_MIN;
}

struct DrivRule {
    double origin_x, origin_y, res, start_x, start_y, clear_r, max_gradient;
    int32_t gw, gh, min_points;
};

__global__ void __launch_bounds__(kDT)
k_driv_classify(DrivRule R, const uint32_t *__restrict__ cnt, const int32_t *__restrict__ zlo,
                const int32_t *__restrict__ zhi, int8_t *__restrict__ grid) {
    const uint32_t c = blockIdx.x * kDT + threadIdx.x;
    if (c >= (uint32_t)R.gw * (uint32_t)R.gh) return;
    const int x = (int)(c % (uint32_t)R.gw), y = (int)(c / (uint32_t)R.gw);
    const double cell_x = R.origin_x + (x + 0.5) * R.res;
    const double cell_y = R.origin_y + (y + 0.5) * R.res;
    const double dx = cell_x - R.start_x, dy = cell_y - R.start_y;
    const double dist = sqrt(dx * dx + dy * dy);   // std::pow(d, 2) is the correctly rounded d*d
    int8_t v;
    if (dist <= R.clear_r) {
        v = 0;
    } else if (cnt[c] == 0 || (uint64_t)cnt[c] < (uint64_t)(int64_t)R.min_points) {
        // static_cast<size_t>(min_points_per_cell_): a negative value compares as huge
        v = -1;
    } else {
        float gradient = 0.0f;
        if (cnt[c] >= 2) {
            const float mn = fkey_inv(zlo[c]), mx = fkey_inv(zhi[c]);
            gradient = (float)((double)(mx - mn) / R.res);
        }
        v = gradient > R.max_gradient ? 100 : 0;
    }
    grid[c] = v;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_drivable_area(pcp_ctx *ctx, const pcp_cloud_view *cloud, const pcp_rigid *cloud_to_map,
                      double robot_x, double robot_y, double start_x, double start_y,
                      const pcp_drivable_params *p, int8_t *grid, uint64_t cap, int32_t dims[2],
                      double origin[2]) {
    if (!ctx) return PCP_E_INVALID;
    if (!cloud_to_map || !p || !dims || !origin)
        return set_err(ctx, PCP_E_INVALID, "pcp_drivable_area: null argument");
    int rc = check_view(ctx, cloud, "pcp_drivable_area");
    if (rc) return rc;
    if (!(p->grid_resolution > 0.0))
        return set_err(ctx, PCP_E_INVALID, "pcp_drivable_area: grid_resolution must be > 0");
    const int gw = (int)(p->map_width / p->grid_resolution);
    const int gh = (int)(p->map_height / p->grid_resolution);
    dims[0] = gw > 0 ? gw : 0;
    dims[1] = gh > 0 ? gh : 0;
    origin[0] = robot_x - p->map_width / 2.0;   // :137-139
    origin[1] = robot_y - p->map_height / 2.0;
    const uint64_t ncell = (uint64_t)dims[0] * (uint64_t)dims[1];
    if (cloud->n == 0) return PCP_OK;   // "Received empty point cloud": nothing published
    if (ncell > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_drivable_area: %llu cells, cap %llu",
                       (unsigned long long)ncell, (unsigned long long)cap);
    if (ncell >= (1ull << 31))
        return set_err(ctx, PCP_E_INVALID, "pcp_drivable_area: grid too large");
    if (ncell && !grid) return set_err(ctx, PCP_E_INVALID, "pcp_drivable_area: null grid");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const uint64_t bytes = cloud->n * (uint64_t)cloud->point_step;
    PCP_HIP(ctx, ctx->f_in.ensure(bytes + 256));
    PCP_HIP(ctx, hipMemcpyAsync(ctx->f_in.p, cloud->data, bytes, hipMemcpyHostToDevice, st));
    PCP_HIP(ctx, ctx->out_a.ensure(ncell * 12 + ncell + 256));
    uint32_t *cnt = ctx->out_a.as<uint32_t>();
    int32_t *zlo = reinterpret_cast<int32_t *>(cnt + ncell);
    int32_t *zhi = zlo + ncell;
    int8_t *g_d = reinterpret_cast<int8_t *>(zhi + ncell);
    if (!ncell) return PCP_OK;
    const uint8_t rgb0[3] = {0, 0, 0};
    DrivArgs a;
    a.raw = ctx->f_in.as<const unsigned char>();
    a.n = cloud->n;
    a.step = cloud->point_step;
    a.ox = cloud->off_x;
    a.oy = cloud->off_y;
    a.oz = cloud->off_z;
    a.r = make_rigid(*cloud_to_map, rgb0);
    a.origin_x = origin[0];
    a.origin_y = origin[1];
    a.res = p->grid_resolution;
    a.gw = gw;
    a.gh = gh;
    const unsigned gc = (unsigned)((ncell + kDT - 1) / kDT);
    hipLaunchKernelGGL(k_driv_init, dim3(gc), dim3(kDT), 0, st, (uint32_t)ncell, cnt, zlo, zhi);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_driv_bin, dim3((unsigned)((cloud->n + kDT - 1) / kDT)), dim3(kDT), 0, st,
                       a, cnt, zlo, zhi);
    PCP_CHECK_LAUNCH(ctx);
    DrivRule R{origin[0], origin[1], p->grid_resolution, start_x, start_y,
               p->start_clear_radius, p->max_gradient, gw, gh, p->min_points_per_cell};
    hipLaunchKernelGGL(k_driv_classify, dim3(gc), dim3(kDT), 0, st, R, (const uint32_t *)cnt,
                       (const int32_t *)zlo, (const int32_t *)zhi, g_d);
    PCP_CHECK_LAUNCH(ctx);
    PCP_HIP(ctx, hipMemcpyAsync(grid, g_d, ncell, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    return PCP_OK;
}

}  // extern "C"
