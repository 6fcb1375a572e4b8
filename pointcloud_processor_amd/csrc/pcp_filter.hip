// pcp_filter.hip -- pointcloud_filter.cpp (crop + VoxelGrid) and pointcloud_merger.cpp
// (tf2::doTransform + colour + concat) on gfx950.
//
//  crop    : two-pass stable stream compaction (wave ballot + block scan, order kept)
//  voxel   : PCL VoxelGrid<PointXYZ> keying in float exactly as applyFilter, stable LSD
//            radix sort of (key, cropped index) with 8-bit digits, segment heads + scan,
//            per-voxel float centroid summed in input order
//  merge   : Eigen float Affine3f * p = ((m0 x + m1 y) + m2 z) + t, PointXYZRGB records
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "pcp_internal.hpp"

namespace pcp {

constexpr int kFT = 256;            // threads per block
constexpr int kCropItems = 16;      // points per thread per crop block
constexpr int kCropTile = kFT * kCropItems;
constexpr int kSortItems = 16;
constexpr int kSortTile = kFT * kSortItems;

struct CloudIn {
    const unsigned char *raw;
    uint64_t n;
    uint32_t step, ox, oy, oz;
};

__device__ __forceinline__ void load_xyz(const CloudIn &c, uint64_t i, float &x, float &y,
                                         float &z) {
    const unsigned char *p = c.raw + i * c.step;
    if (c.step == 16 && c.ox == 0 && c.oy == 4 && c.oz == 8) {
        const float4 v = *reinterpret_cast<const float4 *>(p);
        x = v.x;
        y = v.y;
        z = v.z;
    } else {
        x = *reinterpret_cast<const float *>(p + c.ox);
        y = *reinterpret_cast<const float *>(p + c.oy);
        z = *reinterpret_cast<const float *>(p + c.oz);
    }
}

struct Box {
    double x0, x1, y0, y1, z0, z1;
};

// cropFrontArea predicate (pointcloud_filter.cpp:111-113): float promoted to double
__device__ __forceinline__ bool in_box(const Box &b, float x, float y, float z) {
    const double dx = x, dy = y, dz = z;
    return dx > b.x0 && dx < b.x1 && dy > b.y0 && dy < b.y1 && dz > b.z0 && dz < b.z1;
}

// ---- crop pass 1: per-block kept counts --------------------------------------------------
__global__ void __launch_bounds__(kFT) k_crop_count(CloudIn c, Box b, uint32_t *__restrict__ counts) {
    const uint64_t base = (uint64_t)blockIdx.x * kCropTile;
    uint32_t cnt = 0;
#pragma unroll 4
    for (int it = 0; it < kCropItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
        if (i < c.n) {
            float x, y, z;
            load_xyz(c, i, x, y, z);
            cnt += in_box(b, x, y, z) ? 1u : 0u;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    __shared__ uint32_t w[kFT / 64];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// ---- crop pass 2: stable write + bbox partials of the kept points -------------------------
__global__ void __launch_bounds__(kFT)
k_crop_write(CloudIn c, Box b, const uint32_t *__restrict__ offs, uint32_t *__restrict__ kept_idx,
             float4 *__restrict__ out, float *__restrict__ part) {
    const uint64_t base = (uint64_t)blockIdx.x * kCropTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kFT / 64];
    uint32_t run = offs[blockIdx.x];
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int it = 0; it < kCropItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
        float x = 0.f, y = 0.f, z = 0.f;
        bool keep = false;
        if (i < c.n) {
            load_xyz(c, i, x, y, z);
            keep = in_box(b, x, y, z);
        }
        const uint64_t bal = __ballot(keep);
        if (lane == 0) wcnt[wid] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kFT / 64; ++w) {
            const uint32_t v = wcnt[w];
            pre += (w < wid) ? v : 0u;
            tot += v;
        }
        if (keep) {
            const uint32_t d = run + pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            if (kept_idx) kept_idx[d] = (uint32_t)i;
            if (out) out[d] = make_float4(x, y, z, 1.0f);
            mn[0] = fminf(mn[0], x); mx[0] = fmaxf(mx[0], x);
            mn[1] = fminf(mn[1], y); mx[1] = fmaxf(mx[1], y);
            mn[2] = fminf(mn[2], z); mx[2] = fmaxf(mx[2], z);
        }
        run += tot;
        __syncthreads();
    }
    // bbox partials (used by the voxel stage; exact min/max, order-free)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
        }
    }
    __shared__ float s[6][kFT / 64];
    if (lane == 0)
        for (int a = 0; a < 3; ++a) {
            s[a][wid] = mn[a];
            s[3 + a][wid] = mx[a];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int a = threadIdx.x;
        float v = s[a][0];
        for (int w = 1; w < kFT / 64; ++w) v = (a < 3) ? fminf(v, s[a][w]) : fmaxf(v, s[a][w]);
        part[blockIdx.x * 6 + a] = v;
    }
}

// ---- voxel parameters (VoxelGrid::applyFilter, computed in float exactly) -------------------
struct VoxParams {
    uint32_t m;          // points into the voxel stage
    int32_t overflow;    // PCL int32 guard fired -> passthrough
    float inv;
    int32_t min_b[3];
    int32_t div_b[3];
    uint32_t mul1, mul2;
    uint64_t nvox;       // div product (key upper bound)
};

__global__ void k_vox_params(const float *__restrict__ part, int nb, const uint32_t *__restrict__ m_d,
                             float leaf, VoxParams *__restrict__ vp) {
    if (threadIdx.x != 0) return;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int b = 0; b < nb; ++b)
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], part[b * 6 + a]);
            mx[a] = fmaxf(mx[a], part[b * 6 + 3 + a]);
        }
    VoxParams p{};
    p.m = *m_d;
    const float inv = 1.0f / leaf;
    p.inv = inv;
    if (p.m == 0) {
        *vp = p;
        return;
    }
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    p.overflow = (dx * dy * dz > (int64_t)INT32_MAX) ? 1 : 0;
    for (int a = 0; a < 3; ++a) {
        p.min_b[a] = (int32_t)floorf(mn[a] * inv);
        const int32_t max_b = (int32_t)floorf(mx[a] * inv);
        p.div_b[a] = max_b - p.min_b[a] + 1;
    }
    p.mul1 = (uint32_t)p.div_b[0];
    p.mul2 = (uint32_t)p.div_b[0] * (uint32_t)p.div_b[1];
    p.nvox = (uint64_t)(uint32_t)p.div_b[0] * (uint64_t)(uint32_t)p.div_b[1] *
             (uint64_t)(uint32_t)p.div_b[2];
    *vp = p;
}

__global__ void __launch_bounds__(kFT)
k_vox_keys(const float4 *__restrict__ xyz, const VoxParams *__restrict__ vpp,
           uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const VoxParams vp = *vpp;
    const uint32_t i = blockIdx.x * kFT + threadIdx.x;
    if (i >= vp.m) return;
    const float4 p = xyz[i];
    const int ijk0 = (int)(floorf(p.x * vp.inv) - (float)vp.min_b[0]);
    const int ijk1 = (int)(floorf(p.y * vp.inv) - (float)vp.min_b[1]);
    const int ijk2 = (int)(floorf(p.z * vp.inv) - (float)vp.min_b[2]);
    keys[i] = (uint32_t)ijk0 + (uint32_t)ijk1 * vp.mul1 + (uint32_t)ijk2 * vp.mul2;
    vals[i] = i;
}

// ---- LSD radix sort (stable), 8-bit digit -------------------------------------------------
__global__ void __launch_bounds__(kFT)
k_radix_hist(const uint32_t *__restrict__ keys, uint32_t m, int shift, uint32_t nblk,
             uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll 4
    for (int it = 0; it < kSortItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
        if (i < m) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(uint64_t)threadIdx.x * nblk + blockIdx.x] = h[threadIdx.x];
}

__global__ void __launch_bounds__(kFT)
k_radix_scatter(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin, uint32_t m,
                int shift, uint32_t nblk, const uint32_t *__restrict__ offs,
                uint32_t *__restrict__ kout, uint32_t *__restrict__ vout) {
    __shared__ uint32_t run[256];
    __shared__ uint32_t wc[kFT / 64][256];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    run[threadIdx.x] = offs[(uint64_t)threadIdx.x * nblk + blockIdx.x];
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    for (int it = 0; it < kSortItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
        const bool act = i < m;
        const uint32_t k = act ? kin[i] : 0u;
        const uint32_t v = act ? vin[i] : 0u;
        const uint32_t d = (k >> shift) & 255u;
        // lanes of this wave with the same digit (match_any by 8 ballots)
        uint64_t same = __ballot(act);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const uint64_t bb = __ballot((d >> bit) & 1u);
            same &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        for (int w = 0; w < kFT / 64; ++w) wc[w][threadIdx.x] = 0;
        __syncthreads();
        const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        const bool leader = act && rank == 0;
        if (leader) wc[wid][d] = (uint32_t)__popcll(same);
        __syncthreads();
        if (act) {
            uint32_t pre = run[d];
            for (int w = 0; w < wid; ++w) pre += wc[w][d];
            const uint32_t pos = pre + rank;
            kout[pos] = k;
            vout[pos] = v;
        }
        __syncthreads();
        {
            const uint32_t dd = threadIdx.x;   // 256 threads = 256 digits
            run[dd] += wc[0][dd] + wc[1][dd] + wc[2][dd] + wc[3][dd];
        }
        __syncthreads();
    }
}

// ---- segments + centroids -------------------------------------------------------------------
__global__ void __launch_bounds__(kFT)
k_seg_heads(const uint32_t *__restrict__ keys, uint32_t m, uint32_t *__restrict__ head) {
    const uint32_t i = blockIdx.x * kFT + threadIdx.x;
    if (i >= m) return;
    head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void __launch_bounds__(kFT)
k_seg_start(const uint32_t *__restrict__ head, const uint32_t *__restrict__ sid, uint32_t m,
            uint32_t *__restrict__ seg_start) {
    const uint32_t i = blockIdx.x * kFT + threadIdx.x;
    if (i < m && head[i]) seg_start[sid[i]] = i;
    if (i == 0) seg_start[sid[m]] = m;
}

// CentroidPoint<PointXYZ>: float sums in (stable) input order, then / (float)n
__global__ void __launch_bounds__(kFT)
k_centroid(const float4 *__restrict__ xyz, const uint32_t *__restrict__ keys,
           const uint32_t *__restrict__ vals, const uint32_t *__restrict__ seg_start,
           const uint32_t *__restrict__ nseg_p, float4 *__restrict__ out,
           uint32_t *__restrict__ out_idx, uint32_t *__restrict__ out_cnt) {
    const uint32_t s = blockIdx.x * kFT + threadIdx.x;
    if (s >= *nseg_p) return;
    const uint32_t a = seg_start[s], e = seg_start[s + 1];
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for (uint32_t l = a; l < e; ++l) {
        const float4 p = xyz[vals[l]];
        sx = sx + p.x;
        sy = sy + p.y;
        sz = sz + p.z;
    }
    const float cnt = (float)(e - a);
    out[s] = make_float4(sx / cnt, sy / cnt, sz / cnt, 1.0f);
    if (out_idx) out_idx[s] = keys[a];
    if (out_cnt) out_cnt[s] = e - a;
}

// ---- SE(3) + colour (tf2::doTransform + processRobotCloud loop) ------------------------------
struct Rigid {
    float m00, m01, m02, m10, m11, m12, m20, m21, m22, tx, ty, tz;
    uint32_t rgba;
};

static Rigid make_rigid(const pcp_rigid &t, const uint8_t rgb[3]) {
    // Eigen::Quaternionf(w,x,y,z).toRotationMatrix() in float
    const float qx = (float)t.q[0], qy = (float)t.q[1], qz = (float)t.q[2], qw = (float)t.q[3];
    const float tx = 2.0f * qx, ty = 2.0f * qy, tz = 2.0f * qz;
    const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
    const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    Rigid r;
    r.m00 = 1.0f - (tyy + tzz);
    r.m01 = txy - twz;
    r.m02 = txz + twy;
    r.m10 = txy + twz;
    r.m11 = 1.0f - (txx + tzz);
    r.m12 = tyz - twx;
    r.m20 = txz - twy;
    r.m21 = tyz + twx;
    r.m22 = 1.0f - (txx + tyy);
    r.tx = (float)t.t[0];
    r.ty = (float)t.t[1];
    r.tz = (float)t.t[2];
    r.rgba = (uint32_t)rgb[2] | ((uint32_t)rgb[1] << 8) | ((uint32_t)rgb[0] << 16) | (255u << 24);
    return r;
}

__device__ __forceinline__ void xform_store(const Rigid &r, float x, float y, float z, float4 *o) {
    const float X = ((r.m00 * x + r.m01 * y) + r.m02 * z) + r.tx;
    const float Y = ((r.m10 * x + r.m11 * y) + r.m12 * z) + r.ty;
    const float Z = ((r.m20 * x + r.m21 * y) + r.m22 * z) + r.tz;
    o[0] = make_float4(X, Y, Z, 1.0f);
    o[1] = make_float4(__uint_as_float(r.rgba), 0.f, 0.f, 0.f);
}

// from a float4 xyz stream (voxel/crop output); count from device (or host if cnt_d null)
__global__ void __launch_bounds__(kFT)
k_xform_f4(const float4 *__restrict__ in, const uint32_t *__restrict__ cnt_d, uint32_t cnt_h,
           Rigid r, float4 *__restrict__ out) {
    const uint32_t n = cnt_d ? *cnt_d : cnt_h;
    const uint32_t i = blockIdx.x * kFT + threadIdx.x;
    if (i >= n) return;
    const float4 p = in[i];
    xform_store(r, p.x, p.y, p.z, out + 2 * (size_t)i);
}

// from a raw PointCloud2 blob
__global__ void __launch_bounds__(kFT) k_xform_raw(CloudIn c, Rigid r, float4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kFT + threadIdx.x;
    if (i >= c.n) return;
    float x, y, z;
    load_xyz(c, i, x, y, z);
    xform_store(r, x, y, z, out + 2 * i);
}

// =========================================================================================
// host orchestration
// =========================================================================================
static int stage_cloud(pcp_ctx *ctx, const pcp_cloud_view &v, bool device_in, DevBuf &buf,
                       CloudIn &c) {
    c.n = v.n;
    c.step = v.point_step;
    c.ox = v.off_x;
    c.oy = v.off_y;
    c.oz = v.off_z;
    if (v.n == 0) {
        c.raw = nullptr;
        return PCP_OK;
    }
    if (device_in) {
        c.raw = static_cast<const unsigned char *>(v.data);
        return PCP_OK;
    }
    const uint64_t bytes = v.n * (uint64_t)v.point_step;
    PCP_HIP(ctx, buf.ensure(bytes));
    PCP_HIP(ctx, hipMemcpyAsync(buf.p, v.data, bytes, hipMemcpyHostToDevice, ctx->stream));
    c.raw = buf.as<const unsigned char>();
    return PCP_OK;
}

// crop into ctx->f_xyz (float4) [+ kept idx into ctx->f_idx]; device count at *m_d; bbox
// partials in part (nb*6).  Returns nb through *nb_out.
static int run_crop(pcp_ctx *ctx, const CloudIn &c, const Box &b, bool want_idx, uint32_t **m_d,
                    float **part, int *nb_out) {
    hipStream_t st = ctx->stream;
    const uint64_t nb = (c.n + kCropTile - 1) / kCropTile;
    const uint64_t nbx = nb ? nb : 1;
    PCP_HIP(ctx, ctx->f_xyz.ensure((c.n + 1) * sizeof(float4)));
    if (want_idx) PCP_HIP(ctx, ctx->f_idx.ensure((c.n + 1) * sizeof(uint32_t)));
    const size_t cnt_bytes = (nbx + 1) * sizeof(uint32_t);
    const size_t offs_bytes = (nbx + 1) * sizeof(uint32_t);
    const size_t part_bytes = nbx * 6 * sizeof(float);
    const size_t tmp_bytes = scan_tmp_bytes(nbx);
    PCP_HIP(ctx, ctx->f_hist.ensure(cnt_bytes + offs_bytes + part_bytes + tmp_bytes + 1024));
    char *h = ctx->f_hist.as<char>();
    uint32_t *counts = reinterpret_cast<uint32_t *>(h);
    uint32_t *offs = reinterpret_cast<uint32_t *>(h + cnt_bytes);
    float *pp = reinterpret_cast<float *>(h + cnt_bytes + offs_bytes);
    void *tmp = h + cnt_bytes + offs_bytes + part_bytes + 256;
    if (nb == 0) {
        PCP_HIP(ctx, hipMemsetAsync(offs, 0, sizeof(uint32_t), st));
        float init[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
        PCP_HIP(ctx, hipMemcpyAsync(pp, init, sizeof(init), hipMemcpyHostToDevice, st));
        PCP_HIP(ctx, hipStreamSynchronize(st));
        *m_d = offs;
        *part = pp;
        *nb_out = 1;
        return PCP_OK;
    }
    {
        ProfScope ps(ctx, PCP_K_CROP);
        hipLaunchKernelGGL(k_crop_count, dim3((unsigned)nb), dim3(kFT), 0, st, c, b, counts);
        PCP_CHECK_LAUNCH(ctx);
        int rc = exclusive_scan_u32(ctx, counts, offs, nb, tmp);
        if (rc) return rc;
        hipLaunchKernelGGL(k_crop_write, dim3((unsigned)nb), dim3(kFT), 0, st, c, b,
                           (const uint32_t *)offs, want_idx ? ctx->f_idx.as<uint32_t>() : nullptr,
                           ctx->f_xyz.as<float4>(), pp);
        PCP_CHECK_LAUNCH(ctx);
    }
    *m_d = offs + nb;   // exclusive scan total
    *part = pp;
    *nb_out = (int)nb;
    return PCP_OK;
}

// voxel stage on ctx->f_xyz[0..m): result float4 in *res (device), count in host *n_out and
// device *nres_d; idx/count device arrays (nullable outputs).  Sets *passthrough.
// NOTE: m_d and part live in ctx->f_hist, which this function re-uses: they are dead after
// k_vox_params; the cropped count is returned in *m_out.
static int run_voxel(pcp_ctx *ctx, const uint32_t *m_d, const float *part, int nb, float leaf,
                     const float4 **res, uint32_t **nres_d, uint32_t **idx_d, uint32_t **cnt_d,
                     uint64_t *n_out, int32_t *passthrough, uint32_t *m_out) {
    hipStream_t st = ctx->stream;
    PCP_HIP(ctx, ctx->f_misc.ensure(4096));
    VoxParams *vp_d = reinterpret_cast<VoxParams *>(ctx->f_misc.as<char>());
    uint32_t *nseg_d = reinterpret_cast<uint32_t *>(ctx->f_misc.as<char>() + 512);
    ProfScope ps(ctx, PCP_K_VOXEL);
    hipLaunchKernelGGL(k_vox_params, dim3(1), dim3(64), 0, st, part, nb, m_d, leaf, vp_d);
    PCP_CHECK_LAUNCH(ctx);
    VoxParams vp;
    PCP_HIP(ctx, hipMemcpyAsync(&vp, vp_d, sizeof(vp), hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    const uint32_t m = vp.m;
    *m_out = m;
    *passthrough = 0;
    *idx_d = nullptr;
    *cnt_d = nullptr;
    if (m == 0) {
        *res = ctx->f_xyz.as<const float4>();
        PCP_HIP(ctx, hipMemsetAsync(nseg_d, 0, 4, st));
        *nres_d = nseg_d;
        *n_out = 0;
        return PCP_OK;
    }
    if (vp.overflow) {   // PCL: "Leaf size is too small ... Integer indices would overflow."
        *passthrough = 1;
        *res = ctx->f_xyz.as<const float4>();
        *nres_d = nullptr;
        *n_out = m;
        return PCP_OK;
    }
    const size_t mb = ((size_t)m + 16) * sizeof(uint32_t);
    for (int q = 0; q < 2; ++q) {
        PCP_HIP(ctx, ctx->f_keys[q].ensure(mb));
        PCP_HIP(ctx, ctx->f_vals[q].ensure(mb));
    }
    const unsigned gm = (m + kFT - 1) / kFT;
    hipLaunchKernelGGL(k_vox_keys, dim3(gm), dim3(kFT), 0, st, ctx->f_xyz.as<const float4>(),
                       (const VoxParams *)vp_d, ctx->f_keys[0].as<uint32_t>(),
                       ctx->f_vals[0].as<uint32_t>());
    PCP_CHECK_LAUNCH(ctx);
    int bits = 0;
    while (bits < 32 && (vp.nvox - 1) >> bits) ++bits;
    const int passes = (bits + 7) / 8;
    const uint32_t nblk = (m + kSortTile - 1) / kSortTile;
    const uint64_t hn = 256ull * nblk;
    PCP_HIP(ctx, ctx->f_hist.ensure(2 * (hn + 1) * sizeof(uint32_t) + scan_tmp_bytes(hn) + 1024));
    uint32_t *hist = ctx->f_hist.as<uint32_t>();
    uint32_t *hoff = hist + hn + 1;
    void *tmp = hoff + hn + 1;
    int cur = 0;
    for (int pass = 0; pass < passes; ++pass) {
        const int shift = 8 * pass;
        hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(kFT), 0, st,
                           ctx->f_keys[cur].as<const uint32_t>(), m, shift, nblk, hist);
        PCP_CHECK_LAUNCH(ctx);
        int rc = exclusive_scan_u32(ctx, hist, hoff, hn, tmp);
        if (rc) return rc;
        hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(kFT), 0, st,
                           ctx->f_keys[cur].as<const uint32_t>(), ctx->f_vals[cur].as<const uint32_t>(),
                           m, shift, nblk, (const uint32_t *)hoff, ctx->f_keys[cur ^ 1].as<uint32_t>(),
                           ctx->f_vals[cur ^ 1].as<uint32_t>());
        PCP_CHECK_LAUNCH(ctx);
        cur ^= 1;
    }
    // segments: heads -> scan -> starts -> centroids
    const uint32_t *keys = ctx->f_keys[cur].as<const uint32_t>();
    const uint32_t *vals = ctx->f_vals[cur].as<const uint32_t>();
    uint32_t *head = ctx->f_keys[cur ^ 1].as<uint32_t>();
    uint32_t *sid = ctx->f_vals[cur ^ 1].as<uint32_t>();   // m + 1 entries
    hipLaunchKernelGGL(k_seg_heads, dim3(gm), dim3(kFT), 0, st, keys, m, head);
    PCP_CHECK_LAUNCH(ctx);
    PCP_HIP(ctx, ctx->f_hist.ensure(scan_tmp_bytes(m) + 1024));
    int rc = exclusive_scan_u32(ctx, head, sid, m, ctx->f_hist.p);
    if (rc) return rc;
    // seg_start (m + 1), result float4 (m), idx (m), count (m)
    PCP_HIP(ctx, ctx->f_out.ensure(((size_t)m + 1) * (sizeof(uint32_t) * 3 + sizeof(float4)) + 256));
    float4 *out4 = ctx->f_out.as<float4>();
    uint32_t *seg_start = reinterpret_cast<uint32_t *>(out4 + m + 1);
    uint32_t *oidx = seg_start + m + 1;
    uint32_t *ocnt = oidx + m + 1;
    hipLaunchKernelGGL(k_seg_start, dim3(gm), dim3(kFT), 0, st, (const uint32_t *)head,
                       (const uint32_t *)sid, m, seg_start);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_centroid, dim3(gm), dim3(kFT), 0, st, ctx->f_xyz.as<const float4>(), keys,
                       vals, (const uint32_t *)seg_start, (const uint32_t *)(sid + m), out4, oidx,
                       ocnt);
    PCP_CHECK_LAUNCH(ctx);
    uint32_t nseg = 0;
    PCP_HIP(ctx, hipMemcpyAsync(&nseg, sid + m, 4, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    *res = out4;
    *nres_d = sid + m;
    *idx_d = oidx;
    *cnt_d = ocnt;
    *n_out = nseg;
    return PCP_OK;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_crop_box(pcp_ctx *ctx, const pcp_cloud_view *in, const double box[6], uint32_t *kept_idx,
                 float *out_xyz16, uint64_t cap, uint64_t *n_kept) {
    if (!ctx) return PCP_E_INVALID;
    if (!box || !n_kept) return set_err(ctx, PCP_E_INVALID, "pcp_crop_box: null argument");
    int rc = check_view(ctx, in, "pcp_crop_box");
    if (rc) return rc;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *n_kept = 0;
    if (in->n == 0) return PCP_OK;
    CloudIn c;
    rc = stage_cloud(ctx, *in, false, ctx->f_in, c);
    if (rc) return rc;
    Box b{box[0], box[1], box[2], box[3], box[4], box[5]};
    uint32_t *m_d;
    float *part;
    int nb;
    rc = run_crop(ctx, c, b, kept_idx != nullptr, &m_d, &part, &nb);
    if (rc) return rc;
    uint32_t m = 0;
    PCP_HIP(ctx, hipMemcpyAsync(&m, m_d, 4, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *n_kept = m;
    if ((kept_idx || out_xyz16) && m > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_crop_box: need %u, cap %llu", m,
                       (unsigned long long)cap);
    }
    if (kept_idx && m)
        PCP_HIP(ctx, hipMemcpyAsync(kept_idx, ctx->f_idx.p, (size_t)m * 4, hipMemcpyDeviceToHost,
                                    ctx->stream));
    if (out_xyz16 && m)
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, ctx->f_xyz.p, (size_t)m * 16, hipMemcpyDeviceToHost,
                                    ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

static int crop_voxel_impl(pcp_ctx *ctx, const pcp_cloud_view *in, const Box &b, float leaf,
                           float *out_xyz16, uint32_t *voxel_idx, uint32_t *voxel_count,
                           uint64_t cap, uint64_t *n_out, uint64_t *n_cropped,
                           int32_t *passthrough) {
    CloudIn c;
    int rc = stage_cloud(ctx, *in, false, ctx->f_in, c);
    if (rc) return rc;
    uint32_t *m_d;
    float *part;
    int nb;
    rc = run_crop(ctx, c, b, false, &m_d, &part, &nb);
    if (rc) return rc;
    const float4 *res;
    uint32_t *nres_d, *idx_d = nullptr, *cnt_d = nullptr;
    uint64_t n = 0;
    int32_t pt = 0;
    if (leaf > 0.0f) {
        uint32_t m = 0;
        rc = run_voxel(ctx, m_d, part, nb, leaf, &res, &nres_d, &idx_d, &cnt_d, &n, &pt, &m);
        if (rc) return rc;
        if (n_cropped) *n_cropped = m;
    } else {
        uint32_t m = 0;
        PCP_HIP(ctx, hipMemcpyAsync(&m, m_d, 4, hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        res = ctx->f_xyz.as<const float4>();
        n = m;
        if (n_cropped) *n_cropped = m;
    }
    if (passthrough) *passthrough = pt;
    *n_out = n;
    if (n > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "voxel output needs %llu points, cap %llu",
                       (unsigned long long)n, (unsigned long long)cap);
    }
    if (n) {
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, res, n * 16, hipMemcpyDeviceToHost, ctx->stream));
        if (voxel_idx && idx_d)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_idx, idx_d, n * 4, hipMemcpyDeviceToHost, ctx->stream));
        if (voxel_count && cnt_d)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_count, cnt_d, n * 4, hipMemcpyDeviceToHost, ctx->stream));
    }
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

int pcp_voxel_grid(pcp_ctx *ctx, const pcp_cloud_view *in, float leaf, float *out_xyz16,
                   uint32_t *voxel_idx, uint32_t *voxel_count, uint64_t cap, uint64_t *n_out,
                   int32_t *passthrough) {
    if (!ctx) return PCP_E_INVALID;
    if (!n_out || (cap && !out_xyz16)) return set_err(ctx, PCP_E_INVALID, "pcp_voxel_grid: null argument");
    if (!(leaf > 0.0f)) return set_err(ctx, PCP_E_INVALID, "pcp_voxel_grid: leaf must be > 0");
    int rc = check_view(ctx, in, "pcp_voxel_grid");
    if (rc) return rc;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *n_out = 0;
    if (passthrough) *passthrough = 0;
    if (in->n == 0) return PCP_OK;
    // only non-finite points are dropped (VoxelGrid skips !isXYZFinite points)
    const Box all{-INFINITY, INFINITY, -INFINITY, INFINITY, -INFINITY, INFINITY};
    return crop_voxel_impl(ctx, in, all, leaf, out_xyz16, voxel_idx, voxel_count, cap, n_out,
                           nullptr, passthrough);
}

int pcp_crop_voxel(pcp_ctx *ctx, const pcp_cloud_view *in, const double box[6], float leaf,
                   float *out_xyz16, uint64_t cap, uint64_t *n_out, uint64_t *n_cropped) {
    if (!ctx) return PCP_E_INVALID;
    if (!box || !n_out || (cap && !out_xyz16))
        return set_err(ctx, PCP_E_INVALID, "pcp_crop_voxel: null argument");
    int rc = check_view(ctx, in, "pcp_crop_voxel");
    if (rc) return rc;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *n_out = 0;
    if (n_cropped) *n_cropped = 0;
    if (in->n == 0) return PCP_OK;
    const Box b{box[0], box[1], box[2], box[3], box[4], box[5]};
    return crop_voxel_impl(ctx, in, b, leaf, out_xyz16, nullptr, nullptr, cap, n_out, n_cropped,
                           nullptr);
}

int pcp_transform_concat(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds, const pcp_rigid *tf,
                         const uint8_t *rgb, void *out, uint64_t cap, uint64_t *n_out) {
    if (!ctx) return PCP_E_INVALID;
    if (k < 0 || (k && (!clouds || !tf || !rgb)) || !n_out)
        return set_err(ctx, PCP_E_INVALID, "pcp_transform_concat: bad argument");
    uint64_t total = 0;
    for (int i = 0; i < k; ++i) {
        int rc = check_view(ctx, &clouds[i], "pcp_transform_concat");
        if (rc) return rc;
        total += clouds[i].n;
    }
    *n_out = total;
    if (total > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_transform_concat: need %llu, cap %llu",
                       (unsigned long long)total, (unsigned long long)cap);
    if (total == 0) return PCP_OK;
    if (!out) return set_err(ctx, PCP_E_INVALID, "pcp_transform_concat: null output");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, ctx->out_d.ensure(total * 32));
    float4 *o = ctx->out_d.as<float4>();
    uint64_t base = 0;
    for (int i = 0; i < k; ++i) {
        if (clouds[i].n == 0) continue;
        CloudIn c;
        int rc = stage_cloud(ctx, clouds[i], false, ctx->f_in, c);
        if (rc) return rc;
        const Rigid r = make_rigid(tf[i], rgb + 3 * i);
        {
            ProfScope ps(ctx, PCP_K_TRANSFORM);
            hipLaunchKernelGGL(k_xform_raw, dim3((unsigned)((c.n + kFT - 1) / kFT)), dim3(kFT), 0,
                               ctx->stream, c, r, o + 2 * base);
            PCP_CHECK_LAUNCH(ctx);
        }
        // f_in is reused by the next cloud: finish this one first
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        base += c.n;
    }
    PCP_HIP(ctx, hipMemcpyAsync(out, o, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

int pcp_filter_merge(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds, const double *boxes,
                     float leaf, const pcp_rigid *tf, const uint8_t *rgb, void *out, uint64_t cap,
                     uint64_t *n_out, uint64_t *n_per_cloud, uint32_t flags) {
    if (!ctx) return PCP_E_INVALID;
    if (k < 0 || (k && (!clouds || !boxes || !tf || !rgb)) || !n_out)
        return set_err(ctx, PCP_E_INVALID, "pcp_filter_merge: bad argument");
    for (int i = 0; i < k; ++i) {
        int rc = check_view(ctx, &clouds[i], "pcp_filter_merge");
        if (rc) return rc;
    }
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const bool dev_in = flags & PCP_MEM_DEVICE_IN, dev_out = flags & PCP_MEM_DEVICE_OUT;
    // worst case output = sum of inputs; results land in a device buffer, then out
    uint64_t upper = 0;
    for (int i = 0; i < k; ++i) upper += clouds[i].n;
    float4 *obuf;
    if (dev_out) {
        obuf = static_cast<float4 *>(out);
    } else {
        PCP_HIP(ctx, ctx->out_d.ensure(upper * 32 + 32));
        obuf = ctx->out_d.as<float4>();
    }
    uint64_t base = 0;
    for (int i = 0; i < k; ++i) {
        uint64_t n = 0;
        if (clouds[i].n) {
            CloudIn c;
            int rc = stage_cloud(ctx, clouds[i], dev_in, ctx->f_in, c);
            if (rc) return rc;
            const double *bx = boxes + 6 * i;
            const Box b{bx[0], bx[1], bx[2], bx[3], bx[4], bx[5]};
            uint32_t *m_d;
            float *part;
            int nb;
            rc = run_crop(ctx, c, b, false, &m_d, &part, &nb);
            if (rc) return rc;
            const float4 *res = ctx->f_xyz.as<const float4>();
            uint32_t *nres_d = m_d;
            if (leaf > 0.0f) {
                uint32_t *idx_d, *cnt_d, m = 0;
                int32_t pt;
                rc = run_voxel(ctx, m_d, part, nb, leaf, &res, &nres_d, &idx_d, &cnt_d, &n, &pt, &m);
                if (rc) return rc;
            } else {
                uint32_t m = 0;
                PCP_HIP(ctx, hipMemcpyAsync(&m, m_d, 4, hipMemcpyDeviceToHost, ctx->stream));
                PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
                n = m;
            }
            if (dev_out && base + n > cap) {
                *n_out = base + n;
                prof_resolve(ctx);
                return set_err(ctx, PCP_E_CAPACITY, "pcp_filter_merge: output capacity %llu",
                               (unsigned long long)cap);
            }
            if (n) {
                const Rigid r = make_rigid(tf[i], rgb + 3 * i);
                ProfScope ps(ctx, PCP_K_TRANSFORM);
                hipLaunchKernelGGL(k_xform_f4, dim3((unsigned)((n + kFT - 1) / kFT)), dim3(kFT), 0,
                                   ctx->stream, res, (const uint32_t *)nullptr, (uint32_t)n, r,
                                   obuf + 2 * base);
                PCP_CHECK_LAUNCH(ctx);
            }
            // scratch (f_xyz, f_out) is reused by the next cloud
            PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        }
        if (n_per_cloud) n_per_cloud[i] = n;
        base += n;
    }
    *n_out = base;
    if (!dev_out) {
        if (base > cap) {
            prof_resolve(ctx);
            return set_err(ctx, PCP_E_CAPACITY, "pcp_filter_merge: need %llu, cap %llu",
                           (unsigned long long)base, (unsigned long long)cap);
        }
        if (base)
            PCP_HIP(ctx, hipMemcpyAsync(out, obuf, base * 32, hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    prof_resolve(ctx);
    return PCP_OK;
}

}  // extern "C"
