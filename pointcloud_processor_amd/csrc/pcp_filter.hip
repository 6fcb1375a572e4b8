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
k_crop_write(CloudIn c, Box b, const uint32_t *__restrict__ counts, uint32_t *__restrict__ m_out,
             uint32_t *__restrict__ kept_idx, float4 *__restrict__ out, float *__restrict__ part) {
    const uint64_t base = (uint64_t)blockIdx.x * kCropTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kFT / 64];
    // this tile's output offset = sum of the kept counts of all earlier tiles (each block sums
    // them itself: no separate scan launch; nb is at most a few thousand)
    uint32_t pre_t = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += kFT) pre_t += counts[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre_t += __shfl_xor(pre_t, o, 64);
    if (lane == 0) wcnt[wid] = pre_t;
    __syncthreads();
    uint32_t run = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *m_out = run + counts[blockIdx.x];
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
    uint32_t m;          // points after the crop
    int32_t overflow;    // PCL int32 guard fired -> passthrough
    int32_t do_voxel;    // leaf > 0
    float inv;
    int32_t min_b[3];
    int32_t div_b[3];
    uint32_t mul1, mul2;
    uint64_t nvox;       // div product (key upper bound)
};

// block-reduced voxel parameters (VoxelGrid::applyFilter arithmetic in float, exactly)
__global__ void __launch_bounds__(kFT)
k_vox_params(const float *__restrict__ part, int nb, const uint32_t *__restrict__ m_d, float leaf,
             VoxParams *__restrict__ vp) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int b = threadIdx.x; b < nb; b += kFT)
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], part[b * 6 + a]);
            mx[a] = fmaxf(mx[a], part[b * 6 + 3 + a]);
        }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
        }
    __shared__ float s[6][kFT / 64];
    if ((threadIdx.x & 63) == 0)
        for (int a = 0; a < 3; ++a) {
            s[a][threadIdx.x >> 6] = mn[a];
            s[3 + a][threadIdx.x >> 6] = mx[a];
        }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < kFT / 64; ++w)
        for (int a = 0; a < 3; ++a) {
            s[a][0] = fminf(s[a][0], s[a][w]);
            s[3 + a][0] = fmaxf(s[3 + a][0], s[3 + a][w]);
        }
    for (int a = 0; a < 3; ++a) {
        mn[a] = s[a][0];
        mx[a] = s[3 + a][0];
    }
    VoxParams p{};
    p.m = *m_d;
    p.do_voxel = leaf > 0.0f ? 1 : 0;
    const float inv = p.do_voxel ? 1.0f / leaf : 0.0f;
    p.inv = inv;
    if (p.m == 0 || !p.do_voxel) {
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

// points that go through the sort: all cropped points when voxelising without overflow
__device__ __forceinline__ uint32_t sort_count(const VoxParams &vp) {
    return (vp.do_voxel && !vp.overflow) ? vp.m : 0u;
}

__global__ void __launch_bounds__(kFT)
k_vox_keys(const float4 *__restrict__ xyz, const VoxParams *__restrict__ vpp,
           uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    for (uint32_t i = blockIdx.x * kFT + threadIdx.x; i < m; i += gridDim.x * kFT) {
        const float4 p = xyz[i];
        const int ijk0 = (int)(floorf(p.x * vp.inv) - (float)vp.min_b[0]);
        const int ijk1 = (int)(floorf(p.y * vp.inv) - (float)vp.min_b[1]);
        const int ijk2 = (int)(floorf(p.z * vp.inv) - (float)vp.min_b[2]);
        keys[i] = (uint32_t)ijk0 + (uint32_t)ijk1 * vp.mul1 + (uint32_t)ijk2 * vp.mul2;
        vals[i] = i;
    }
}

// ---- LSD radix sort (stable), 8-bit digits; tile count from the host-known upper bound -------
__global__ void __launch_bounds__(kFT)
k_radix_hist(const uint32_t *__restrict__ keys, const VoxParams *__restrict__ vpp, int shift,
             uint32_t nblk, uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t m = sort_count(*vpp);
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    if (base < m) {
#pragma unroll 4
        for (int it = 0; it < kSortItems; ++it) {
            const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
            if (i < m) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
        }
    }
    __syncthreads();
    hist[(uint64_t)blockIdx.x * 256 + threadIdx.x] = h[threadIdx.x];
}

// digit offsets of every (tile, digit): base[d] (exclusive over digits of the totals) + sum of
// earlier tiles' counts of d.  One block, thread = digit, tiles read coalesced (block-major).
__global__ void __launch_bounds__(kFT)
k_digit_offsets(const uint32_t *__restrict__ hist, const VoxParams *__restrict__ vpp,
                uint32_t *__restrict__ offs) {
    const uint32_t m = sort_count(*vpp);
    const uint32_t nact = (m + kSortTile - 1) / kSortTile;
    const uint32_t d = threadIdx.x;
    uint32_t tot = 0;
    for (uint32_t t = 0; t < nact; ++t) tot += hist[(size_t)t * 256 + d];
    __shared__ uint32_t lds4[kFT / 64];
    // exclusive scan of the 256 digit totals
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) lds4[wid] = incl;
    __syncthreads();
    uint32_t run = incl - tot;
    for (int w = 0; w < wid; ++w) run += lds4[w];
    for (uint32_t t = 0; t < nact; ++t) {
        offs[(size_t)t * 256 + d] = run;
        run += hist[(size_t)t * 256 + d];
    }
}

__global__ void __launch_bounds__(kFT)
k_radix_scatter(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                const VoxParams *__restrict__ vpp, int shift, uint32_t nblk,
                const uint32_t *__restrict__ offs, uint32_t *__restrict__ kout,
                uint32_t *__restrict__ vout) {
    const uint32_t m = sort_count(*vpp);
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    if (base >= m) return;   // uniform per block
    __shared__ uint32_t run[256];
    __shared__ uint32_t wc[kFT / 64][256];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    run[threadIdx.x] = offs[(uint64_t)blockIdx.x * 256 + threadIdx.x];
    for (int it = 0; it < kSortItems; ++it) {
        const uint64_t i = base + (uint64_t)it * kFT + threadIdx.x;
        const bool act = i < m;
        const uint32_t k = act ? kin[i] : 0u;
        const uint32_t v = act ? vin[i] : 0u;
        const uint32_t d = (k >> shift) & 255u;
        // lanes of this wave with the same digit (match-any from 8 ballots)
        uint64_t same = __ballot(act);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const uint64_t bb = __ballot((d >> bit) & 1u);
            same &= ((d >> bit) & 1u) ? bb : ~bb;
        }
        for (int w = 0; w < kFT / 64; ++w) wc[w][threadIdx.x] = 0;
        __syncthreads();
        const uint32_t rank = (uint32_t)__popcll(same & ((1ull << lane) - 1ull));
        if (act && rank == 0) wc[wid][d] = (uint32_t)__popcll(same);
        __syncthreads();
        if (act) {
            uint32_t pre = run[d];
            for (int w = 0; w < wid; ++w) pre += wc[w][d];
            kout[pre + rank] = k;
            vout[pre + rank] = v;
        }
        __syncthreads();
        run[threadIdx.x] += wc[0][threadIdx.x] + wc[1][threadIdx.x] + wc[2][threadIdx.x] +
                            wc[3][threadIdx.x];
        __syncthreads();
    }
}

// ---- segments + centroids (sizes on the device) ----------------------------------------------
// a sorted position starts a voxel iff its key differs from the previous one
__device__ __forceinline__ bool seg_head(const uint32_t *keys, uint32_t i, uint32_t m) {
    return i < m && (i == 0 || keys[i] != keys[i - 1]);
}

__global__ void __launch_bounds__(kFT)
k_seg_count(const uint32_t *__restrict__ keys, const VoxParams *__restrict__ vpp,
            uint32_t *__restrict__ tcount) {
    const uint32_t m = sort_count(*vpp);
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    uint32_t c = 0;
    if (base < m)
        for (int it = 0; it < kSortItems; ++it)
            c += seg_head(keys, (uint32_t)(base + (uint64_t)it * kFT + threadIdx.x), m) ? 1u : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    __shared__ uint32_t w[kFT / 64];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) tcount[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// seg_start[s] = sorted position of voxel s (ascending key), seg_start[nseg] = m, *nseg_out
__global__ void __launch_bounds__(kFT)
k_seg_emit(const uint32_t *__restrict__ keys, const VoxParams *__restrict__ vpp,
           const uint32_t *__restrict__ tcount, uint32_t *__restrict__ seg_start,
           uint32_t *__restrict__ nseg_out) {
    const uint32_t m = sort_count(*vpp);
    const uint32_t nact = (m + kSortTile - 1) / kSortTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t wcnt[kFT / 64];
    if (blockIdx.x >= nact) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {   // m == 0
            *nseg_out = 0;
            seg_start[0] = 0;
        }
        return;
    }
    uint32_t pre_t = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += kFT) pre_t += tcount[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre_t += __shfl_xor(pre_t, o, 64);
    if (lane == 0) wcnt[wid] = pre_t;
    __syncthreads();
    uint32_t run = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
    for (int it = 0; it < kSortItems; ++it) {
        const uint32_t i = (uint32_t)(base + (uint64_t)it * kFT + threadIdx.x);
        const bool h = seg_head(keys, i, m);
        const uint64_t bal = __ballot(h);
        if (lane == 0) wcnt[wid] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kFT / 64; ++w) {
            pre += (w < wid) ? wcnt[w] : 0u;
            tot += wcnt[w];
        }
        if (h) seg_start[run + pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = i;
        run += tot;
        __syncthreads();
    }
    if (blockIdx.x == nact - 1 && threadIdx.x == 0) {
        *nseg_out = run;
        seg_start[run] = m;
    }
}

// CentroidPoint<PointXYZ>: float sums in (stable) input order, then / (float)n
__global__ void __launch_bounds__(kFT)
k_centroid(const float4 *__restrict__ xyz, const uint32_t *__restrict__ keys,
           const uint32_t *__restrict__ vals, const uint32_t *__restrict__ seg_start,
           const uint32_t *__restrict__ nseg_p, float4 *__restrict__ out,
           uint32_t *__restrict__ out_idx, uint32_t *__restrict__ out_cnt) {
    const uint32_t nseg = *nseg_p;
    for (uint32_t s = blockIdx.x * kFT + threadIdx.x; s < nseg; s += gridDim.x * kFT) {
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
        out_idx[s] = keys[a];
        out_cnt[s] = e - a;
    }
}

// per-cloud result size: voxel count, or the cropped count (crop only / PCL passthrough)
__global__ void k_finish(const VoxParams *__restrict__ vpp, const uint32_t *__restrict__ nseg_p,
                         uint32_t *__restrict__ counts, uint32_t *__restrict__ info, int slot) {
    if (threadIdx.x != 0) return;
    const VoxParams vp = *vpp;
    const bool vox = vp.do_voxel && !vp.overflow;
    counts[slot] = vox ? *nseg_p : vp.m;
    info[2 * slot] = vp.m;          // points after the crop
    info[2 * slot + 1] = vp.overflow;
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

// Affine3f * Vector3f as the homogeneous 4x4 packet product: ((m0 x + m1 y) + m2 z) + t
__device__ __forceinline__ void xform_store(const Rigid &r, float x, float y, float z, float4 *o) {
    const float X = ((r.m00 * x + r.m01 * y) + r.m02 * z) + r.tx;
    const float Y = ((r.m10 * x + r.m11 * y) + r.m12 * z) + r.ty;
    const float Z = ((r.m20 * x + r.m21 * y) + r.m22 * z) + r.tz;
    o[0] = make_float4(X, Y, Z, 1.0f);
    o[1] = make_float4(__uint_as_float(r.rgba), 0.f, 0.f, 0.f);
}

// transform + colour of cloud `slot`'s result into the concatenated output (robot first)
__global__ void __launch_bounds__(kFT)
k_emit_rgb(const float4 *__restrict__ cropped, const float4 *__restrict__ voxels,
           const VoxParams *__restrict__ vpp, const uint32_t *__restrict__ counts, int slot,
           Rigid r, float4 *__restrict__ out) {
    const VoxParams vp = *vpp;
    const float4 *src = (vp.do_voxel && !vp.overflow) ? voxels : cropped;
    uint32_t base = 0;
    for (int j = 0; j < slot; ++j) base += counts[j];
    const uint32_t n = counts[slot];
    for (uint32_t i = blockIdx.x * kFT + threadIdx.x; i < n; i += gridDim.x * kFT) {
        const float4 p = src[i];
        xform_store(r, p.x, p.y, p.z, out + 2 * ((size_t)base + i));
    }
}

// from a raw PointCloud2 blob (pcp_transform_concat)
__global__ void __launch_bounds__(kFT) k_xform_raw(CloudIn c, Rigid r, float4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kFT + threadIdx.x;
    if (i >= c.n) return;
    float x, y, z;
    load_xyz(c, i, x, y, z);
    xform_store(r, x, y, z, out + 2 * i);
}

// =========================================================================================
// host orchestration: every stage enqueued on ctx->stream with sizes kept on the device, so a
// whole crop -> voxel -> transform pipeline runs without host round trips (and can be captured
// into a hipGraph, see pcp_filter_merge).
// =========================================================================================
constexpr int kMaxClouds = 64;

// device views of one cloud's scratch (ctx->fbuf[slot]) plus the shared per-slot results
struct Scratch {
    CloudBufs *B = nullptr;
    uint64_t ncap = 0;        // points the buffers hold
    uint32_t nb = 0;          // crop tiles
    uint32_t nt = 0;          // sort tiles
    uint32_t *counts = nullptr, *mcrop = nullptr;  // crop tile counts, cropped count
    float *part = nullptr;                         // crop bbox partials
    uint32_t *rhist = nullptr, *rhoff = nullptr;   // radix [tile][digit]
    uint32_t *tcount = nullptr, *nseg = nullptr;   // voxel-head counts per sort tile, voxels
    VoxParams *vp = nullptr;  // [kMaxClouds]
    uint32_t *res = nullptr;  // [kMaxClouds] result counts, [2*kMaxClouds] info
    float4 *xyz() const { return B->xyz.as<float4>(); }
    float4 *out4() const { return B->out.as<float4>(); }
    uint32_t *seg_start() const { return reinterpret_cast<uint32_t *>(out4() + ncap + 1); }
    uint32_t *vidx() const { return seg_start() + ncap + 2; }
    uint32_t *vcnt() const { return vidx() + ncap + 1; }
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// (callers holding Scratch objects of several slots must size ctx->fbuf beforehand)
static int ensure_scratch(pcp_ctx *ctx, int slot, uint64_t ncap, bool want_idx, Scratch &S) {
    if ((int)ctx->fbuf.size() <= slot) ctx->fbuf.resize(slot + 1);
    CloudBufs &B = ctx->fbuf[slot];
    S.B = &B;
    ncap = ncap ? ncap : 1;
    S.ncap = ncap;
    S.nb = (uint32_t)((ncap + kCropTile - 1) / kCropTile);
    S.nt = (uint32_t)((ncap + kSortTile - 1) / kSortTile);
    PCP_HIP(ctx, B.xyz.ensure((ncap + 1) * sizeof(float4)));
    if (want_idx) PCP_HIP(ctx, B.idx.ensure((ncap + 1) * sizeof(uint32_t)));
    for (int q = 0; q < 2; ++q) {
        PCP_HIP(ctx, B.keys[q].ensure((ncap + 16) * sizeof(uint32_t)));
        PCP_HIP(ctx, B.vals[q].ensure((ncap + 16) * sizeof(uint32_t)));
    }
    const size_t cb = align256((S.nb + 1) * 4), pb = align256((size_t)S.nb * 24);
    const size_t hb = align256((size_t)S.nt * 256 * 4), tb = align256((S.nt + 1) * 4);
    PCP_HIP(ctx, B.hist.ensure(cb + 256 + pb + 2 * hb + tb + 256));
    char *h = B.hist.as<char>();
    S.counts = reinterpret_cast<uint32_t *>(h);
    S.mcrop = reinterpret_cast<uint32_t *>(h + cb);
    S.part = reinterpret_cast<float *>(h + cb + 256);
    S.rhist = reinterpret_cast<uint32_t *>(h + cb + 256 + pb);
    S.rhoff = reinterpret_cast<uint32_t *>(h + cb + 256 + pb + hb);
    S.tcount = reinterpret_cast<uint32_t *>(h + cb + 256 + pb + 2 * hb);
    S.nseg = S.tcount + S.nt;
    // voxel results: out4 (ncap+1) | seg_start (ncap+2) | idx (ncap+1) | cnt (ncap+1)
    PCP_HIP(ctx, B.out.ensure((ncap + 1) * sizeof(float4) + (3 * ncap + 8) * 4 + 256));
    PCP_HIP(ctx, ctx->f_misc.ensure(align256(kMaxClouds * sizeof(VoxParams)) + 3 * kMaxClouds * 4));
    S.vp = reinterpret_cast<VoxParams *>(ctx->f_misc.as<char>());
    S.res = reinterpret_cast<uint32_t *>(ctx->f_misc.as<char>() + align256(kMaxClouds * sizeof(VoxParams)));
    return PCP_OK;
}

// radix passes needed for the voxel keys: from the crop box when it is finite (keys are below
// prod((hi-lo)/leaf + 3)), else all 32 bits
static int radix_passes(const Box &b, float leaf) {
    const double lo[3] = {b.x0, b.y0, b.z0}, hi[3] = {b.x1, b.y1, b.z1};
    double nv = 1.0;
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return 4;
        nv *= std::floor((hi[a] - lo[a]) / (double)leaf) + 3.0;
    }
    int bits = 0;
    while (bits < 32 && std::ldexp(1.0, bits) < nv) ++bits;
    return std::max(1, (bits + 7) / 8);
}

// enqueue crop [-> voxel] for one cloud into slot `slot` on stream `st` (results stay on the
// device: S.res[slot] = result count)
static int enqueue_cloud(pcp_ctx *ctx, Scratch &S, const CloudIn &c, const Box &b, float leaf,
                         bool want_idx, int slot, hipStream_t st) {
    const uint32_t nb = (uint32_t)((c.n + kCropTile - 1) / kCropTile);
    {
        ProfScope ps(ctx, PCP_K_CROP, st);
        if (nb) {
            hipLaunchKernelGGL(k_crop_count, dim3(nb), dim3(kFT), 0, st, c, b, S.counts);
            PCP_CHECK_LAUNCH(ctx);
            hipLaunchKernelGGL(k_crop_write, dim3(nb), dim3(kFT), 0, st, c, b,
                               (const uint32_t *)S.counts, S.mcrop,
                               want_idx ? S.B->idx.as<uint32_t>() : nullptr, S.xyz(), S.part);
            PCP_CHECK_LAUNCH(ctx);
        } else {
            PCP_HIP(ctx, hipMemsetAsync(S.mcrop, 0, 4, st));
        }
    }
    VoxParams *vp = S.vp + slot;
    ProfScope ps(ctx, PCP_K_VOXEL, st);
    hipLaunchKernelGGL(k_vox_params, dim3(1), dim3(kFT), 0, st, (const float *)S.part, (int)nb,
                       (const uint32_t *)S.mcrop, leaf, vp);
    PCP_CHECK_LAUNCH(ctx);
    const uint32_t *nseg = S.mcrop;
    if (leaf > 0.0f && c.n > 0) {
        const uint32_t ncap = (uint32_t)c.n;
        const unsigned gk = std::min<unsigned>((ncap + kFT - 1) / kFT, 2048);
        CloudBufs &B = *S.B;
        hipLaunchKernelGGL(k_vox_keys, dim3(gk), dim3(kFT), 0, st, (const float4 *)S.xyz(),
                           (const VoxParams *)vp, B.keys[0].as<uint32_t>(), B.vals[0].as<uint32_t>());
        PCP_CHECK_LAUNCH(ctx);
        const uint32_t nblk = (ncap + kSortTile - 1) / kSortTile;
        const int passes = radix_passes(b, leaf);
        int cur = 0;
        for (int pass = 0; pass < passes; ++pass) {
            const int shift = 8 * pass;
            hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(kFT), 0, st,
                               B.keys[cur].as<const uint32_t>(), (const VoxParams *)vp, shift, nblk,
                               S.rhist);
            PCP_CHECK_LAUNCH(ctx);
            hipLaunchKernelGGL(k_digit_offsets, dim3(1), dim3(kFT), 0, st,
                               (const uint32_t *)S.rhist, (const VoxParams *)vp, S.rhoff);
            PCP_CHECK_LAUNCH(ctx);
            hipLaunchKernelGGL(k_radix_scatter, dim3(nblk), dim3(kFT), 0, st,
                               B.keys[cur].as<const uint32_t>(), B.vals[cur].as<const uint32_t>(),
                               (const VoxParams *)vp, shift, nblk, (const uint32_t *)S.rhoff,
                               B.keys[cur ^ 1].as<uint32_t>(), B.vals[cur ^ 1].as<uint32_t>());
            PCP_CHECK_LAUNCH(ctx);
            cur ^= 1;
        }
        const uint32_t *keys = B.keys[cur].as<const uint32_t>();
        const uint32_t *vals = B.vals[cur].as<const uint32_t>();
        hipLaunchKernelGGL(k_seg_count, dim3(nblk), dim3(kFT), 0, st, keys, (const VoxParams *)vp,
                           S.tcount);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_seg_emit, dim3(nblk), dim3(kFT), 0, st, keys, (const VoxParams *)vp,
                           (const uint32_t *)S.tcount, S.seg_start(), S.nseg);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_centroid, dim3(gk), dim3(kFT), 0, st, (const float4 *)S.xyz(), keys,
                           vals, (const uint32_t *)S.seg_start(), (const uint32_t *)S.nseg,
                           S.out4(), S.vidx(), S.vcnt());
        PCP_CHECK_LAUNCH(ctx);
        nseg = S.nseg;
    }
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(64), 0, st, (const VoxParams *)vp, nseg, S.res,
                       S.res + kMaxClouds, slot);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

static int enqueue_emit(pcp_ctx *ctx, Scratch &S, uint64_t ncap, int slot, const Rigid &r,
                        float4 *out) {
    if (ncap == 0) return PCP_OK;
    ProfScope ps(ctx, PCP_K_TRANSFORM);
    const unsigned g = (unsigned)std::min<uint64_t>((ncap + kFT - 1) / kFT, 4096);
    hipLaunchKernelGGL(k_emit_rgb, dim3(g), dim3(kFT), 0, ctx->stream, (const float4 *)S.xyz(),
                       (const float4 *)S.out4(), (const VoxParams *)(S.vp + slot),
                       (const uint32_t *)S.res, slot, r, out);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

static int stage_cloud(pcp_ctx *ctx, const pcp_cloud_view &v, bool device_in, DevBuf &buf,
                       CloudIn &c) {
    c.n = v.n;
    c.step = v.point_step;
    c.ox = v.off_x;
    c.oy = v.off_y;
    c.oz = v.off_z;
    c.raw = nullptr;
    if (v.n == 0) return PCP_OK;
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

struct ResultInfo {
    uint32_t n;          // result points
    uint32_t m;          // points after the crop
    uint32_t overflow;
};

static int read_result(pcp_ctx *ctx, const Scratch &S, int slot, ResultInfo &ri) {
    uint32_t buf[3 * kMaxClouds];
    PCP_HIP(ctx, hipMemcpyAsync(buf, S.res, sizeof(buf), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    ri.n = buf[slot];
    ri.m = buf[kMaxClouds + 2 * slot];
    ri.overflow = buf[kMaxClouds + 2 * slot + 1];
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
    Scratch S;
    if ((rc = ensure_scratch(ctx, 0, in->n, kept_idx != nullptr, S))) return rc;
    CloudIn c;
    if ((rc = stage_cloud(ctx, *in, false, ctx->f_in, c))) return rc;
    const Box b{box[0], box[1], box[2], box[3], box[4], box[5]};
    if ((rc = enqueue_cloud(ctx, S, c, b, 0.0f, kept_idx != nullptr, 0, ctx->stream))) return rc;
    ResultInfo ri;
    if ((rc = read_result(ctx, S, 0, ri))) return rc;
    *n_kept = ri.m;
    if ((kept_idx || out_xyz16) && ri.m > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_crop_box: need %u, cap %llu", ri.m,
                       (unsigned long long)cap);
    }
    if (kept_idx && ri.m)
        PCP_HIP(ctx, hipMemcpyAsync(kept_idx, S.B->idx.p, (size_t)ri.m * 4, hipMemcpyDeviceToHost,
                                    ctx->stream));
    if (out_xyz16 && ri.m)
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, S.xyz(), (size_t)ri.m * 16,
                                    hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

static int crop_voxel_impl(pcp_ctx *ctx, const pcp_cloud_view *in, const Box &b, float leaf,
                           float *out_xyz16, uint32_t *voxel_idx, uint32_t *voxel_count,
                           uint64_t cap, uint64_t *n_out, uint64_t *n_cropped,
                           int32_t *passthrough) {
    Scratch S;
    int rc = ensure_scratch(ctx, 0, in->n, false, S);
    if (rc) return rc;
    CloudIn c;
    if ((rc = stage_cloud(ctx, *in, false, ctx->f_in, c))) return rc;
    if ((rc = enqueue_cloud(ctx, S, c, b, leaf, false, 0, ctx->stream))) return rc;
    ResultInfo ri;
    if ((rc = read_result(ctx, S, 0, ri))) return rc;
    const bool vox = leaf > 0.0f && !ri.overflow;
    if (passthrough) *passthrough = (leaf > 0.0f && ri.overflow) ? 1 : 0;
    if (n_cropped) *n_cropped = ri.m;
    *n_out = ri.n;
    if (ri.n > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "voxel output needs %u points, cap %llu", ri.n,
                       (unsigned long long)cap);
    }
    if (ri.n) {
        const void *src = vox ? (const void *)S.out4() : (const void *)S.xyz();
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, src, (size_t)ri.n * 16, hipMemcpyDeviceToHost,
                                    ctx->stream));
        if (vox && voxel_idx)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_idx, S.vidx(), (size_t)ri.n * 4,
                                        hipMemcpyDeviceToHost, ctx->stream));
        if (vox && voxel_count)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_count, S.vcnt(), (size_t)ri.n * 4,
                                        hipMemcpyDeviceToHost, ctx->stream));
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
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));   // f_in is reused by the next cloud
        base += c.n;
    }
    PCP_HIP(ctx, hipMemcpyAsync(out, o, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

// key of a captured filter_merge graph: everything baked into its nodes
static std::vector<uint8_t> fm_key(int k, const pcp_cloud_view *clouds, const double *boxes,
                                   float leaf, const pcp_rigid *tf, const uint8_t *rgb,
                                   const void *out, uint64_t cap) {
    std::vector<uint8_t> key;
    auto put = [&key](const void *p, size_t n) {
        const uint8_t *b = static_cast<const uint8_t *>(p);
        key.insert(key.end(), b, b + n);
    };
    put(&k, sizeof(k));
    put(clouds, sizeof(pcp_cloud_view) * k);
    put(boxes, sizeof(double) * 6 * k);
    put(&leaf, sizeof(leaf));
    put(tf, sizeof(pcp_rigid) * k);
    put(rgb, 3 * (size_t)k);
    put(&out, sizeof(out));
    put(&cap, sizeof(cap));
    return key;
}

int pcp_filter_merge(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds, const double *boxes,
                     float leaf, const pcp_rigid *tf, const uint8_t *rgb, void *out, uint64_t cap,
                     uint64_t *n_out, uint64_t *n_per_cloud, uint32_t flags) {
    if (!ctx) return PCP_E_INVALID;
    if (k < 0 || k > kMaxClouds || (k && (!clouds || !boxes || !tf || !rgb)) || !n_out)
        return set_err(ctx, PCP_E_INVALID, "pcp_filter_merge: bad argument");
    uint64_t upper = 0;
    for (int i = 0; i < k; ++i) {
        int rc = check_view(ctx, &clouds[i], "pcp_filter_merge");
        if (rc) return rc;
        upper += clouds[i].n;
    }
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    const bool dev_in = flags & PCP_MEM_DEVICE_IN, dev_out = flags & PCP_MEM_DEVICE_OUT;
    if (dev_out && !out && upper) return set_err(ctx, PCP_E_INVALID, "pcp_filter_merge: null output");
    float4 *obuf;
    if (dev_out) {
        obuf = static_cast<float4 *>(out);
    } else {
        PCP_HIP(ctx, ctx->out_d.ensure(upper * 32 + 32));
        obuf = ctx->out_d.as<float4>();
    }
    // staging (host input): one region per cloud, so no buffer is reused while in flight
    std::vector<size_t> soff(k + 1, 0);
    for (int i = 0; i < k; ++i)
        soff[i + 1] = soff[i] + (dev_in ? 0 : align256(clouds[i].n * clouds[i].point_step));
    if (!dev_in) PCP_HIP(ctx, ctx->f_in.ensure(soff[k] + 256));
    // per-cloud scratch and one side stream per cloud (clouds run as concurrent branches).
    // Size fbuf once: Scratch keeps CloudBufs pointers, a later resize would invalidate them.
    if ((int)ctx->fbuf.size() < k) ctx->fbuf.resize(k);
    std::vector<Scratch> S(k);
    for (int i = 0; i < k; ++i) {
        int rc = ensure_scratch(ctx, i, clouds[i].n, false, S[i]);
        if (rc) return rc;
    }
    while ((int)ctx->side.size() < k) {
        hipStream_t s2 = nullptr;
        PCP_HIP(ctx, hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
        ctx->side.push_back(s2);
        hipEvent_t e = nullptr;
        PCP_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->side_ev.push_back(e);
    }
    if (!ctx->fork_ev) PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
    // fork: every cloud's crop/voxel chain on its own stream; join; then the emits (they need
    // every earlier cloud's count for their output offset)
    auto enqueue_all = [&]() -> int {
        PCP_HIP(ctx, hipEventRecord(ctx->fork_ev, ctx->stream));
        for (int i = 0; i < k; ++i) {
            hipStream_t si = ctx->side[i];
            PCP_HIP(ctx, hipStreamWaitEvent(si, ctx->fork_ev, 0));
            CloudIn c{};
            c.n = clouds[i].n;
            c.step = clouds[i].point_step;
            c.ox = clouds[i].off_x;
            c.oy = clouds[i].off_y;
            c.oz = clouds[i].off_z;
            c.raw = static_cast<const unsigned char *>(clouds[i].data);
            if (!dev_in && c.n) {
                unsigned char *dst = ctx->f_in.as<unsigned char>() + soff[i];
                PCP_HIP(ctx, hipMemcpyAsync(dst, clouds[i].data, c.n * (uint64_t)c.step,
                                            hipMemcpyHostToDevice, si));
                c.raw = dst;
            }
            const double *bx = boxes + 6 * i;
            const Box b{bx[0], bx[1], bx[2], bx[3], bx[4], bx[5]};
            int r = enqueue_cloud(ctx, S[i], c, b, leaf, false, i, si);
            if (r) return r;
            PCP_HIP(ctx, hipEventRecord(ctx->side_ev[i], si));
        }
        for (int i = 0; i < k; ++i) PCP_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[i], 0));
        if (dev_out && upper > cap) return PCP_OK;   // sizes checked on the host afterwards
        for (int i = 0; i < k; ++i) {
            int r = enqueue_emit(ctx, S[i], clouds[i].n, i, make_rigid(tf[i], rgb + 3 * i), obuf);
            if (r) return r;
        }
        return PCP_OK;
    };
    int rc = PCP_OK;
    const bool graphable = dev_in && dev_out && upper <= cap && ctx->use_graphs;
    if (graphable) {
        std::vector<uint8_t> key = fm_key(k, clouds, boxes, leaf, tf, rgb, out, cap);
        std::vector<const void *> sp;
        for (int i = 0; i < k; ++i) {
            const CloudBufs &B = ctx->fbuf[i];
            const void *v[] = {B.xyz.p, B.keys[0].p, B.keys[1].p, B.vals[0].p, B.vals[1].p,
                               B.hist.p, B.out.p};
            sp.insert(sp.end(), v, v + 7);
        }
        sp.push_back(ctx->f_misc.p);
        key.insert(key.end(), reinterpret_cast<const uint8_t *>(sp.data()),
                   reinterpret_cast<const uint8_t *>(sp.data() + sp.size()));
        if (!ctx->fm_exec || key != ctx->fm_key) {
            if (ctx->fm_exec) (void)hipGraphExecDestroy(ctx->fm_exec);
            if (ctx->fm_graph) (void)hipGraphDestroy(ctx->fm_graph);
            ctx->fm_exec = nullptr;
            ctx->fm_graph = nullptr;
            ctx->fm_key.clear();
            PCP_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
            ctx->capturing = true;
            rc = enqueue_all();
            ctx->capturing = false;
            hipGraph_t g = nullptr;
            const hipError_t e = hipStreamEndCapture(ctx->stream, &g);
            if (rc) {
                if (g) (void)hipGraphDestroy(g);
                return rc;
            }
            if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamEndCapture", __FILE__, __LINE__);
            ctx->fm_graph = g;
            PCP_HIP(ctx, hipGraphInstantiate(&ctx->fm_exec, g, nullptr, nullptr, 0));
            ctx->fm_key = key;
        }
        ProfScope ps(ctx, PCP_K_FILTER_MERGE);
        PCP_HIP(ctx, hipGraphLaunch(ctx->fm_exec, ctx->stream));
    } else {
        ProfScope ps(ctx, PCP_K_FILTER_MERGE);
        rc = enqueue_all();
        if (rc) return rc;
    }
    uint32_t res[3 * kMaxClouds];
    PCP_HIP(ctx, hipMemcpyAsync(res, ctx->f_misc.as<char>() + align256(kMaxClouds * sizeof(VoxParams)),
                                sizeof(res), hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint64_t total = 0;
    for (int i = 0; i < k; ++i) {
        if (n_per_cloud) n_per_cloud[i] = clouds[i].n ? res[i] : 0;
        total += clouds[i].n ? res[i] : 0;
    }
    *n_out = total;
    if (total > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_filter_merge: need %llu, cap %llu",
                       (unsigned long long)total, (unsigned long long)cap);
    }
    if (dev_out && upper > cap && total) {   // emits were deferred until the size was known
        for (int i = 0; i < k; ++i) {
            rc = enqueue_emit(ctx, S[i], clouds[i].n, i, make_rigid(tf[i], rgb + 3 * i), obuf);
            if (rc) return rc;
        }
    }
    if (!dev_out && total)
        PCP_HIP(ctx, hipMemcpyAsync(out, obuf, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

}  // extern "C"
