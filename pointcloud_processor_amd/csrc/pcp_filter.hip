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
constexpr int kCropItems = 16;      // points per thread per crop tile
constexpr int kCropTile = kFT * kCropItems;
constexpr int kST = 512;            // threads of the sort-tile kernels (8 waves)
constexpr int kSW = kST / 64;
constexpr int kSortItems = 8;       // keys per thread per sort tile
constexpr int kSortTile = kST * kSortItems;
constexpr int kGroup = 16;          // sort tiles per prefix group (radix digit prefix sums)
constexpr int kDigitBits = 9;       // radix digit: 512 bins, 3 passes for the C3 crop box
constexpr int kBins = 1 << kDigitBits;
constexpr int kMaxPasses = 4;       // ceil(32 / 9)

// diagnostic build only (make STAMPS=1): per-tile phase times, s_memrealtime (100 MHz)
#ifdef PCP_STAMPS
constexpr int kStampTiles = 4096, kStampPh = 8;
__device__ unsigned long long g_flt_stamps[2][kStampTiles * kStampPh];   // [scatter, centroid]
#define FLT_STAMP(k, t, ph)                                                                  \
    do {                                                                                      \
        if (threadIdx.x == 0 && (t) < kStampTiles)                                            \
            g_flt_stamps[k][(t) * kStampPh + (ph)] = __builtin_amdgcn_s_memrealtime();        \
    } while (0)
#else
#define FLT_STAMP(k, t, ph) \
    do {                    \
    } while (0)
#endif

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

__device__ __forceinline__ uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// sum of a[0 .. n) (a 16-byte aligned) over the block with 16-byte loads; every thread gets it
template <int NT>
__device__ __forceinline__ uint32_t block_prefix_sum(const uint32_t *__restrict__ a, uint32_t n,
                                                     uint32_t *lds) {
    uint32_t s = 0;
    const uint32_t nq = (n + 3) / 4;
    for (uint32_t q = threadIdx.x; q < nq; q += NT) {
        const uint4 v = reinterpret_cast<const uint4 *>(a)[q];
        const uint32_t b = 4 * q;
        s += v.x + (b + 1 < n ? v.y : 0u) + (b + 2 < n ? v.z : 0u) + (b + 3 < n ? v.w : 0u);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = s;
    __syncthreads();
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) t += lds[w];
    return t;
}

// exclusive block scan of one value per thread (thread order); every thread gets its prefix
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    uint32_t ex = incl - v;
    for (int w = 0; w < wid; ++w) ex += lds[w];
    return ex;
}

// ordered compaction offsets of J rounds x W waves: wo[j][w] = kept items before (round j,
// wave w) in (round, wave, lane) order, returns the tile total.  bal: this wave's ballots.
template <int J, int W>
__device__ __forceinline__ uint32_t round_offsets(const uint64_t (&bal)[J], uint32_t (*wo)[W]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    static_assert(J * W == 64, "one wave scans the (round, wave) counts");
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < J; ++j) wo[j][wid] = (uint32_t)__popcll(bal[j]);
    __syncthreads();
    __shared__ uint32_t tot;
    if (threadIdx.x < 64) {
        const int j = threadIdx.x / W, w = threadIdx.x % W;
        const uint32_t v = wo[j][w];
        uint32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (threadIdx.x >= o) incl += u;
        }
        wo[j][w] = incl - v;
        if (threadIdx.x == 63) tot = incl;
    }
    __syncthreads();
    return tot;
}

// ---- crop: one read of the input; stable compaction of each tile into its own slot of a
//      sparse buffer (kept count + bbox partial per tile); k_compact_keys closes the gaps ----
__global__ void __launch_bounds__(kFT)
k_crop_tile(CloudIn c, Box b, uint32_t *__restrict__ counts, float *__restrict__ part,
            float4 *__restrict__ sparse, uint32_t *__restrict__ sparse_idx) {
    const uint64_t base = (uint64_t)blockIdx.x * kCropTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float x[kCropItems], y[kCropItems], z[kCropItems];
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        const uint64_t i = base + (uint64_t)j * kFT + threadIdx.x;
        x[j] = y[j] = z[j] = 0.f;
        if (i < c.n) load_xyz(c, i, x[j], y[j], z[j]);
    }
    uint64_t bal[kCropItems];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        const uint64_t i = base + (uint64_t)j * kFT + threadIdx.x;
        const bool k = i < c.n && in_box(b, x[j], y[j], z[j]);
        keep |= (k ? 1u : 0u) << j;
        bal[j] = __ballot(k);
    }
    __shared__ uint32_t wo[kCropItems][kFT / 64];
    const uint32_t tot = round_offsets(bal, wo);
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        if (!((keep >> j) & 1u)) continue;
        const uint32_t d = wo[j][wid] + (uint32_t)__popcll(bal[j] & lanemask_lt(lane));
        sparse[base + d] = make_float4(x[j], y[j], z[j], 1.0f);
        if (sparse_idx) sparse_idx[base + d] = (uint32_t)(base + (uint64_t)j * kFT + threadIdx.x);
        mn[0] = fminf(mn[0], x[j]); mx[0] = fmaxf(mx[0], x[j]);
        mn[1] = fminf(mn[1], y[j]); mx[1] = fmaxf(mx[1], y[j]);
        mn[2] = fminf(mn[2], z[j]); mx[2] = fmaxf(mx[2], z[j]);
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

// points that go through the sort: all cropped points when voxelising without overflow
__device__ __forceinline__ uint32_t sort_count(const VoxParams &vp) {
    return (vp.do_voxel && !vp.overflow) ? vp.m : 0u;
}
__device__ __forceinline__ uint32_t sort_tiles(const VoxParams &vp) {
    return (sort_count(vp) + kSortTile - 1) / kSortTile;
}

// cropped count + bbox -> parameters; the result count of a crop-only / passthrough cloud
// (res[slot] = m; a voxelised cloud's count is written by k_seg_centroid)
__global__ void __launch_bounds__(kFT)
k_vox_params(const float *__restrict__ part, const uint32_t *__restrict__ counts, int nb,
             float leaf, VoxParams *__restrict__ vp, uint32_t *__restrict__ res,
             uint32_t *__restrict__ info, int slot) {
    __shared__ uint32_t lds4[kFT / 64];
    const uint32_t m = block_prefix_sum<kFT>(counts, (uint32_t)nb, lds4);
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
    p.m = m;
    p.do_voxel = leaf > 0.0f ? 1 : 0;
    const float inv = p.do_voxel ? 1.0f / leaf : 0.0f;
    p.inv = inv;
    if (p.m != 0 && p.do_voxel) {
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
    }
    *vp = p;
    const bool vox = p.do_voxel && !p.overflow;
    res[slot] = vox ? 0u : m;
    info[2 * slot] = m;          // points after the crop
    info[2 * slot + 1] = p.overflow;
}

// ---- gaps closed: tile t's kept points go to [sum of earlier counts ...); voxel keys -------
__global__ void __launch_bounds__(kFT)
k_compact_keys(const float4 *__restrict__ sparse, const uint32_t *__restrict__ sparse_idx,
               const uint32_t *__restrict__ counts, const VoxParams *__restrict__ vpp,
               float4 *__restrict__ xyz, uint32_t *__restrict__ kept_idx,
               uint32_t *__restrict__ keys, uint32_t *__restrict__ zero, uint32_t nzero) {
    // digit totals + group sums of every radix pass (accumulated by k_radix_hist) start at 0
    for (uint32_t q = blockIdx.x * kFT + threadIdx.x; q < nzero; q += gridDim.x * kFT) zero[q] = 0;
    const uint32_t cnt = counts[blockIdx.x];
    if (cnt == 0) return;   // uniform per block
    __shared__ uint32_t lds4[kFT / 64];
    const uint32_t pre = block_prefix_sum<kFT>(counts, blockIdx.x, lds4);
    const VoxParams vp = *vpp;
    const bool sort = sort_count(vp) != 0;
    const uint64_t sb = (uint64_t)blockIdx.x * kCropTile;
    for (uint32_t j = threadIdx.x; j < cnt; j += kFT) {
        const float4 p = sparse[sb + j];
        xyz[pre + j] = p;
        if (kept_idx) kept_idx[pre + j] = sparse_idx[sb + j];
        if (sort) {
            const int ijk0 = (int)(floorf(p.x * vp.inv) - (float)vp.min_b[0]);
            const int ijk1 = (int)(floorf(p.y * vp.inv) - (float)vp.min_b[1]);
            const int ijk2 = (int)(floorf(p.z * vp.inv) - (float)vp.min_b[2]);
            keys[pre + j] = (uint32_t)ijk0 + (uint32_t)ijk1 * vp.mul1 + (uint32_t)ijk2 * vp.mul2;
        }
    }
}

// ---- LSD radix sort (stable), 9-bit digits, (key, float4 point) pairs ----------------------
// Sort tiles of 4096 items, 512-thread blocks, tile-strided grids (<= one block per CU).
// hist[d * ntp + t] = count of digit d in tile t; totals[d] and the group sums
// gsum[(t / kGroup) * kBins + d] accumulate the tiles' counts (one 256-B atomic row per wave),
// so a tile's count of earlier items of digit d needs <= ngroups + 4 independent loads.
__global__ void __launch_bounds__(kST)
k_radix_hist(const uint32_t *__restrict__ keys, const VoxParams *__restrict__ vpp, int shift,
             uint32_t ntp, uint32_t *__restrict__ hist, uint32_t *__restrict__ totals,
             uint32_t *__restrict__ gsum) {
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    const uint32_t nact = sort_tiles(vp);
    __shared__ uint32_t h[kBins];
    static_assert(kBins == kST, "one digit per thread");
    const uint32_t d = threadIdx.x;
    for (uint32_t t = blockIdx.x; t < nact; t += gridDim.x) {
        h[d] = 0;
        __syncthreads();
        const uint64_t base = (uint64_t)t * kSortTile;
        uint32_t k[kSortItems];
#pragma unroll
        for (int j = 0; j < kSortItems; ++j) {
            const uint64_t i = base + (uint64_t)j * kST + threadIdx.x;
            k[j] = i < m ? keys[i] : 0u;
        }
#pragma unroll
        for (int j = 0; j < kSortItems; ++j)
            if (base + (uint64_t)j * kST + threadIdx.x < m)
                atomicAdd(&h[(k[j] >> shift) & (kBins - 1)], 1u);
        __syncthreads();
        const uint32_t v = h[d];
        hist[(size_t)d * ntp + t] = v;
        if (v) {
            atomicAdd(&totals[d], v);
            atomicAdd(&gsum[(size_t)(t / kGroup) * kBins + d], v);
        }
        __syncthreads();
    }
}

// stable scatter of sort tile t: items of wave w are [w*512, (w+1)*512) of the tile, round j
// covers 64 of them; rank = earlier same-digit items of the wave (running per-wave counters in
// LDS + match-any of the round) + earlier waves of the tile.  The tile is then laid out in LDS
// in digit order and written out run by run (each digit's items are contiguous in the output),
// so the global stores are coalesced instead of one cache line per item.
__global__ void __launch_bounds__(kST)
k_radix_scatter(const uint32_t *__restrict__ kin, const float4 *__restrict__ pin,
                const VoxParams *__restrict__ vpp, int shift, uint32_t ntp,
                const uint32_t *__restrict__ hist, const uint32_t *__restrict__ totals,
                const uint32_t *__restrict__ gsum, uint32_t *__restrict__ kout,
                float4 *__restrict__ pout) {
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    const uint32_t nact = sort_tiles(vp);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int kWaveItems = kSortTile / kSW;
    __shared__ uint32_t wh[kSW][kBins];
    __shared__ uint32_t g[kBins];     // output position of the tile's first item of digit d
    __shared__ uint32_t tx[kBins];    // tile-local exclusive digit offsets
    __shared__ uint32_t lsa[kSW], lsb[kSW];
    __shared__ uint32_t lk[kSortTile];
    __shared__ float4 lp[kSortTile];
    const uint32_t d = threadIdx.x;   // this thread's digit in the offset phase
    for (uint32_t t = blockIdx.x; t < nact; t += gridDim.x) {
    const uint64_t tbase = (uint64_t)t * kSortTile;
    FLT_STAMP(0, t, 0);
    const uint64_t wbase = tbase + (uint64_t)wid * kWaveItems;
    const uint32_t tn = (uint32_t)min<uint64_t>(kSortTile, m - tbase);   // items in this tile
#pragma unroll
    for (int w = 0; w < kSW; ++w) wh[w][d] = 0;
    uint32_t k[kSortItems];
    float4 pv[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const uint64_t i = wbase + (uint64_t)j * 64 + lane;
        k[j] = i < m ? kin[i] : 0u;
        pv[j] = i < m ? pin[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // earlier tiles' count of digit d: whole groups, then the tiles of t's own group
    const uint32_t grp = t / kGroup;
    uint32_t pre = 0;
#pragma unroll 8
    for (uint32_t q = 0; q < grp; ++q) pre += gsum[(size_t)q * kBins + d];
    {
        const uint4 *row = reinterpret_cast<const uint4 *>(hist + (size_t)d * ntp + grp * kGroup);
        const uint32_t nin = t - grp * kGroup;   // 0 .. kGroup-1
#pragma unroll
        for (uint32_t qq = 0; qq < kGroup / 4; ++qq) {
            if (4 * qq < nin) {
                const uint4 v = row[qq];
                const uint32_t b = 4 * qq;
                pre += v.x + (b + 1 < nin ? v.y : 0u) + (b + 2 < nin ? v.z : 0u) +
                       (b + 3 < nin ? v.w : 0u);
            }
        }
    }
    const uint32_t tot_d = totals[d];
    __syncthreads();
    FLT_STAMP(0, t, 1);
    uint32_t r[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const bool act = wbase + (uint64_t)j * 64 + lane < m;
        const uint32_t dj = (k[j] >> shift) & (kBins - 1);
        uint64_t same = __ballot(act);
#pragma unroll
        for (int bit = 0; bit < kDigitBits; ++bit) {
            const uint64_t bb = __ballot((dj >> bit) & 1u);
            same &= ((dj >> bit) & 1u) ? bb : ~bb;
        }
        const uint32_t lower = (uint32_t)__popcll(same & lanemask_lt(lane));
        r[j] = act ? wh[wid][dj] + lower : 0u;
        if (act && lower == 0) wh[wid][dj] += (uint32_t)__popcll(same);
    }
    __syncthreads();
    FLT_STAMP(0, t, 2);
    // digit d: per-wave exclusive offsets and the tile's count
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < kSW; ++w) {
        const uint32_t v = wh[w][d];
        wh[w][d] = cnt;
        cnt += v;
    }
    // exclusive scans over the digits: global totals (-> digit base), tile counts (-> LDS layout)
    const uint32_t base_d = block_excl_scan<kST>(tot_d, lsa);
    const uint32_t tx_d = block_excl_scan<kST>(cnt, lsb);
    g[d] = base_d + pre;
    tx[d] = tx_d;
    __syncthreads();
    FLT_STAMP(0, t, 3);
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        if (wbase + (uint64_t)j * 64 + lane < m) {
            const uint32_t dj = (k[j] >> shift) & (kBins - 1);
            const uint32_t lpos = tx[dj] + wh[wid][dj] + r[j];
            lk[lpos] = k[j];
            lp[lpos] = pv[j];
        }
    }
    __syncthreads();
    FLT_STAMP(0, t, 4);
#pragma unroll 4
    for (uint32_t q = threadIdx.x; q < tn; q += kST) {
        const uint32_t kk = lk[q];
        const uint32_t dq = (kk >> shift) & (kBins - 1);
        const uint32_t dst = g[dq] + (q - tx[dq]);
        kout[dst] = kk;
        pout[dst] = lp[q];
    }
    __syncthreads();
    FLT_STAMP(0, t, 5);
    }
}

// ---- segments (voxels) of the sorted keys and their centroids ------------------------------
// a sorted position starts a voxel iff its key differs from the previous one
__device__ __forceinline__ bool seg_head(const uint32_t *keys, uint64_t i, uint32_t m) {
    return i < m && (i == 0 || keys[i] != keys[i - 1]);
}

// heads per sort tile and the tile's first head position (UINT32_MAX: none)
__global__ void __launch_bounds__(kST)
k_seg_count(const uint32_t *__restrict__ keys, const VoxParams *__restrict__ vpp,
            uint32_t *__restrict__ tcount, uint32_t *__restrict__ fhead) {
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    const uint32_t nact = sort_tiles(vp);
    __shared__ uint32_t w[kSW], f[kSW];
    for (uint32_t t = blockIdx.x; t < nact; t += gridDim.x) {
        const uint64_t base = (uint64_t)t * kSortTile;
        uint32_t c = 0, first = UINT32_MAX;
#pragma unroll
        for (int j = 0; j < kSortItems; ++j) {
            const uint64_t i = base + (uint64_t)j * kST + threadIdx.x;
            if (seg_head(keys, i, m)) {
                ++c;
                first = min(first, (uint32_t)i);
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            c += __shfl_xor(c, o, 64);
            first = min(first, (uint32_t)__shfl_xor((int)first, o, 64));
        }
        if ((threadIdx.x & 63) == 0) {
            w[threadIdx.x >> 6] = c;
            f[threadIdx.x >> 6] = first;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t cs = 0, fs = UINT32_MAX;
            for (int q = 0; q < kSW; ++q) {
                cs += w[q];
                fs = min(fs, f[q]);
            }
            tcount[t] = cs;
            fhead[t] = fs;
        }
        __syncthreads();
    }
}

// voxel s = the s-th head in sorted order: CentroidPoint<PointXYZ> = float sums of its points
// in (stable) input order, / (float)n.  The tile's sorted points are staged in LDS; run ends
// come from the tile's head list and the next tile holding a head.  The last tile writes the
// voxel count (res[slot]).
__global__ void __launch_bounds__(kST)
k_seg_centroid(const uint32_t *__restrict__ keys, const float4 *__restrict__ pay,
               const VoxParams *__restrict__ vpp, const uint32_t *__restrict__ tcount,
               const uint32_t *__restrict__ fhead, float4 *__restrict__ out,
               uint32_t *__restrict__ out_idx, uint32_t *__restrict__ out_cnt,
               uint32_t *__restrict__ res, int slot) {
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    const uint32_t nact = sort_tiles(vp);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t lds[kSW];
    __shared__ uint32_t hpos[kSortTile + 1];
    __shared__ float4 lp[kSortTile];   // the tile's sorted points
    __shared__ uint32_t wo[kSortItems][kSW];
    for (uint32_t t = blockIdx.x; t < nact; t += gridDim.x) {
    const uint64_t base = (uint64_t)t * kSortTile;
    FLT_STAMP(1, t, 0);
    uint64_t bal[kSortItems];
    uint32_t head = 0, hkey[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const uint64_t i = base + (uint64_t)j * kST + threadIdx.x;
        lp[j * kST + threadIdx.x] = i < m ? pay[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        const uint32_t kc = i < m ? keys[i] : 0u;
        const uint32_t kp = (i < m && i > 0) ? keys[i - 1] : 0u;
        const bool h = i < m && (i == 0 || kc != kp);
        hkey[j] = kc;
        head |= (h ? 1u : 0u) << j;
        bal[j] = __ballot(h);
    }
    const uint32_t pre = block_prefix_sum<kST>(tcount, t, lds);
    FLT_STAMP(1, t, 1);
    const uint32_t tot = round_offsets(bal, wo);
    FLT_STAMP(1, t, 2);
    if (t == nact - 1 && threadIdx.x == 0) res[slot] = pre + tot;
    if (tot != 0) {   // uniform; 0: a tile inside one long voxel
    uint32_t loc[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        loc[j] = wo[j][wid] + (uint32_t)__popcll(bal[j] & lanemask_lt(lane));
        if ((head >> j) & 1u) hpos[loc[j]] = (uint32_t)(base + (uint64_t)j * kST + threadIdx.x);
    }
    if (threadIdx.x == 0) {   // end of the tile's last run: the next head after this tile
        uint32_t e = m;
        for (uint32_t u = t + 1; u < nact; ++u) {
            const uint32_t fh = fhead[u];
            if (fh != UINT32_MAX) {
                e = fh;
                break;
            }
        }
        hpos[tot] = e;
    }
    __syncthreads();
    FLT_STAMP(1, t, 3);
    // run sums, point index outer / head inner: the sum of each voxel still runs in input order,
    // while the loads of one step (LDS, or global past the tile) are independent of each other
    uint32_t a_[kSortItems], n_[kSortItems], nmax = 0;
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const bool h = (head >> j) & 1u;
        a_[j] = h ? hpos[loc[j]] : 0u;
        n_[j] = h ? hpos[loc[j] + 1] - a_[j] : 0u;
        nmax = max(nmax, n_[j]);
    }
    float sx[kSortItems], sy[kSortItems], sz[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) sx[j] = sy[j] = sz[j] = 0.f;
    const uint64_t tend = base + kSortTile;
    FLT_STAMP(1, t, 4);
    for (uint32_t q = 0; q < nmax; ++q) {
#pragma unroll
        for (int j = 0; j < kSortItems; ++j) {
            if (q < n_[j]) {
                const uint32_t l = a_[j] + q;
                const float4 p = l < tend ? lp[l - base] : pay[l];
                sx[j] = sx[j] + p.x;
                sy[j] = sy[j] + p.y;
                sz[j] = sz[j] + p.z;
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        if (!((head >> j) & 1u)) continue;
        const float cnt = (float)n_[j];
        const uint32_t s = pre + loc[j];
        out[s] = make_float4(sx[j] / cnt, sy[j] / cnt, sz[j] / cnt, 1.0f);
        out_idx[s] = hkey[j];
        out_cnt[s] = n_[j];
    }
    }   // tot != 0
    __syncthreads();
    FLT_STAMP(1, t, 5);
    }
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
    uint32_t nt = 0;          // sort tiles (upper bound)
    uint32_t ntp = 0;         // radix histogram row stride (nt rounded up to 16)
    uint32_t ngp = 0;         // prefix groups of kGroup sort tiles
    uint32_t *counts = nullptr;                    // crop tile kept counts
    float *part = nullptr;                         // crop bbox partials
    uint32_t *totals = nullptr;                    // [kMaxPasses][kBins] digit totals, then
                                                   // [kMaxPasses][ngp][kBins] group sums
    uint32_t nzero = 0;                            // words of totals + group sums
    uint32_t *rhist = nullptr;                     // [kBins][ntp] tile digit counts
    uint32_t *tcount = nullptr;                    // voxel heads per sort tile
    uint32_t *fhead = nullptr;                     // first head position per sort tile
    VoxParams *vp = nullptr;  // [kMaxClouds]
    uint32_t *res = nullptr;  // [kMaxClouds] result counts, [2*kMaxClouds] info
    float4 *xyz() const { return B->xyz.as<float4>(); }        // compact cropped points
    float4 *sparse() const { return B->sparse.as<float4>(); }  // crop tiles / sort ping-pong
    float4 *out4() const { return B->out.as<float4>(); }
    uint32_t *vidx() const { return reinterpret_cast<uint32_t *>(out4() + ncap + 1); }
    uint32_t *vcnt() const { return vidx() + ncap + 1; }
};

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// (callers holding Scratch objects of several slots must size ctx->fbuf beforehand)
static int ensure_scratch(pcp_ctx *ctx, int slot, uint64_t ncap, bool want_idx, Scratch &S) {
    if (ncap >= (1ull << 31))
        return set_err(ctx, PCP_E_INVALID, "cloud of %llu points: at most 2^31-1 per call",
                       (unsigned long long)ncap);
    if ((int)ctx->fbuf.size() <= slot) ctx->fbuf.resize(slot + 1);
    CloudBufs &B = ctx->fbuf[slot];
    S.B = &B;
    ncap = ncap ? ncap : 1;
    S.ncap = ncap;
    S.nb = (uint32_t)((ncap + kCropTile - 1) / kCropTile);
    S.nt = (uint32_t)((ncap + kSortTile - 1) / kSortTile);
    S.ntp = (S.nt + 15) & ~15u;
    S.ngp = (S.nt + kGroup - 1) / kGroup;
    // sparse crop tiles are whole tiles: nb * kCropTile points
    PCP_HIP(ctx, B.xyz.ensure((ncap + 1) * sizeof(float4)));
    PCP_HIP(ctx, B.sparse.ensure((size_t)S.nb * kCropTile * sizeof(float4)));
    if (want_idx) {
        PCP_HIP(ctx, B.idx.ensure((ncap + 1) * sizeof(uint32_t)));
        PCP_HIP(ctx, B.sparse_idx.ensure((size_t)S.nb * kCropTile * sizeof(uint32_t)));
    }
    for (int q = 0; q < 2; ++q) PCP_HIP(ctx, B.keys[q].ensure((ncap + 16) * sizeof(uint32_t)));
    const size_t cb = align256((size_t)(S.nb + 4) * 4), pb = align256((size_t)S.nb * 24);
    S.nzero = (uint32_t)((size_t)kMaxPasses * kBins * (1 + S.ngp));
    const size_t tb = align256((size_t)S.nzero * 4);
    const size_t hb = align256((size_t)kBins * S.ntp * 4), sb = align256((size_t)(S.ntp + 4) * 4);
    PCP_HIP(ctx, B.hist.ensure(cb + pb + tb + hb + 2 * sb));
    char *h = B.hist.as<char>();
    S.counts = reinterpret_cast<uint32_t *>(h);
    S.part = reinterpret_cast<float *>(h + cb);
    S.totals = reinterpret_cast<uint32_t *>(h + cb + pb);
    S.rhist = reinterpret_cast<uint32_t *>(h + cb + pb + tb);
    S.tcount = reinterpret_cast<uint32_t *>(h + cb + pb + tb + hb);
    S.fhead = reinterpret_cast<uint32_t *>(h + cb + pb + tb + hb + sb);
    // voxel results: out4 (ncap+1) | idx (ncap+1) | cnt (ncap+1)
    PCP_HIP(ctx, B.out.ensure((ncap + 1) * sizeof(float4) + (2 * ncap + 8) * 4 + 256));
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
    int bits = 32;
    bool finite = true;
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) finite = false;
        else nv *= std::floor((hi[a] - lo[a]) / (double)leaf) + 3.0;
    }
    if (finite) {
        bits = 0;
        while (bits < 32 && std::ldexp(1.0, bits) < nv) ++bits;
    }
    return std::max(1, (bits + kDigitBits - 1) / kDigitBits);
}

// enqueue crop [-> voxel] for one cloud into slot `slot` on stream `st` (results stay on the
// device: S.res[slot] = result count)
static int enqueue_cloud(pcp_ctx *ctx, Scratch &S, const CloudIn &c, const Box &b, float leaf,
                         bool want_idx, int slot, hipStream_t st) {
    const uint32_t nb = (uint32_t)((c.n + kCropTile - 1) / kCropTile);
    CloudBufs &B = *S.B;
    VoxParams *vp = S.vp + slot;
    {
        ProfScope ps(ctx, PCP_K_CROP, st);
        if (nb) {
            hipLaunchKernelGGL(k_crop_tile, dim3(nb), dim3(kFT), 0, st, c, b, S.counts, S.part,
                               S.sparse(), want_idx ? B.sparse_idx.as<uint32_t>() : nullptr);
            PCP_CHECK_LAUNCH(ctx);
        }
        hipLaunchKernelGGL(k_vox_params, dim3(1), dim3(kFT), 0, st, (const float *)S.part,
                           (const uint32_t *)S.counts, (int)nb, leaf, vp, S.res,
                           S.res + kMaxClouds, slot);
        PCP_CHECK_LAUNCH(ctx);
        if (nb) {
            hipLaunchKernelGGL(k_compact_keys, dim3(nb), dim3(kFT), 0, st,
                               (const float4 *)S.sparse(),
                               want_idx ? B.sparse_idx.as<const uint32_t>() : nullptr,
                               (const uint32_t *)S.counts, (const VoxParams *)vp, S.xyz(),
                               want_idx ? B.idx.as<uint32_t>() : nullptr, B.keys[0].as<uint32_t>(),
                               S.totals, S.nzero);
            PCP_CHECK_LAUNCH(ctx);
        }
    }
    if (!(leaf > 0.0f) || c.n == 0) return PCP_OK;
    ProfScope ps(ctx, PCP_K_VOXEL, st);
    const uint32_t nt = (uint32_t)((c.n + kSortTile - 1) / kSortTile);
    const int passes = radix_passes(b, leaf);
    const uint32_t ntg = std::min<uint32_t>(nt, (uint32_t)std::max(ctx->num_cus, 1));
    // payload ping-pong: the compact points, then the (dead) sparse crop buffer
    float4 *pay[2] = {S.xyz(), S.sparse()};
    int cur = 0;
    for (int pass = 0; pass < passes; ++pass) {
        const int shift = kDigitBits * pass;
        uint32_t *tot = S.totals + pass * kBins;
        uint32_t *gs = S.totals + (size_t)kMaxPasses * kBins + (size_t)pass * S.ngp * kBins;
        hipLaunchKernelGGL(k_radix_hist, dim3(ntg), dim3(kST), 0, st,
                           B.keys[cur].as<const uint32_t>(), (const VoxParams *)vp, shift, S.ntp,
                           S.rhist, tot, gs);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_radix_scatter, dim3(ntg), dim3(kST), 0, st,
                           B.keys[cur].as<const uint32_t>(), (const float4 *)pay[cur],
                           (const VoxParams *)vp, shift, S.ntp, (const uint32_t *)S.rhist,
                           (const uint32_t *)tot, (const uint32_t *)gs,
                           B.keys[cur ^ 1].as<uint32_t>(), pay[cur ^ 1]);
        PCP_CHECK_LAUNCH(ctx);
        cur ^= 1;
    }
    const uint32_t *keys = B.keys[cur].as<const uint32_t>();
    hipLaunchKernelGGL(k_seg_count, dim3(ntg), dim3(kST), 0, st, keys, (const VoxParams *)vp,
                       S.tcount, S.fhead);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_seg_centroid, dim3(ntg), dim3(kST), 0, st, keys, (const float4 *)pay[cur],
                       (const VoxParams *)vp, (const uint32_t *)S.tcount, (const uint32_t *)S.fhead,
                       S.out4(), S.vidx(), S.vcnt(), S.res, slot);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

static int enqueue_emit(pcp_ctx *ctx, Scratch &S, uint64_t ncap, int slot, const Rigid &r,
                        float4 *out, hipStream_t st) {
    if (ncap == 0) return PCP_OK;
    ProfScope ps(ctx, PCP_K_TRANSFORM, st);
    const unsigned g = (unsigned)std::min<uint64_t>((ncap + kFT - 1) / kFT, 4096);
    hipLaunchKernelGGL(k_emit_rgb, dim3(g), dim3(kFT), 0, st, (const float4 *)S.xyz(),
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
        PCP_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ctx->emit_ev.push_back(e);
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
        if (dev_out && upper > cap) {   // sizes checked on the host afterwards
            for (int i = 0; i < k; ++i) PCP_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->side_ev[i], 0));
            return PCP_OK;
        }
        // cloud i's emit needs the counts of clouds 0..i-1 (its offset in the concatenation):
        // it runs on branch i once those chains are done, so emit 0 overlaps the later chains
        for (int i = 0; i < k; ++i) {
            hipStream_t si = ctx->side[i];
            for (int j = 0; j < i; ++j) PCP_HIP(ctx, hipStreamWaitEvent(si, ctx->side_ev[j], 0));
            int r = enqueue_emit(ctx, S[i], clouds[i].n, i, make_rigid(tf[i], rgb + 3 * i), obuf, si);
            if (r) return r;
            PCP_HIP(ctx, hipEventRecord(ctx->emit_ev[i], si));
        }
        for (int i = 0; i < k; ++i) PCP_HIP(ctx, hipStreamWaitEvent(ctx->stream, ctx->emit_ev[i], 0));
        return PCP_OK;
    };
    int rc = PCP_OK;
    const bool graphable = dev_in && dev_out && upper <= cap && ctx->use_graphs;
    if (graphable) {
        std::vector<uint8_t> key = fm_key(k, clouds, boxes, leaf, tf, rgb, out, cap);
        std::vector<const void *> sp;
        for (int i = 0; i < k; ++i) {
            const CloudBufs &B = ctx->fbuf[i];
            const void *v[] = {B.xyz.p, B.keys[0].p, B.keys[1].p, B.sparse.p, B.sparse_idx.p,
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
            rc = enqueue_emit(ctx, S[i], clouds[i].n, i, make_rigid(tf[i], rgb + 3 * i), obuf,
                              ctx->stream);
            if (rc) return rc;
        }
    }
    if (!dev_out && total)
        PCP_HIP(ctx, hipMemcpyAsync(out, obuf, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

#ifdef PCP_STAMPS
// diagnostic build only: the stamps of the last k_radix_scatter / k_seg_centroid launches
int pcp_diag_filter_stamps(pcp_ctx *ctx, int which, unsigned long long *out, size_t n) {
    PCP_HIP(ctx, hipDeviceSynchronize());
    n = std::min<size_t>(n, (size_t)kStampTiles * kStampPh);
    PCP_HIP(ctx, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_flt_stamps), n * 8,
                                     (size_t)(which ? 1 : 0) * kStampTiles * kStampPh * 8,
                                     hipMemcpyDeviceToHost));
    return PCP_OK;
}
#endif

}  // extern "C"
