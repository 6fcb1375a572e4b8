// pcp_filter.hip -- pointcloud_filter.cpp (crop + VoxelGrid) and pointcloud_merger.cpp
// (tf2::doTransform + colour + concat) on gfx950.
//
// Every kernel is batched over clouds: blockIdx.y = cloud, its job (input view, box, leaf,
// scratch, transform) read from a device table, so a dual-LiDAR frame is one chain of ~12
// launches in which every launch covers all clouds' tiles.
//  crop    : one read of the input; stable compaction per 4096-point tile into a sparse buffer,
//            gaps closed (and voxel keys computed) by a second, small kernel
//  voxel   : PCL VoxelGrid<PointXYZ> keying in float exactly as applyFilter; stable LSD radix
//            sort of (key, point) with 9-bit digits (LDS-staged, coalesced scatter); voxel
//            heads + float centroids summed in input order
//  merge   : Eigen float Affine3f * p = ((m0 x + m1 y) + m2 z) + t, PointXYZRGB records
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "pcp_internal.hpp"
#include "pcp_rigid.hpp"

namespace pcp {

constexpr int kFT = 256;            // threads per block
#ifndef PCP_CROP_THREADS
#define PCP_CROP_THREADS 256
#endif
constexpr int kCT = PCP_CROP_THREADS;   // threads of a crop block (build knob)
#ifndef PCP_CROP_TILE
#define PCP_CROP_TILE 4096
#endif
constexpr int kCropTile = PCP_CROP_TILE;   // points per crop tile (build knob)
constexpr int kCropItems = kCropTile / kCT;   // points per thread per crop tile
constexpr int kST = 512;            // threads of the sort-tile kernels (8 waves)
constexpr int kSW = kST / 64;
#ifndef PCP_SORT_ITEMS
#define PCP_SORT_ITEMS 8
#endif
constexpr int kSortItems = PCP_SORT_ITEMS;   // keys per thread per sort tile
constexpr int kSortTile = kST * kSortItems;
constexpr int kGroup = 16;          // sort tiles per prefix group (radix digit prefix sums)
constexpr int kDigitBits = 9;       // radix digit: 512 bins, 3 passes for the C3 crop box
constexpr int kBins = 1 << kDigitBits;
constexpr int kMaxPasses = 4;       // ceil(32 / 9)
constexpr int kMaxCloudsDev = 64;   // result slots of a call (= kMaxClouds below)

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

// a crop tile's points: item j of thread t is base + j*kCT + t (coalesced); indices past the
// end are clamped to the last point (the caller masks them)
template <bool PXYZ16>
__device__ __forceinline__ void load_tile(const CloudIn &c, uint64_t base, float (&x)[kCropItems],
                                          float (&y)[kCropItems], float (&z)[kCropItems]) {
    const uint64_t last = c.n - 1;
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        const uint64_t i = min(base + (uint64_t)j * kCT + threadIdx.x, last);
        if constexpr (PXYZ16) {
            const float4 v = reinterpret_cast<const float4 *>(c.raw)[i];
            x[j] = v.x;
            y[j] = v.y;
            z[j] = v.z;
        } else {
            const unsigned char *p = c.raw + i * c.step;
            x[j] = *reinterpret_cast<const float *>(p + c.ox);
            y[j] = *reinterpret_cast<const float *>(p + c.oy);
            z[j] = *reinterpret_cast<const float *>(p + c.oz);
        }
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

// wave64 inclusive scan by DPP (row_shr 1, 2, 4, 8 inside each 16-lane row, then row_bcast 15
// / 31 across rows): VALU moves, no LDS-crossbar (ds_bpermute) round trips as __shfl_up takes
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
__device__ __forceinline__ uint32_t wave_sum_dpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(x), 63);
}
// wave min / max of floats by the same DPP pattern (identity in the lanes without a source)
template <bool MAX>
__device__ __forceinline__ float wave_minmax_dpp(float x) {
    const int id = __float_as_int(MAX ? -FLT_MAX : FLT_MAX);
#define PCP_MM_STEP(ctrl, rm)                                                                    \
    {                                                                                            \
        const float y = __int_as_float(__builtin_amdgcn_update_dpp(id, __float_as_int(x), ctrl, \
                                                                   rm, 0xF, false));            \
        x = MAX ? fmaxf(x, y) : fminf(x, y);                                                     \
    }
    PCP_MM_STEP(0x111, 0xF) PCP_MM_STEP(0x112, 0xF) PCP_MM_STEP(0x114, 0xF)
    PCP_MM_STEP(0x118, 0xF) PCP_MM_STEP(0x142, 0xA) PCP_MM_STEP(0x143, 0xC)
#undef PCP_MM_STEP
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
// exclusive block scan (thread order) with DPP wave scans; every thread gets its prefix
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_dpp(uint32_t v, uint32_t *lds) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t incl = wave_incl_scan_dpp(v);
    if (lane == 63) lds[wid] = incl;
    __syncthreads();
    uint32_t ex = incl - v;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) ex += w < wid ? lds[w] : 0u;
    return ex;
}

// sum of one value per thread over the block; every thread gets it (lds: NT / 64 words)
template <int NT>
__device__ __forceinline__ uint32_t block_prefix_sum_reg(uint32_t s, uint32_t *lds) {
    s = wave_sum_dpp(s);
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
    // one wave scans the J x W counts, R consecutive (round, wave) entries per lane
    constexpr int E = J * W, R = (E + 63) / 64;
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < J; ++j) wo[j][wid] = (uint32_t)__popcll(bal[j]);
    __syncthreads();
    __shared__ uint32_t tot;
    if (threadIdx.x < 64) {
        uint32_t v[R], s = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = lane * R + r;
            v[r] = e < E ? wo[e / W][e % W] : 0u;
            s += v[r];
        }
        const uint32_t incl = wave_incl_scan_dpp(s);
        uint32_t ex = incl - s;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int e = lane * R + r;
            if (e < E) wo[e / W][e % W] = ex;
            ex += v[r];
        }
        if (lane == 63) tot = incl;
    }
    __syncthreads();
    return tot;
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
    uint32_t bs, nbk;    // the bucket chain: key bits below the bucket, buckets (0: none)
};

// applyFilter's parameters from the cropped count and bbox (float, as PCL computes them)
__device__ __forceinline__ VoxParams vox_params_from(uint32_t m, const float (&mn)[3],
                                                     const float (&mx)[3], float leaf) {
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
    return p;
}

// PCL's voxel index of a point (applyFilter: ijk in float relative to min_b, then idx)
__device__ __forceinline__ uint32_t vox_key(const VoxParams &vp, float x, float y, float z) {
    const int ijk0 = (int)(floorf(x * vp.inv) - (float)vp.min_b[0]);
    const int ijk1 = (int)(floorf(y * vp.inv) - (float)vp.min_b[1]);
    const int ijk2 = (int)(floorf(z * vp.inv) - (float)vp.min_b[2]);
    return (uint32_t)ijk0 + (uint32_t)ijk1 * vp.mul1 + (uint32_t)ijk2 * vp.mul2;
}

// points that go through the sort: all cropped points when voxelising without overflow
__device__ __forceinline__ uint32_t sort_count(const VoxParams &vp) {
    return (vp.do_voxel && !vp.overflow) ? vp.m : 0u;
}
__device__ __forceinline__ uint32_t sort_tiles(const VoxParams &vp) {
    return (sort_count(vp) + kSortTile - 1) / kSortTile;
}

// one cloud's job in a batched launch (blockIdx.y indexes the device table of these)
struct CloudJob {
    CloudIn in;           // input view (raw may be null when n == 0)
    Box box;
    float leaf;           // <= 0: crop only
    int32_t passes;       // radix passes (0: no voxel stage)
    uint32_t nb;          // crop tiles, ceil(n / kCropTile)
    uint32_t ntp, ngp, nzero;
    uint32_t *counts;     // [nb] kept points per crop tile
    float *part;          // [nb][6] bbox partials
    float4 *sparse;       // crop tiles, later the odd radix passes' payload
    uint32_t *sparse_idx; // crop tiles' input indices (null unless kept indices wanted)
    float4 *xyz;          // compact cropped points, the even passes' payload
    uint32_t *kept_idx;   // compact kept indices (null unless wanted)
    uint32_t *keys0, *keys1;
    uint32_t *zero;       // digit totals [kMaxPasses][kBins] then group sums [kMaxPasses][ngp][kBins]
    uint32_t *rhist;      // [kBins][ntp] tile digit counts (reused by every pass)
    uint32_t *tcount, *fhead;
    float4 *out4;         // voxel centroids
    uint32_t *vidx, *vcnt;
    VoxParams *vp;
    Rigid rig;            // pcp_filter_merge's transform + colour of this cloud
    int32_t slot;         // result slot (index of the cloud in the call)
    // the fast chain (pcp_filter_merge when every cloud certainly voxelises, enqueue_fast):
    // the crop forms BOX-relative voxel keys -- (floor(p * inv) - kb) per axis, mixed radix
    // kdx, kdxy -- whose order is PCL's idx order (a constant shift per axis does not change
    // the lexicographic (k, j, i) order), plus each crop tile's digit-0 counts; the first radix
    // pass then reads the crop tiles in groups of gt, no compaction, no parameters
    int32_t fast;
    float kinv, kb[3];
    uint32_t kdx, kdxy;
    uint32_t *skeys;      // [nb * kCropTile] keys in the crop tiles' slots
    uint32_t *h0;         // [nb][kBins] digit-0 counts per crop tile
    uint32_t ng;          // groups of gt crop tiles (pass 0's sort tiles)
    uint32_t gt;          // crop tiles per group: all groups of a batch in ONE round of blocks
    // the bucket chain (k_bk_group -> k_bk_sort -> k_bk_emit): groups of gt crop tiles sorted by
    // bucket (PCL idx >> vp.bs) into xyz, one row of bucket starts per group
    int32_t bk;
    int32_t bkpb;         // bits(input points / PCP_BK_PTS): bs >= bits(nvox) - bkpb (64: unused)
    uint32_t nbkcap;      // buckets the rows and the look-back words are sized for
    uint32_t *brows;      // [ng][nbk + 1] compact position of the group's first item of bucket b
    // pcp_filter_merge_nodes: the cloud's centroids in its own frame beside the merged records
    // (the filter node's message), written by k_bk_emit; null otherwise
    float4 *keep16;
};
constexpr int kMaxGroupTiles = 32;   // crop tiles per pass-0 sort tile, at most
constexpr int kS0Items = 10;         // pass-0 chunk: 5,120 items (a group of ~10 C3 crop tiles
constexpr int kS0Tile = kST * kS0Items;   // holds ~4,000 +- 100: one chunk)

// up to kBatch clouds per launch, passed BY VALUE: pointers loaded from kernel arguments are
// known to be global (global_load, independent waits), which a table in memory would lose
constexpr int kBatch = 8;
struct JobBatch {
    CloudJob j[kBatch];
};

// ---- crop: one read of the input; stable compaction of each tile into its own slot of a
//      sparse buffer (kept count + bbox partial per tile); k_compact_keys closes the gaps ----
// PCP_CROP_WAVES (build knob, A/B): the crop's waves-per-SIMD floor (84 VGPRs -> 5 by default)
#ifdef PCP_CROP_WAVES
#define PCP_CROP_ATTR __attribute__((amdgpu_waves_per_eu(PCP_CROP_WAVES, PCP_CROP_WAVES)))
#else
#define PCP_CROP_ATTR
#endif
template <bool KEYS>
__global__ void __launch_bounds__(kCT) PCP_CROP_ATTR k_crop_tile(const JobBatch jobs,
                                                                 uint32_t *__restrict__ res) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if constexpr (KEYS) {
        // the fast chain's zeroing (k_compact_keys does it in the other chain): digit totals
        // and group sums of every pass, the sort count (k_hist0 adds to it) and the result
        // slots (a cloud with nothing cropped keeps 0 voxels)
        for (uint32_t q = blockIdx.x * kCT + threadIdx.x; q < J.nzero; q += gridDim.x * kCT)
            J.zero[q] = 0;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            VoxParams p{};
            p.do_voxel = 1;
            p.inv = J.kinv;
            *J.vp = p;
            res[J.slot] = 0;
            res[kMaxCloudsDev + 2 * J.slot] = 0;
            res[kMaxCloudsDev + 2 * J.slot + 1] = 0;
        }
    }
    else if (J.bk && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
        res[3 * kMaxCloudsDev] = 0;   // the bucket chain's redo flag (k_bk_* set it)
    if (blockIdx.x >= J.nb) return;
    const CloudIn c = J.in;
    const Box b = J.box;
    uint32_t *counts = J.counts;
    float *part = J.part;
    float4 *sparse = J.sparse;
    uint32_t *sparse_idx = J.sparse_idx;
    const uint64_t base = (uint64_t)blockIdx.x * kCropTile;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    float x[kCropItems], y[kCropItems], z[kCropItems];
    // one uniform layout branch, then unconditional loads (indices clamped to the last point,
    // masked below): no control flow between the loads, all 16 in flight at once
    if (c.step == 16 && c.ox == 0 && c.oy == 4 && c.oz == 8)
        load_tile<true>(c, base, x, y, z);
    else
        load_tile<false>(c, base, x, y, z);
    uint64_t bal[kCropItems];
    uint32_t keep = 0;
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        const uint64_t i = base + (uint64_t)j * kCT + threadIdx.x;
        const bool k = i < c.n && in_box(b, x[j], y[j], z[j]);
        keep |= (k ? 1u : 0u) << j;
        bal[j] = __ballot(k);
    }
    __shared__ uint32_t wo[kCropItems][kCT / 64];
    __shared__ uint32_t h0s[KEYS ? kBins : 1];
    if constexpr (KEYS) {
        for (int q = threadIdx.x; q < kBins; q += kCT) h0s[q] = 0;
    }
    const uint32_t tot = round_offsets(bal, wo);   // (its barriers order the zeroing above)
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
#pragma unroll
    for (int j = 0; j < kCropItems; ++j) {
        if (!((keep >> j) & 1u)) continue;
        const uint32_t d = wo[j][wid] + (uint32_t)__popcll(bal[j] & lanemask_lt(lane));
        sparse[base + d] = make_float4(x[j], y[j], z[j], 1.0f);
        if constexpr (KEYS) {
            // applyFilter's float keying, shifted by the box floor (exact: integers < 2^24)
            const uint32_t i0 = (uint32_t)(int)(floorf(x[j] * J.kinv) - J.kb[0]);
            const uint32_t i1 = (uint32_t)(int)(floorf(y[j] * J.kinv) - J.kb[1]);
            const uint32_t i2 = (uint32_t)(int)(floorf(z[j] * J.kinv) - J.kb[2]);
            const uint32_t key = i0 + i1 * J.kdx + i2 * J.kdxy;
            J.skeys[base + d] = key;
            atomicAdd(&h0s[key & (kBins - 1)], 1u);
        } else {
            if (sparse_idx)
                sparse_idx[base + d] = (uint32_t)(base + (uint64_t)j * kCT + threadIdx.x);
            mn[0] = fminf(mn[0], x[j]); mx[0] = fmaxf(mx[0], x[j]);
            mn[1] = fminf(mn[1], y[j]); mx[1] = fmaxf(mx[1], y[j]);
            mn[2] = fminf(mn[2], z[j]); mx[2] = fmaxf(mx[2], z[j]);
        }
    }
    if constexpr (KEYS) {   // the tile's digit-0 row (the fast chain needs no bbox)
        __syncthreads();
        for (int q = threadIdx.x; q < kBins; q += kCT)
            J.h0[(size_t)blockIdx.x * kBins + q] = h0s[q];
        return;
    }
    // bbox partials (used by the voxel stage; exact min/max, order-free), DPP wave reductions
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        mn[a] = wave_minmax_dpp<false>(mn[a]);
        mx[a] = wave_minmax_dpp<true>(mx[a]);
    }
    __shared__ float s[6][kCT / 64];
    if (lane == 0)
        for (int a = 0; a < 3; ++a) {
            s[a][wid] = mn[a];
            s[3 + a][wid] = mx[a];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int a = threadIdx.x;
        float v = s[a][0];
        for (int w = 1; w < kCT / 64; ++w) v = (a < 3) ? fminf(v, s[a][w]) : fmaxf(v, s[a][w]);
        part[blockIdx.x * 6 + a] = v;
    }
}

// cropped count + bbox -> parameters; the result count of a crop-only / passthrough cloud
// (res[slot] = m; a voxelised cloud's count is written by k_seg_centroid)
__global__ void __launch_bounds__(kFT)
k_vox_params(const JobBatch jobs, uint32_t *__restrict__ res,
             uint32_t *__restrict__ info) {
    const CloudJob &J = jobs.j[blockIdx.y];
    const float *part = J.part;
    const uint32_t *counts = J.counts;
    const int nb = (int)J.nb;
    const float leaf = J.leaf;
    VoxParams *vp = J.vp;
    const int slot = J.slot;
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
    const VoxParams p = vox_params_from(m, mn, mx, leaf);
    *vp = p;
    const bool vox = p.do_voxel && !p.overflow;
    res[slot] = vox ? 0u : m;
    info[2 * slot] = m;          // points after the crop
    info[2 * slot + 1] = p.overflow;
}

// ---- gaps closed: tile t's kept points go to [sum of earlier counts ...); voxel keys -------
__global__ void __launch_bounds__(kFT) k_compact_keys(const JobBatch jobs) {
    const CloudJob &J = jobs.j[blockIdx.y];
    // digit totals + group sums of every radix pass (accumulated by k_radix_hist) start at 0
    if (J.passes > 0)
        for (uint32_t q = blockIdx.x * kFT + threadIdx.x; q < J.nzero; q += gridDim.x * kFT)
            J.zero[q] = 0;
    if (blockIdx.x >= J.nb) return;
    const float4 *sparse = J.sparse;
    const uint32_t *sparse_idx = J.sparse_idx, *counts = J.counts;
    const VoxParams *vpp = J.vp;
    float4 *xyz = J.xyz;
    uint32_t *kept_idx = J.kept_idx, *keys = J.keys0;
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
        if (sort) keys[pre + j] = vox_key(vp, p.x, p.y, p.z);
    }
}

// ---- LSD radix sort (stable), 9-bit digits, (key, float4 point) pairs ----------------------
// Sort tiles of 4096 items, 512-thread blocks, tile-strided grids (<= one block per CU).
// hist[d * ntp + t] = count of digit d in tile t; totals[d] and the group sums
// gsum[(t / kGroup) * kBins + d] accumulate the tiles' counts (one 256-B atomic row per wave),
// so a tile's count of earlier items of digit d needs <= ngroups + 4 independent loads.
__global__ void __launch_bounds__(kST) k_radix_hist(const JobBatch jobs, int pass) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if (pass >= J.passes) return;
    const uint32_t *keys = (pass & 1) ? J.keys1 : J.keys0;
    const VoxParams *vpp = J.vp;
    const int shift = kDigitBits * pass;
    const uint32_t ntp = J.ntp;
    uint32_t *hist = J.rhist;
    uint32_t *totals = J.zero + pass * kBins;
    uint32_t *gsum = J.zero + (size_t)kMaxPasses * kBins + (size_t)pass * J.ngp * kBins;
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
k_radix_scatter(const JobBatch jobs, int pass) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if (pass >= J.passes) return;
    const bool odd = pass & 1;
    const uint32_t *kin = odd ? J.keys1 : J.keys0;
    uint32_t *kout = odd ? J.keys0 : J.keys1;
    // the fast chain's pass 0 wrote its payload to xyz (it read the crop tiles in sparse)
    const bool sw = odd != (J.fast != 0);
    const float4 *pin = sw ? J.sparse : J.xyz;
    float4 *pout = sw ? J.xyz : J.sparse;
    const VoxParams *vpp = J.vp;
    const int shift = kDigitBits * pass;
    const uint32_t ntp = J.ntp;
    const uint32_t *hist = J.rhist;
    const uint32_t *totals = J.zero + pass * kBins;
    const uint32_t *gsum = J.zero + (size_t)kMaxPasses * kBins + (size_t)pass * J.ngp * kBins;
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

// ---- the fast chain's pass 0 -------------------------------------------------------------
// digit-0 counts of each group of gt crop tiles (their rows summed), the pass's
// totals and group sums, and the sort count m (k_vox_params's and k_compact_keys's jobs for the
// sort, without their passes over the points)
__global__ void __launch_bounds__(kST) k_hist0(const JobBatch jobs) {
    const CloudJob &J = jobs.j[blockIdx.y];
    const uint32_t g = blockIdx.x;
    if (!J.fast || g >= J.ng) return;
    static_assert(kBins == kST, "one digit per thread");
    const uint32_t d = threadIdx.x;
    const uint32_t c0 = g * J.gt, c1 = min(c0 + J.gt, J.nb);
    uint32_t v = 0;
    for (uint32_t c = c0; c < c1; ++c) v += J.h0[(size_t)c * kBins + d];
    J.rhist[(size_t)d * J.ntp + g] = v;
    if (v) {
        atomicAdd(&J.zero[d], v);   // pass 0's digit totals
        atomicAdd(&J.zero[(size_t)kMaxPasses * kBins + (size_t)(g / kGroup) * kBins + d], v);
    }
    if (threadIdx.x < 64) {
        uint32_t n = (c0 + threadIdx.x < c1) ? J.counts[c0 + threadIdx.x] : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) n += __shfl_xor(n, o, 64);
        if (threadIdx.x == 0 && n) atomicAdd(&J.vp->m, n);
    }
}

// pass 0 of the fast chain: sort tile g = the kept points of crop tiles [g gt, (g + 1) gt), read in
// place from their sparse slots (input order = tile order, then slot order), in chunks of up to
// kSortTile items; otherwise k_radix_scatter's stable ranking and run-wise stores, with each
// digit's running count carried from chunk to chunk
__global__ void __launch_bounds__(kST) k_radix_scatter0(const JobBatch jobs) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if (!J.fast || J.passes <= 0) return;
    const int shift = 0;
    const uint32_t ntp = J.ntp;
    const uint32_t *hist = J.rhist;
    const uint32_t *totals = J.zero;
    const uint32_t *gsum = J.zero + (size_t)kMaxPasses * kBins;
    uint32_t *kout = J.keys1;
    float4 *pout = J.xyz;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr int kWaveItems = kS0Tile / kSW;
    __shared__ uint32_t wh[kSW][kBins];
    __shared__ uint32_t gbase[kBins];   // output position of the group's first item of digit d
    __shared__ uint32_t tx[kBins];
    __shared__ uint32_t lsa[kSW], lsb[kSW];
    __shared__ uint32_t lk[kS0Tile];
    __shared__ float4 lp[kS0Tile];
    __shared__ uint32_t cpre[kMaxGroupTiles + 1];
    const uint32_t d = threadIdx.x;
    for (uint32_t g = blockIdx.x; g < J.ng; g += gridDim.x) {
        const uint32_t c0 = g * J.gt, gt = J.gt;
        if (threadIdx.x < 64) {   // the group's crop-tile counts, prefix by one wave
            const uint32_t v = (threadIdx.x < gt && c0 + threadIdx.x < J.nb) ? J.counts[c0 + threadIdx.x]
                                                                          : 0u;
            uint32_t incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t u = __shfl_up(incl, o, 64);
                if ((int)threadIdx.x >= o) incl += u;
            }
            if (threadIdx.x == 0) cpre[0] = 0;
            if (threadIdx.x < gt) cpre[threadIdx.x + 1] = incl;
        }
        // earlier groups' count of digit d: whole 16-group sets, then the groups of g's set
        const uint32_t grp = g / kGroup;
        uint32_t pre = 0;
#pragma unroll 8
        for (uint32_t q = 0; q < grp; ++q) pre += gsum[(size_t)q * kBins + d];
        {
            const uint4 *row = reinterpret_cast<const uint4 *>(hist + (size_t)d * ntp + grp * kGroup);
            const uint32_t nin = g - grp * kGroup;
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
        const uint32_t base_d = block_excl_scan<kST>(totals[d], lsa);
        gbase[d] = base_d + pre;
        __syncthreads();
        const uint32_t T = cpre[gt];
        for (uint32_t cb = 0; cb < T; cb += kS0Tile) {
            const uint32_t tn = min((uint32_t)kS0Tile, T - cb);
#pragma unroll
            for (int w = 0; w < kSW; ++w) wh[w][d] = 0;
            uint32_t k[kS0Items];
            float4 pv[kS0Items];
#pragma unroll
            for (int j = 0; j < kS0Items; ++j) {
                const uint32_t q = cb + (uint32_t)(wid * kWaveItems + j * 64 + lane);
                k[j] = 0u;
                pv[j] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (q < T) {
                    uint32_t c = 0;
                    for (uint32_t u = 1; u < gt; ++u) c += q >= cpre[u] ? 1u : 0u;
                    const size_t sp = (size_t)(c0 + c) * kCropTile + (q - cpre[c]);
                    k[j] = J.skeys[sp];
                    pv[j] = J.sparse[sp];
                }
            }
            __syncthreads();
            uint32_t r[kS0Items];
#pragma unroll
            for (int j = 0; j < kS0Items; ++j) {
                const bool act = cb + (uint32_t)(wid * kWaveItems + j * 64 + lane) < T;
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
            uint32_t cnt = 0;
#pragma unroll
            for (int w = 0; w < kSW; ++w) {
                const uint32_t v = wh[w][d];
                wh[w][d] = cnt;
                cnt += v;
            }
            const uint32_t tx_d = block_excl_scan<kST>(cnt, lsb);
            tx[d] = tx_d;
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kS0Items; ++j) {
                if (cb + (uint32_t)(wid * kWaveItems + j * 64 + lane) < T) {
                    const uint32_t dj = (k[j] >> shift) & (kBins - 1);
                    const uint32_t lpos = tx[dj] + wh[wid][dj] + r[j];
                    lk[lpos] = k[j];
                    lp[lpos] = pv[j];
                }
            }
            __syncthreads();
#pragma unroll 4
            for (uint32_t q = threadIdx.x; q < tn; q += kST) {
                const uint32_t kk = lk[q];
                const uint32_t dq = (kk >> shift) & (kBins - 1);
                const uint32_t dst = gbase[dq] + (q - tx[dq]);
                kout[dst] = kk;
                pout[dst] = lp[q];
            }
            __syncthreads();
            gbase[d] += cnt;   // the next chunk's items of digit d follow these
            __syncthreads();
        }
        __syncthreads();   // cpre / gbase of this group are read above before the next one
    }
}

// ---- segments (voxels) of the sorted keys and their centroids ------------------------------
// a sorted position starts a voxel iff its key differs from the previous one
__device__ __forceinline__ bool seg_head(const uint32_t *keys, uint64_t i, uint32_t m) {
    return i < m && (i == 0 || keys[i] != keys[i - 1]);
}

// heads per sort tile and the tile's first head position (UINT32_MAX: none)
__global__ void __launch_bounds__(kST) k_seg_count(const JobBatch jobs) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if (J.passes == 0) return;
    const uint32_t *keys = (J.passes & 1) ? J.keys1 : J.keys0;
    const VoxParams *vpp = J.vp;
    uint32_t *tcount = J.tcount, *fhead = J.fhead;
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
// voxel count (res[slot]).  emit != null (pcp_filter_merge when every cloud is voxelised): the
// centroid goes straight through the cloud's transform + colour into the concatenated output
// at the cloud's offset (the voxel counts of the earlier clouds, from their k_seg_count), as
// k_emit_rgb would write it -- one launch and the out4 round trip fewer.
__global__ void __launch_bounds__(kST)
k_seg_centroid(const JobBatch jobs, uint32_t *__restrict__ res, float4 *__restrict__ emit) {
    const CloudJob &J = jobs.j[blockIdx.y];
    if (J.passes == 0) return;
    const uint32_t *keys = (J.passes & 1) ? J.keys1 : J.keys0;
    const float4 *pay = ((J.passes & 1) != (J.fast != 0)) ? J.sparse : J.xyz;
    const VoxParams *vpp = J.vp;
    const uint32_t *tcount = J.tcount, *fhead = J.fhead;
    float4 *out = J.out4;
    uint32_t *out_idx = J.vidx, *out_cnt = J.vcnt;
    const int slot = J.slot;
    const VoxParams vp = *vpp;
    const uint32_t m = sort_count(vp);
    const uint32_t nact = sort_tiles(vp);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t lds[kSW];
    __shared__ uint32_t hpos[kSortTile + 1];
    __shared__ float4 lp[kSortTile];   // the tile's sorted points
    __shared__ uint32_t wo[kSortItems][kSW];
    uint32_t ebase = 0;   // the cloud's first output record (emit)
    if (emit && nact > blockIdx.x)
        for (int y = 0; y < (int)blockIdx.y; ++y) {
            const CloudJob &K = jobs.j[y];
            ebase += block_prefix_sum<kST>(K.tcount, sort_tiles(*K.vp), lds);
        }
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
    if (t == nact - 1 && threadIdx.x == 0) {
        res[slot] = pre + tot;
        if (J.fast) {   // no k_vox_params in the fast chain: the cropped count, no passthrough
            res[kMaxCloudsDev + 2 * slot] = m;
            res[kMaxCloudsDev + 2 * slot + 1] = 0;
        }
    }
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
    uint32_t a_[kSortItems], n_[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        const bool h = (head >> j) & 1u;
        a_[j] = h ? hpos[loc[j]] : 0u;
        n_[j] = h ? hpos[loc[j] + 1] - a_[j] : 0u;
    }
    float sx[kSortItems], sy[kSortItems], sz[kSortItems];
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) sx[j] = sy[j] = sz[j] = 0.f;
    // the part of each run inside this tile comes from LDS; only the tile's last run can go on
    // past the tile end (global loads, in order, after its in-tile part)
    const uint32_t tend = (uint32_t)(base + kSortTile);
    uint32_t nin[kSortItems], nmax_in = 0;
#pragma unroll
    for (int j = 0; j < kSortItems; ++j) {
        nin[j] = min(n_[j], tend - a_[j]);
        nmax_in = max(nmax_in, nin[j]);
    }
    FLT_STAMP(1, t, 4);
    for (uint32_t q = 0; q < nmax_in; ++q) {
#pragma unroll
        for (int j = 0; j < kSortItems; ++j) {
            if (q < nin[j]) {
                const float4 p = lp[a_[j] + q - (uint32_t)base];
                sx[j] = sx[j] + p.x;
                sy[j] = sy[j] + p.y;
                sz[j] = sz[j] + p.z;
            }
        }
    }
    {
#pragma unroll
        for (int j = 0; j < kSortItems; ++j) {
            for (uint32_t l = a_[j] + nin[j]; l < a_[j] + n_[j]; ++l) {
                const float4 p = pay[l];
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
        if (emit) {
            xform_store(J.rig, sx[j] / cnt, sy[j] / cnt, sz[j] / cnt, emit + 2 * ((size_t)ebase + s));
        } else {
            out[s] = make_float4(sx[j] / cnt, sy[j] / cnt, sz[j] / cnt, 1.0f);
            out_idx[s] = hkey[j];
            out_cnt[s] = n_[j];
        }
    }
    }   // tot != 0
    __syncthreads();
    FLT_STAMP(1, t, 5);
    }
}

// =========================================================================================
// The bucket chain (round 4, pcp_filter_merge / pcp_crop_voxel when every cloud certainly
// voxelises): crop -> k_bk_group -> k_bk_sort -> k_bk_emit, three launches for the voxel stage.
// PCL's idx order is the order of (bucket = idx >> bs, sub = idx & (2^bs - 1)).
//  k_bk_group : one block per group of gt crop tiles (~4 k kept points): the cloud's parameters
//               from the crop's counts and bbox partials, then a counting sort of the group's
//               points by bucket in LDS -- written to xyz at the group's compact offset, one row
//               of bucket starts per group (no global atomics, no cross-block prefix)
//  k_bk_sort  : one block per bucket (consecutive over the clouds): gathers the bucket's runs
//               of every group, counting-sorts them by sub in LDS (unstable), puts each voxel's
//               points back in input order by their crop-slot position (stored in .w), sums
//               them in that order; centroids at the bucket's item offset, voxel count per bucket
//  k_bk_emit  : output offset of each bucket (voxels of the earlier buckets), the centroids
//               copied there -- as merged records (transform + colour) for pcp_filter_merge
// A bucket past kBkCap points (or a parameter past the sizes the host allotted) sets the redo
// flag (res[3 * kMaxCloudsDev]); the host then runs the frame again on the LSD chain.
// =========================================================================================
constexpr int kBkT = 512;                 // threads of the bucket kernels
#ifndef PCP_BK_BITS
#define PCP_BK_BITS 11
#endif
#ifndef PCP_BK_SUB
#define PCP_BK_SUB 12
#endif
constexpr int kBkBits = PCP_BK_BITS;      // target: ~2^kBkBits buckets per cloud
constexpr int kBkSubMax = PCP_BK_SUB;     // sub-key bits at most (LDS table of 2^kBkSubMax + 1)
constexpr int kBkMax = 4096;              // buckets per cloud at most
#ifndef PCP_BK_CAP
#define PCP_BK_CAP 4096
#endif
constexpr int kBkCap = PCP_BK_CAP;        // points per bucket at most (LDS of k_bk_sort)
#ifndef PCP_BK_DENSE
#define PCP_BK_DENSE 512
#endif
constexpr int kBkDense = PCP_BK_DENSE;    // points per voxel ranked in k_bk_sort at most
// bkv layout: [0, kBkChunkOff) per-bucket (voxels, item offset), then per-64-bucket voxel sums
constexpr uint32_t kBkChunkOff = kBatch * kBkMax;
constexpr int kBkGt = 15;                 // crop tiles per group at most
constexpr int kBkGItems = 12;             // per thread and chunk in k_bk_group
#ifndef PCP_BK_STAGE
#define PCP_BK_STAGE 1                    // k_bk_group places a one-chunk group in LDS first
#endif

__device__ __forceinline__ void bk_redo(uint32_t *res) { res[3 * kMaxCloudsDev] = 1u; }

// crop tile u of the group holding item q: the last u with cpre[u] <= q (cpre ascending)
__device__ __forceinline__ uint32_t bk_tile_of(const uint32_t *cpre, uint32_t gt, uint32_t q) {
    uint32_t lo = 0, hi = gt;   // cpre[lo] <= q < cpre[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cpre[mid] <= q) lo = mid; else hi = mid;
    }
    return lo;
}

__global__ void __launch_bounds__(kBkT)
k_bk_group(const JobBatch jobs, uint32_t *__restrict__ res, uint2 *__restrict__ bkv) {
    const CloudJob &J = jobs.j[blockIdx.y];
    // k_bk_sort's per-64-bucket voxel sums start at 0
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (uint32_t q = threadIdx.x; q < (uint32_t)kBatch * kBkMax / 64; q += kBkT)
            bkv[kBkChunkOff + q] = make_uint2(0u, 0u);
    const uint32_t g = blockIdx.x;
    if (!J.bk || g >= J.ng) return;
    [[maybe_unused]] const uint32_t stt = blockIdx.y * gridDim.x + blockIdx.x;   // stamp slot
    FLT_STAMP(0, stt, 0);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint32_t nb = J.nb, c0 = g * J.gt, c1 = min(c0 + J.gt, nb), gt = c1 - c0;
    // the cloud's cropped count, the points of tiles before the group, the cropped bbox
    uint32_t tot = 0, pre = 0;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    // the group's crop-tile counts (wave 0), issued with the loads below
    const uint32_t gcnt = (threadIdx.x < 64 && threadIdx.x < gt) ? J.counts[c0 + threadIdx.x] : 0u;
    // four tiles per thread and round, every load of a round issued before any is used
    for (uint32_t t0 = threadIdx.x; t0 < nb; t0 += 4 * kBkT) {
        uint32_t v[4];
        float2 pa[4], pb[4], pc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t t = min(t0 + u * kBkT, nb - 1);
            v[u] = J.counts[t];
            pa[u] = reinterpret_cast<const float2 *>(J.part)[3 * t];
            pb[u] = reinterpret_cast<const float2 *>(J.part)[3 * t + 1];
            pc[u] = reinterpret_cast<const float2 *>(J.part)[3 * t + 2];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t t = t0 + u * kBkT;
            if (t >= nb) continue;   // (a clamped duplicate: min/max only, never counted)
            tot += v[u];
            pre += t < c0 ? v[u] : 0u;
            mn[0] = fminf(mn[0], pa[u].x); mn[1] = fminf(mn[1], pa[u].y);
            mn[2] = fminf(mn[2], pb[u].x); mx[0] = fmaxf(mx[0], pb[u].y);
            mx[1] = fmaxf(mx[1], pc[u].x); mx[2] = fmaxf(mx[2], pc[u].y);
        }
    }
    tot = wave_sum_dpp(tot);
    pre = wave_sum_dpp(pre);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        mn[a] = wave_minmax_dpp<false>(mn[a]);
        mx[a] = wave_minmax_dpp<true>(mx[a]);
    }
    __shared__ float sred[8][kBkT / 64];
    __shared__ uint32_t cpre[kBkGt + 1];
    __shared__ uint32_t h[kBkMax + 1];
    if (lane == 0) {
        sred[0][wid] = __uint_as_float(tot);
        sred[1][wid] = __uint_as_float(pre);
        for (int a = 0; a < 3; ++a) {
            sred[2 + a][wid] = mn[a];
            sred[5 + a][wid] = mx[a];
        }
    }
    if (threadIdx.x < 64) {   // the group's crop-tile counts, prefix by one wave
        const uint32_t incl = wave_incl_scan_dpp(gcnt);
        if (threadIdx.x == 0) cpre[0] = 0;
        if (threadIdx.x < gt) cpre[threadIdx.x + 1] = incl;
    }
    __syncthreads();
    tot = 0;
    pre = 0;
#pragma unroll
    for (int w = 0; w < kBkT / 64; ++w) {
        tot += __float_as_uint(sred[0][w]);
        pre += __float_as_uint(sred[1][w]);
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], sred[2 + a][w]);
            mx[a] = fmaxf(mx[a], sred[5 + a][w]);
        }
    }
    VoxParams p = vox_params_from(tot, mn, mx, J.leaf);
    // buckets: bs = clamp(max(bits(nvox) - kBkBits, bits(nvox) - bkpb), 0, kBkSubMax), nbk =
    // ceil(nvox / 2^bs): ~2^kBkBits buckets, and no more than ~ input points / PCP_BK_PTS (a
    // sparse cloud -- C5's scans: ~100 points per 2^11 buckets of its box -- fills fewer, fuller
    // buckets instead of thousands of near-empty blocks)
    bool redo = p.overflow != 0;
    if (tot != 0 && !redo) {
        int bits = 0;
        while (bits < 40 && (1ull << bits) < p.nvox) ++bits;
        p.bs = (uint32_t)min(max(max(bits - kBkBits, bits - J.bkpb), 0), kBkSubMax);
        const uint64_t nbk = (p.nvox + (1ull << p.bs) - 1) >> p.bs;
        if (nbk > J.nbkcap) redo = true;
        else p.nbk = (uint32_t)nbk;
    }
    if (redo) p.nbk = 0;
    if (g == 0 && threadIdx.x == 0) {
        *J.vp = p;
        res[J.slot] = 0;   // k_bk_emit writes it when the cloud has buckets
        res[kMaxCloudsDev + 2 * J.slot] = tot;
        res[kMaxCloudsDev + 2 * J.slot + 1] = 0;
        if (redo) bk_redo(res);
    }
    if (p.nbk == 0) return;   // uniform: nothing cropped, or the frame is redone
    FLT_STAMP(0, stt, 1);
    const uint32_t nbk = p.nbk, bs = p.bs;
    const uint32_t T = cpre[gt];
    for (uint32_t b = threadIdx.x; b <= nbk; b += kBkT) h[b] = 0;
    __syncthreads();
    constexpr uint32_t kChunk = (uint32_t)kBkT * kBkGItems;
    const uint32_t nch = (T + kChunk - 1) / kChunk;
    float4 v[kBkGItems];
    uint32_t bk[kBkGItems];
    // pass A: bucket counts (the last chunk stays in registers for pass B); a chunk's loads
    // are all issued before its LDS atomics
    uint32_t spj[kBkGItems];
    for (uint32_t ch = 0; ch < nch; ++ch) {
#pragma unroll
        for (int j = 0; j < kBkGItems; ++j) {
            const uint32_t q = ch * kChunk + (uint32_t)j * kBkT + threadIdx.x;
            const uint32_t qc = min(q, T - 1);
            const uint32_t u = bk_tile_of(cpre, gt, qc);
            spj[j] = (c0 + u) * (uint32_t)kCropTile + (qc - cpre[u]);
            v[j] = J.sparse[spj[j]];
        }
#pragma unroll
        for (int j = 0; j < kBkGItems; ++j) {
            const uint32_t q = ch * kChunk + (uint32_t)j * kBkT + threadIdx.x;
            v[j].w = __uint_as_float(spj[j]);
            bk[j] = vox_key(p, v[j].x, v[j].y, v[j].z) >> bs;
            if (q < T) atomicAdd(&h[bk[j]], 1u);
        }
    }
    __syncthreads();
    FLT_STAMP(0, stt, 2);
    // exclusive scan of the counts -> starts (contiguous runs of B buckets per thread)
    {
        __shared__ uint32_t lsc[kBkT / 64];
        const uint32_t per = (nbk + kBkT - 1) / kBkT;
        const uint32_t b0 = min(threadIdx.x * per, nbk), b1 = min(b0 + per, nbk);
        uint32_t loc = 0;
        for (uint32_t b = b0; b < b1; ++b) loc += h[b];
        uint32_t ex = block_excl_scan_dpp<kBkT>(loc, lsc);
        uint32_t *row = J.brows + (size_t)g * (nbk + 1);
        for (uint32_t b = b0; b < b1; ++b) {
            const uint32_t c = h[b];
            h[b] = ex;
            row[b] = pre + ex;
            ex += c;
        }
        if (threadIdx.x == 0) row[nbk] = pre + T;
    }
    __syncthreads();
    FLT_STAMP(0, stt, 3);
    // pass B: each point to its bucket's next slot (LDS arrival order: not stable, k_bk_sort
    // restores input order inside each voxel from the slot position in .w)
    float4 *gout = J.xyz + pre;
#if PCP_BK_STAGE
    if (nch == 1) {   // uniform: the group fits one chunk -- placed in LDS, stored coalesced
        __shared__ float4 stg[kChunk];
#pragma unroll
        for (int j = 0; j < kBkGItems; ++j) {
            const uint32_t q = (uint32_t)j * kBkT + threadIdx.x;
            if (q < T) stg[atomicAdd(&h[bk[j]], 1u)] = v[j];
        }
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < T; q += kBkT) gout[q] = stg[q];
        FLT_STAMP(0, stt, 4);
        return;
    }
#endif
    for (int32_t ch = (int32_t)nch - 1; ch >= 0; --ch) {
#pragma unroll
        for (int j = 0; j < kBkGItems; ++j) {
            const uint32_t q = (uint32_t)ch * kChunk + (uint32_t)j * kBkT + threadIdx.x;
            if (q < T) {
                if ((uint32_t)ch != nch - 1) {   // (only groups past one chunk)
                    const uint32_t u = bk_tile_of(cpre, gt, q);
                    const uint32_t sp = (c0 + u) * (uint32_t)kCropTile + (q - cpre[u]);
                    const float4 a = J.sparse[sp];
                    v[j] = make_float4(a.x, a.y, a.z, __uint_as_float(sp));
                    bk[j] = vox_key(p, a.x, a.y, a.z) >> bs;
                }
                gout[atomicAdd(&h[bk[j]], 1u)] = v[j];
            }
        }
    }
    FLT_STAMP(0, stt, 4);
}

// the cloud of look-back position f and its first position b0 (the clouds' buckets follow one
// another); -1: past the last bucket
__device__ __forceinline__ int bk_cloud_of(const JobBatch &jobs, int k, uint32_t f, uint32_t &b0) {
    b0 = 0;
    for (int y = 0; y < k; ++y) {
        const uint32_t nb = jobs.j[y].bk ? jobs.j[y].vp->nbk : 0u;
        if (f < b0 + nb) return y;
        b0 += nb;
    }
    return -1;
}

// k_bk_sort: one block per bucket.  The bucket's runs of every group gathered (one point per
// thread and round, registers), counted per sub-key in LDS (arrival order), one packed scan ->
// (start | voxel rank << 16) per sub-key, slots by arrival, then each point's rank among its
// voxel's points by crop-slot position (input order), and the voxel sums in that order by the
// voxel's first point.  The centroids land at the bucket's item offset in the cloud (sparse is
// free after k_bk_group), (voxels, offset) in bkv[f]; k_bk_emit places them.
#ifndef PCP_BK_T3
#define PCP_BK_T3 512
#endif
constexpr int kBkT3 = PCP_BK_T3;
// 64 VGPRs: 8 waves per SIMD, four 512-thread blocks per CU (LDS admits four); build knob
// PCP_BK_W8=0 lets the compiler take 68 (three blocks per CU): 0.104 vs 0.101 ms per frame
#ifndef PCP_BK_W8
#define PCP_BK_W8 1
#endif
#if PCP_BK_W8
#define PCP_BK_SORT_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define PCP_BK_SORT_ATTR
#endif
constexpr int kBkItems3 = kBkCap / kBkT3;
constexpr int kBkNg = kBkT3;              // groups per cloud at most (one per k_bk_sort thread)
__global__ void __launch_bounds__(kBkT3) PCP_BK_SORT_ATTR
k_bk_sort(const JobBatch jobs, int k, uint32_t *__restrict__ res, uint2 *__restrict__ bkv,
          int idx_out) {
    const uint32_t f = blockIdx.x;
    uint32_t b0;
    const int c = bk_cloud_of(jobs, k, f, b0);
    if (c < 0) return;
    FLT_STAMP(1, f, 0);
    const CloudJob &J = jobs.j[c];
    const VoxParams P = *J.vp;
    const uint32_t b = f - b0, bs = P.bs, nsub = 1u << bs, stride = P.nbk + 1;
    const uint32_t ng = J.ng;
    __shared__ uint32_t og[kBkNg + 1], sg[kBkNg];
    __shared__ uint32_t tab[(1 << kBkSubMax) + 1];   // counts, then start | voxel rank << 16
    __shared__ uint32_t p1[kBkCap];                  // slot -> crop-slot position, then
                                                     // input-order slot -> xyz index
    __shared__ uint32_t lsa[kBkT3 / 64], lsb[kBkT3 / 64];
    __shared__ uint32_t sdense;   // a voxel of the bucket holds more than kBkDense points
    // the bucket's run in every group, and its item offset in the cloud (points of the earlier
    // buckets: sum over the groups of row[b] - row[0])
    uint32_t gc = 0, gsum = 0;
    if (threadIdx.x < ng) {
        const uint32_t *row = J.brows + (size_t)threadIdx.x * stride;
        const uint32_t r0 = row[0], rb = row[b], rb1 = row[b + 1];
        gsum = rb - r0;
        gc = rb1 - rb;
        sg[threadIdx.x] = rb;
    }
    gsum = wave_sum_dpp(gsum);
    if ((threadIdx.x & 63) == 0) lsb[threadIdx.x >> 6] = gsum;
    const uint32_t gex = block_excl_scan_dpp<kBkT3>(gc, lsa);
    if (threadIdx.x < ng) og[threadIdx.x] = gex;
    if (threadIdx.x == kBkT3 - 1) og[ng] = gex + gc;
    for (uint32_t e = threadIdx.x; e <= nsub; e += kBkT3) tab[e] = 0;
    if (threadIdx.x == 0) sdense = 0u;
    __syncthreads();
    uint32_t ioff = 0;
#pragma unroll
    for (int w = 0; w < kBkT3 / 64; ++w) ioff += lsb[w];
    const uint32_t n = og[ng];
    const bool fits = n <= (uint32_t)kBkCap;
    FLT_STAMP(1, f, 1);
    uint32_t pos[kBkItems3], sxi[kBkItems3], sub[kBkItems3], arr[kBkItems3];
    if (fits) {
        float4 a[kBkItems3];
#pragma unroll
        for (int j = 0; j < kBkItems3; ++j) {
            const uint32_t q = (uint32_t)j * kBkT3 + threadIdx.x;
            if (q < n) {
                uint32_t lo = 0, hi = ng;   // og[lo] <= q < og[hi]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (og[mid] <= q) lo = mid; else hi = mid;
                }
                sxi[j] = sg[lo] + (q - og[lo]);
                a[j] = J.xyz[sxi[j]];
            }
        }
#pragma unroll
        for (int j = 0; j < kBkItems3; ++j) {
            const uint32_t q = (uint32_t)j * kBkT3 + threadIdx.x;
            if (q < n) {
                pos[j] = __float_as_uint(a[j].w);
                sub[j] = vox_key(P, a[j].x, a[j].y, a[j].z) & (nsub - 1u);
                arr[j] = atomicAdd(&tab[sub[j]], 1u);
            }
        }
    }
    __syncthreads();
    FLT_STAMP(1, f, 2);
    if (!fits) {   // uniform: the host redoes the frame on the LSD chain
        if (threadIdx.x == 0) {
            bk_redo(res);
            bkv[f] = make_uint2(0u, ioff);
        }
        return;
    }
    // one packed exclusive scan of the table: points (low 16 bits) and occupied sub-keys (high
    // 16).  Wave w owns the contiguous segment [w S, (w + 1) S); round r covers its entries
    // r * 64 + lane (no bank conflicts).  All rounds' loads and DPP scans are independent of
    // each other (ILP), the rounds' totals chain in scalar adds, one barrier for the waves
    uint32_t nvox;
    {
        constexpr int kR = ((1 << kBkSubMax) + kBkT3 - 1) / kBkT3;   // rounds per wave at most
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        const uint32_t S = max(64u, nsub / (uint32_t)(kBkT3 / 64));
        const uint32_t e0 = (uint32_t)wid * S;
        uint32_t wtot = 0;
        constexpr int kH = kR < 4 ? kR : 4;   // rounds in flight together (register pressure)
#pragma unroll
        for (int r0 = 0; r0 < kR; r0 += kH) {
            uint32_t v[kH];
#pragma unroll
            for (int h = 0; h < kH; ++h) {
                const int r = r0 + h;
                const uint32_t e = e0 + (uint32_t)r * 64 + lane;
                const uint32_t t = (r < kR && (uint32_t)r * 64 < S && e < nsub) ? tab[e] : 0u;
                v[h] = t | (t ? 0x10000u : 0u);
            }
#pragma unroll
            for (int h = 0; h < kH; ++h) {
                if (r0 + h >= kR) continue;
                const uint32_t x = wave_incl_scan_dpp(v[h]);
                const uint32_t rt = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
                const int r = r0 + h;
                const uint32_t e = e0 + (uint32_t)r * 64 + lane;
                if ((uint32_t)r * 64 < S && e < nsub)
                    tab[e] = x - v[h] + wtot;   // exclusive within the wave's segment
                wtot += rt;
            }
        }
        if (lane == 0) lsa[wid] = wtot;
        __syncthreads();
        uint32_t off = 0, all = 0;
#pragma unroll
        for (int w = 0; w < kBkT3 / 64; ++w) {
            off += w < wid ? lsa[w] : 0u;
            all += lsa[w];
        }
        nvox = all >> 16;
        if (off) {   // wave-uniform: the segments after the first get their wave's offset
#pragma unroll
            for (int r = 0; r < kR; ++r) {
                const uint32_t e = e0 + (uint32_t)r * 64 + lane;
                if ((uint32_t)r * 64 < S && e < nsub) tab[e] += off;
            }
        }
        if (threadIdx.x == 0) tab[nsub] = n | (nvox << 16);
    }
    __syncthreads();
    FLT_STAMP(1, f, 3);
    // slots in sub-key order, arrival order inside a voxel
#pragma unroll
    for (int j = 0; j < kBkItems3; ++j) {
        const uint32_t q = (uint32_t)j * kBkT3 + threadIdx.x;
        if (q < n) p1[(tab[sub[j]] & 0xffffu) + arr[j]] = pos[j];
    }
    __syncthreads();
    FLT_STAMP(1, f, 4);
    // input order inside each voxel: rank by crop-slot position among the voxel's points.  A
    // voxel past kBkDense points would cost cnt^2 LDS reads in this one block (4,096 points: ~16 M,
    // more than the whole frame): such a frame is redone on the LSD chain instead,
    // and the block stops here -- no rank, no sums (dense points left r = 0, so every
    // one of them summed the whole voxel)
    uint32_t head = 0, fin[kBkItems3];
#pragma unroll
    for (int j = 0; j < kBkItems3; ++j) {
        const uint32_t q = (uint32_t)j * kBkT3 + threadIdx.x;
        if (q < n) {
            const uint32_t st = tab[sub[j]] & 0xffffu;
            const uint32_t cnt = (tab[sub[j] + 1] & 0xffffu) - st;
            uint32_t r = 0;
            if (cnt > (uint32_t)kBkDense) sdense = 1u;
            else
                for (uint32_t u = st; cnt > 1 && u < st + cnt; ++u) r += p1[u] < pos[j] ? 1u : 0u;
            fin[j] = st + r;
            head |= (r == 0 ? 1u : 0u) << j;
        }
    }
    __syncthreads();   // every rank read p1 before it holds xyz indices
    if (sdense) {   // uniform: the host redoes the frame on the LSD chain
        if (threadIdx.x == 0) {
            bk_redo(res);
            bkv[f] = make_uint2(0u, ioff);
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < kBkItems3; ++j) {
        const uint32_t q = (uint32_t)j * kBkT3 + threadIdx.x;
        if (q < n) p1[fin[j]] = sxi[j];
    }
    __syncthreads();
    FLT_STAMP(1, f, 5);
    // each voxel's first point (in input order) sums the voxel in input order
    float4 *tmp = J.sparse + ioff;
#pragma unroll
    for (int j = 0; j < kBkItems3; ++j) {
        if (!((head >> j) & 1u)) continue;
        const uint32_t t0 = tab[sub[j]], st = t0 & 0xffffu, vr = t0 >> 16;
        const uint32_t cnt = (tab[sub[j] + 1] & 0xffffu) - st;
        float sx = 0.f, sy = 0.f, sz = 0.f;
        // four loads in flight, then the adds in input order (bit-identical)
        for (uint32_t u = st; u < st + cnt; u += 4) {
            float4 a[4];
#pragma unroll
            for (int h = 0; h < 4; ++h)
                if (u + h < st + cnt) a[h] = J.xyz[p1[u + h]];
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                if (u + h >= st + cnt) break;
                sx = sx + a[h].x;
                sy = sy + a[h].y;
                sz = sz + a[h].z;
            }
        }
        const float fc = (float)cnt;
        tmp[vr] = make_float4(sx / fc, sy / fc, sz / fc, 1.0f);
        if (idx_out) {   // pcp_crop_voxel: idx and count beside the centroid
            J.keys0[ioff + vr] = (b << bs) | sub[j];
            J.keys1[ioff + vr] = cnt;
        }
    }
    if (threadIdx.x == 0) {
        bkv[f] = make_uint2(nvox, ioff);
        if (nvox) atomicAdd(&bkv[kBkChunkOff + (f >> 6)].x, nvox);   // k_bk_emit's chunk sums
    }
    FLT_STAMP(1, f, 6);
}

// k_bk_emit: one block per bucket.  Output offset = voxels of every earlier bucket of the call:
// the per-64-bucket sums k_bk_sort accumulated before f's chunk + the buckets of f's chunk
// before f (one load per lane of one wave); the centroids copied there (emit: through the
// cloud's transform + colour as merged records); the cloud's last bucket writes its count.
#ifndef PCP_BK_TE
#define PCP_BK_TE 256
#endif
constexpr int kBkTE = PCP_BK_TE;          // k_bk_emit threads (build knob)
__device__ __forceinline__ uint32_t bk_voxels_before(const uint2 *bkv, uint32_t f) {
    // wave 0 only (full wave): lanes sum chunk sums [0, f / 64) and buckets [f & ~63, f)
    const uint32_t lane = threadIdx.x & 63, nch = f >> 6, c0 = f & ~63u;
    uint32_t s = 0;
    for (uint32_t q = lane; q < nch; q += 64) s += bkv[kBkChunkOff + q].x;
    if (c0 + lane < f) s += bkv[c0 + lane].x;
    return wave_sum_dpp(s);
}
__global__ void __launch_bounds__(kBkTE)
k_bk_emit(const JobBatch jobs, int k, uint32_t *__restrict__ res, float4 *__restrict__ emit,
          const uint2 *__restrict__ bkv) {
    const uint32_t f = blockIdx.x;
    uint32_t b0;
    const int c = bk_cloud_of(jobs, k, f, b0);
    if (c < 0) return;
    const CloudJob &J = jobs.j[c];
    __shared__ uint32_t sh[2];
    // the cloud's own outputs (centroids, or keep16 beside the merged records) are indexed from
    // the cloud's first voxel: eb = the voxels of the earlier clouds' buckets
    const bool own = !emit || J.keep16;
    if (threadIdx.x < 64) {
        const uint32_t e = bk_voxels_before(bkv, f);
        const uint32_t eb = own ? bk_voxels_before(bkv, b0) : 0u;
        if (threadIdx.x == 0) {
            sh[0] = e;
            sh[1] = eb;
        }
    }
    __syncthreads();
    const uint32_t e = sh[0], eo = sh[0] - sh[1];
    const uint2 kv = bkv[f];
    const float4 *tmp = J.sparse + kv.y;
    for (uint32_t v0 = 0; v0 < kv.x; v0 += 4 * kBkTE) {
        float4 a[4];
        uint32_t iv[4], cv[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t v = v0 + u * kBkTE + threadIdx.x;
            if (v < kv.x) {
                a[u] = tmp[v];
                if (!emit) {
                    iv[u] = J.keys0[kv.y + v];
                    cv[u] = J.keys1[kv.y + v];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t v = v0 + u * kBkTE + threadIdx.x;
            if (v >= kv.x) continue;
            if (emit) {
                xform_store(J.rig, a[u].x, a[u].y, a[u].z, emit + 2 * ((size_t)e + v));
                if (J.keep16) J.keep16[eo + v] = a[u];
            } else {
                J.out4[eo + v] = a[u];
                J.vidx[eo + v] = iv[u];
                J.vcnt[eo + v] = cv[u];
            }
        }
    }
    if (f - b0 == J.vp->nbk - 1 && threadIdx.x < 64) {   // the cloud's last bucket
        const uint32_t before = bk_voxels_before(bkv, b0);
        if (threadIdx.x == 0) res[J.slot] = e + kv.x - before;
    }
}

// transform + colour of every cloud's result into the concatenated output (cloud order: the
// robot first), counts[] = result counts of the clouds
__global__ void __launch_bounds__(kFT)
k_emit_rgb(const JobBatch jobs, const uint32_t *__restrict__ counts,
           float4 *__restrict__ out) {
    const CloudJob &J = jobs.j[blockIdx.y];
    const int slot = J.slot;
    const VoxParams vp = *J.vp;
    const float4 *src = (vp.do_voxel && !vp.overflow) ? J.out4 : J.xyz;
    const Rigid r = J.rig;
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

// several raw blobs in one launch (pcp_transform_concat): block b belongs to the cloud whose
// tile range [tile0[i], tile0[i+1]) holds it; cloud i's records land at out + 2 * base[i]
constexpr int kXfMax = 8;
struct XformBatch {
    int k;
    CloudIn c[kXfMax];
    Rigid r[kXfMax];
    uint64_t base[kXfMax];
    uint32_t tile0[kXfMax + 1];
};
__global__ void __launch_bounds__(kFT) k_xform_batch(XformBatch B, float4 *__restrict__ out) {
    int i = 0;
    while (i + 1 < B.k && blockIdx.x >= B.tile0[i + 1]) ++i;
    const uint64_t j = (uint64_t)(blockIdx.x - B.tile0[i]) * kFT + threadIdx.x;
    if (j >= B.c[i].n) return;
    float x, y, z;
    load_xyz(B.c[i], j, x, y, z);
    xform_store(B.r[i], x, y, z, out + 2 * (B.base[i] + j));
}

// =========================================================================================
// host orchestration: one job per cloud in a device table; every stage is one batched launch
// (grid.y = clouds) on ctx->stream with sizes kept on the device, so a whole crop -> voxel ->
// transform frame runs without host round trips (and is captured into a hipGraph by
// pcp_filter_merge when its inputs are device-resident).
// =========================================================================================
constexpr int kMaxClouds = 64;
// result words of a call: counts [kMaxClouds], (cropped, passthrough) [2 kMaxClouds], the bucket
// chain's redo flag
constexpr int kResWords = 3 * kMaxClouds + 4;

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// per-slot results shared by all clouds of a call: VoxParams[kMaxClouds], then
// res[kMaxClouds] result counts and info[2*kMaxClouds] (cropped count, passthrough flag)
static int ensure_misc(pcp_ctx *ctx, VoxParams *&vp, uint32_t *&res) {
    const size_t vb = align256(kMaxClouds * sizeof(VoxParams));
    PCP_HIP(ctx, ctx->f_misc.ensure(vb + kResWords * 4));
    vp = reinterpret_cast<VoxParams *>(ctx->f_misc.as<char>());
    res = reinterpret_cast<uint32_t *>(ctx->f_misc.as<char>() + vb);
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

// scratch of cloud `slot` (ctx->fbuf[slot], grow-only) and its job; the caller sized ctx->fbuf
static int make_job(pcp_ctx *ctx, int slot, const CloudIn &c, const Box &b, float leaf,
                    bool want_idx, const Rigid &rig, VoxParams *vp_all, CloudJob &J) {
    if (c.n >= (1ull << 31))
        return set_err(ctx, PCP_E_INVALID, "cloud of %llu points: at most 2^31-1 per call",
                       (unsigned long long)c.n);
    CloudBufs &B = ctx->fbuf[slot];
    const uint64_t ncap = c.n ? c.n : 1;
    const uint32_t nb = (uint32_t)((ncap + kCropTile - 1) / kCropTile);
    const uint32_t nt = (uint32_t)((ncap + kSortTile - 1) / kSortTile);
    const uint32_t ntp = (nt + 15) & ~15u, ngp = (nt + kGroup - 1) / kGroup;
    const uint32_t nzero = (uint32_t)((size_t)kMaxPasses * kBins * (1 + ngp));
    PCP_HIP(ctx, B.xyz.ensure((ncap + 1) * sizeof(float4)));
    PCP_HIP(ctx, B.sparse.ensure((size_t)nb * kCropTile * sizeof(float4)));   // whole tiles
    if (want_idx) {
        PCP_HIP(ctx, B.idx.ensure((ncap + 1) * sizeof(uint32_t)));
        PCP_HIP(ctx, B.sparse_idx.ensure((size_t)nb * kCropTile * sizeof(uint32_t)));
    }
    for (int q = 0; q < 2; ++q) PCP_HIP(ctx, B.keys[q].ensure((ncap + 16) * sizeof(uint32_t)));
    const size_t cb = align256((size_t)(nb + 4) * 4), pb = align256((size_t)nb * 24);
    const size_t zb = align256((size_t)nzero * 4);
    const size_t hb = align256((size_t)kBins * ntp * 4), sb = align256((size_t)(ntp + 4) * 4);
    PCP_HIP(ctx, B.hist.ensure(cb + pb + zb + hb + 2 * sb));
    // voxel results: out4 (ncap+1) | idx (ncap+1) | cnt (ncap+1)
    PCP_HIP(ctx, B.out.ensure((ncap + 1) * sizeof(float4) + (2 * ncap + 8) * 4 + 256));
    char *h = B.hist.as<char>();
    J = CloudJob{};
    J.in = c;
    J.box = b;
    J.leaf = leaf;
    J.passes = (leaf > 0.0f && c.n > 0) ? radix_passes(b, leaf) : 0;
    J.nb = c.n ? nb : 0;
    J.ntp = ntp;
    J.ngp = ngp;
    J.nzero = nzero;
    J.counts = reinterpret_cast<uint32_t *>(h);
    J.part = reinterpret_cast<float *>(h + cb);
    J.zero = reinterpret_cast<uint32_t *>(h + cb + pb);
    J.rhist = reinterpret_cast<uint32_t *>(h + cb + pb + zb);
    J.tcount = reinterpret_cast<uint32_t *>(h + cb + pb + zb + hb);
    J.fhead = reinterpret_cast<uint32_t *>(h + cb + pb + zb + hb + sb);
    J.sparse = B.sparse.as<float4>();
    J.sparse_idx = want_idx ? B.sparse_idx.as<uint32_t>() : nullptr;
    J.xyz = B.xyz.as<float4>();
    J.kept_idx = want_idx ? B.idx.as<uint32_t>() : nullptr;
    J.keys0 = B.keys[0].as<uint32_t>();
    J.keys1 = B.keys[1].as<uint32_t>();
    J.out4 = B.out.as<float4>();
    J.vidx = reinterpret_cast<uint32_t *>(J.out4 + ncap + 1);
    J.vcnt = J.vidx + ncap + 1;
    J.vp = vp_all + slot;
    J.rig = rig;
    J.slot = slot;
    return PCP_OK;
}

// the fast chain's key geometry for job J (its box finite, leaf > 0, n > 0): box floor kb =
// floor(lo * inv) - 2 per axis (a margin for the float product p * inv of a point just inside
// the box), dims DX, DY, DZ past floor(hi * inv) + 1; false when the keys or the float
// integers would not be exact (|values| >= 2^23, or DX * DY * DZ >= 2^31)
static bool fast_geometry(pcp_ctx *ctx, int slot, CloudJob &J, int clouds = 1) {
    if (J.in.n == 0 || !(J.leaf > 0.0f)) return false;
    const float inv = 1.0f / J.leaf;
    const double invd = (double)inv;
    const double lo[3] = {J.box.x0, J.box.y0, J.box.z0}, hi[3] = {J.box.x1, J.box.y1, J.box.z1};
    double dim[3];
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
        const double f0 = std::floor(lo[a] * invd) - 2.0, f1 = std::floor(hi[a] * invd) + 2.0;
        if (std::fabs(f0) >= 8388608.0 || std::fabs(f1) >= 8388608.0 || !(f1 > f0)) return false;
        J.kb[a] = (float)f0;
        dim[a] = f1 - f0 + 1.0;
    }
    const double nv = dim[0] * dim[1] * dim[2];
    if (!(nv < 2147483647.0)) return false;
    int bits = 0;
    while (bits < 31 && std::ldexp(1.0, bits) < nv) ++bits;
    const uint32_t nb = J.nb;
    CloudBufs &B = ctx->fbuf[slot];
    if (B.skeys.ensure((size_t)nb * kCropTile * 4 + (size_t)nb * kBins * 4 + 256) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    J.fast = 1;
    J.kinv = inv;
    J.kdx = (uint32_t)dim[0];
    J.kdxy = (uint32_t)dim[0] * (uint32_t)dim[1];
    J.passes = std::max(1, (bits + kDigitBits - 1) / kDigitBits);
    J.skeys = B.skeys.as<uint32_t>();
    J.h0 = J.skeys + (size_t)nb * kCropTile;
    // groups: every group of every cloud in one round of one-block-per-CU blocks (the pass-0
    // scatter's LDS admits one per CU), at least 8 crop tiles each
    const uint32_t cus = (uint32_t)std::max(ctx->num_cus, 1);
    J.gt = std::min<uint32_t>(kMaxGroupTiles,
                              std::max<uint32_t>(8, (nb * (uint32_t)clouds + cus - 1) / cus));
    J.ng = (nb + J.gt - 1) / J.gt;
    return true;
}

// the bucket chain's sizes for job J (finite box, leaf > 0, n > 0, box keys below 2^31): groups
// of gt crop tiles (<= kBkNg per cloud), rows for the most buckets the cropped bbox can need
static bool bucket_geometry(pcp_ctx *ctx, int slot, CloudJob &J, int clouds = 1) {
    if (J.in.n == 0 || !(J.leaf > 0.0f)) return false;
    const double lo[3] = {J.box.x0, J.box.y0, J.box.z0}, hi[3] = {J.box.x1, J.box.y1, J.box.z1};
    double nv = 1.0;
    for (int a = 0; a < 3; ++a) {
        if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
        nv *= std::floor((hi[a] - lo[a]) / (double)J.leaf) + 3.0;
    }
    if (!(nv < 2147483647.0)) return false;
    const uint32_t nb = J.nb;
    const uint32_t cus = (uint32_t)std::max(ctx->num_cus, 1);
    // one round of blocks for all groups of the call, at most kBkGt tiles (< 64 Ki points) each;
    // a frame that packs >= 8 tiles per group anyway takes 14: fewer, longer runs per bucket for
    // k_bk_sort to gather (C3: 314 -> 304 MB per frame, same time), still one round
    uint32_t gt = std::max<uint32_t>(1, (nb * (uint32_t)clouds + cus - 1) / cus);
    if (gt >= 8) gt = std::max<uint32_t>(gt, 14);
    if (ctx->bk_gt > 0) gt = (uint32_t)ctx->bk_gt;   // PCP_BK_GT (A/B)
    gt = std::min<uint32_t>(gt, kBkGt);
    const uint32_t ng = (nb + gt - 1) / gt;
    if (ng > (uint32_t)kBkNg) return false;
    // device: bs = clamp(max(bits(nvox) - kBkBits, bits(nvox) - bkpb), 0, kBkSubMax), nbk =
    // ceil(nvox / 2^bs) <= 2^min(kBkBits, bkpb), or ceil(nvox / 2^kBkSubMax) where bs is clamped
    int pb = 64;
    if (ctx->bk_pts > 0) {
        const uint64_t tgt = std::max<uint64_t>(J.in.n / (uint64_t)ctx->bk_pts, 1);
        pb = 0;
        while ((1ull << pb) < tgt) ++pb;
    }
    const double cap = std::max(std::ldexp(1.0, std::min(kBkBits, pb)),
                                std::ceil(nv / std::ldexp(1.0, kBkSubMax)));
    const uint32_t nbkcap = (uint32_t)std::min<double>(cap, (double)kBkMax);
    CloudBufs &B = ctx->fbuf[slot];
    // rows, and the look-back words of a call's clouds (sized here: enqueue may be capturing)
    if (B.skeys.ensure((size_t)ng * (nbkcap + 1) * 4 + 256) != hipSuccess ||
        ctx->bk_stat.ensure(((size_t)kBkChunkOff + kBatch * kBkMax / 64) * 8) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    J.bk = 1;
    J.bkpb = pb;
    J.gt = gt;
    J.ng = ng;
    J.nbkcap = nbkcap;
    J.brows = B.skeys.as<uint32_t>();
    J.fast = 0;
    return true;
}

struct Batch {
    JobBatch jb{};
    int k = 0;
    uint32_t max_nb = 0, max_nt = 0;
    int max_passes = 0;
    uint64_t max_n = 0;
};

// the clouds in launch batches of <= kBatch (one batch for any realistic frame)
static std::vector<Batch> batches_of(const std::vector<CloudJob> &jobs) {
    std::vector<Batch> out;
    for (size_t b0 = 0; b0 < jobs.size(); b0 += kBatch) {
        Batch bt;
        bt.k = (int)std::min<size_t>(kBatch, jobs.size() - b0);
        for (int i = 0; i < bt.k; ++i) {
            const CloudJob &J = jobs[b0 + i];
            bt.jb.j[i] = J;
            bt.max_nb = std::max(bt.max_nb, J.nb);
            bt.max_nt = std::max(bt.max_nt, (uint32_t)((J.in.n + kSortTile - 1) / kSortTile));
            bt.max_passes = std::max(bt.max_passes, (int)J.passes);
            bt.max_n = std::max<uint64_t>(bt.max_n, J.in.n);
        }
        out.push_back(bt);
    }
    return out;
}

// crop [-> voxel] of every cloud of one batch, on stream st
static int enqueue_chain(pcp_ctx *ctx, const Batch &bt, uint32_t *res, hipStream_t st,
                         float4 *emit = nullptr) {
    const unsigned k = (unsigned)bt.k;
    {
        ProfScope ps(ctx, PCP_K_CROP, st);
        if (bt.max_nb) {
            hipLaunchKernelGGL(k_crop_tile<false>, dim3(bt.max_nb, k), dim3(kCT), 0, st, bt.jb,
                               res);
            PCP_CHECK_LAUNCH(ctx);
        }
        hipLaunchKernelGGL(k_vox_params, dim3(1, k), dim3(kFT), 0, st, bt.jb, res,
                           res + kMaxClouds);
        PCP_CHECK_LAUNCH(ctx);
        if (bt.max_nb) {
            hipLaunchKernelGGL(k_compact_keys, dim3(bt.max_nb, k), dim3(kFT), 0, st, bt.jb);
            PCP_CHECK_LAUNCH(ctx);
        }
    }
    if (bt.max_passes > 0) {
        ProfScope ps(ctx, PCP_K_VOXEL, st);
        // sort-tile kernels: LDS admits 8192 / kSortTile blocks per CU; the clouds share the CUs
        const unsigned per_cu = (unsigned)std::max(1, 8192 / kSortTile);
        const unsigned gx = std::max(1u, std::min<unsigned>(
                                             bt.max_nt, per_cu * (unsigned)std::max(ctx->num_cus, 1) / k));
        for (int pass = 0; pass < bt.max_passes; ++pass) {
            hipLaunchKernelGGL(k_radix_hist, dim3(gx, k), dim3(kST), 0, st, bt.jb, pass);
            PCP_CHECK_LAUNCH(ctx);
            hipLaunchKernelGGL(k_radix_scatter, dim3(gx, k), dim3(kST), 0, st, bt.jb, pass);
            PCP_CHECK_LAUNCH(ctx);
        }
        hipLaunchKernelGGL(k_seg_count, dim3(gx, k), dim3(kST), 0, st, bt.jb);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_seg_centroid, dim3(gx, k), dim3(kST), 0, st, bt.jb, res, emit);
        PCP_CHECK_LAUNCH(ctx);
    }
    return PCP_OK;
}

// the fast chain of one batch whose clouds all certainly voxelise (make_job set J.fast): keyed
// crop -> digit-0 group counts -> pass 0 from the crop tiles -> passes 1.. -> voxels -> the
// centroids emitted as merged records.  No k_vox_params / k_compact_keys and their passes.
static int enqueue_fast(pcp_ctx *ctx, const Batch &bt, uint32_t *res, hipStream_t st,
                        float4 *emit) {
    const unsigned k = (unsigned)bt.k;
    uint32_t max_ng = 0;
    for (int i = 0; i < bt.k; ++i) max_ng = std::max(max_ng, bt.jb.j[i].ng);
    {
        ProfScope ps(ctx, PCP_K_CROP, st);
        hipLaunchKernelGGL(k_crop_tile<true>, dim3(std::max(bt.max_nb, 1u), k), dim3(kCT), 0, st,
                           bt.jb, res);
        PCP_CHECK_LAUNCH(ctx);
    }
    ProfScope ps(ctx, PCP_K_VOXEL, st);
    hipLaunchKernelGGL(k_hist0, dim3(std::max(max_ng, 1u), k), dim3(kST), 0, st, bt.jb);
    PCP_CHECK_LAUNCH(ctx);
    const unsigned per_cu = (unsigned)std::max(1, 8192 / kSortTile);
    const unsigned cap = per_cu * (unsigned)std::max(ctx->num_cus, 1) / k;
    const unsigned g0 = std::max(1u, std::min<unsigned>(max_ng, cap));
    hipLaunchKernelGGL(k_radix_scatter0, dim3(g0, k), dim3(kST), 0, st, bt.jb);
    PCP_CHECK_LAUNCH(ctx);
    const unsigned gx = std::max(1u, std::min<unsigned>(bt.max_nt, cap));
    for (int pass = 1; pass < bt.max_passes; ++pass) {
        hipLaunchKernelGGL(k_radix_hist, dim3(gx, k), dim3(kST), 0, st, bt.jb, pass);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_radix_scatter, dim3(gx, k), dim3(kST), 0, st, bt.jb, pass);
        PCP_CHECK_LAUNCH(ctx);
    }
    hipLaunchKernelGGL(k_seg_count, dim3(gx, k), dim3(kST), 0, st, bt.jb);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_seg_centroid, dim3(gx, k), dim3(kST), 0, st, bt.jb, res, emit);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

// the bucket chain of one batch whose clouds all certainly voxelise (bucket_geometry): crop ->
// k_bk_group -> k_bk_sort -> k_bk_emit (emit: the centroids as merged records)
static int enqueue_bucket(pcp_ctx *ctx, const Batch &bt, uint32_t *res, hipStream_t st,
                          float4 *emit) {
    const unsigned k = (unsigned)bt.k;
    uint32_t max_ng = 0, nseq = 0;
    for (int i = 0; i < bt.k; ++i) {
        max_ng = std::max(max_ng, bt.jb.j[i].ng);
        nseq += bt.jb.j[i].nbkcap;
    }
    if (ctx->bk_stat.cap < ((size_t)kBkChunkOff + kBatch * kBkMax / 64) * 8)   // bucket_geometry
        return set_err(ctx, PCP_E_STATE, "bucket chain: bucket words not allocated");
    uint2 *bkv = ctx->bk_stat.as<uint2>();
    {
        ProfScope ps(ctx, PCP_K_CROP, st);
        hipLaunchKernelGGL(k_crop_tile<false>, dim3(std::max(bt.max_nb, 1u), k), dim3(kCT), 0, st,
                           bt.jb, res);
        PCP_CHECK_LAUNCH(ctx);
    }
    ProfScope ps(ctx, PCP_K_VOXEL, st);
    hipLaunchKernelGGL(k_bk_group, dim3(std::max(max_ng, 1u), k), dim3(kBkT), 0, st, bt.jb, res,
                       bkv);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_bk_sort, dim3(std::max(nseq, 1u)), dim3(kBkT3), 0, st, bt.jb, (int)k,
                       res, bkv, emit ? 0 : 1);
    PCP_CHECK_LAUNCH(ctx);
    hipLaunchKernelGGL(k_bk_emit, dim3(std::max(nseq, 1u)), dim3(kBkTE), 0, st, bt.jb, (int)k, res,
                       emit, bkv);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

// transform + colour + concat of one batch (after every batch's chain: offsets need all counts)
static int enqueue_emit(pcp_ctx *ctx, const Batch &bt, const uint32_t *res, float4 *out,
                        hipStream_t st) {
    if (!bt.max_n) return PCP_OK;
    ProfScope ps(ctx, PCP_K_TRANSFORM, st);
    const unsigned g = (unsigned)std::min<uint64_t>((bt.max_n + kFT - 1) / kFT, 2048);
    hipLaunchKernelGGL(k_emit_rgb, dim3(g, (unsigned)bt.k), dim3(kFT), 0, st, bt.jb, res, out);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

// every cloud of a one-batch call certainly voxelised: a non-empty input and a finite crop box
// whose voxel keys fit 31 bits (then PCL's int32 guard cannot fire on the cropped points'
// smaller bbox) -- the centroid kernel can emit the merged records itself
static bool emit_in_centroid(const std::vector<Batch> &bts) {
    if (bts.size() != 1) return false;
    const Batch &bt = bts[0];
    for (int i = 0; i < bt.k; ++i) {
        const CloudJob &J = bt.jb.j[i];
        if (J.in.n == 0 || !(J.leaf > 0.0f) || J.passes <= 0 ||
            J.passes * kDigitBits > 31 + kDigitBits - 1)
            return false;
        const Box &b = J.box;
        const double lo[3] = {b.x0, b.y0, b.z0}, hi[3] = {b.x1, b.y1, b.z1};
        double nv = 1.0;
        for (int a = 0; a < 3; ++a) {
            if (!std::isfinite(lo[a]) || !std::isfinite(hi[a])) return false;
            nv *= std::floor((hi[a] - lo[a]) / (double)J.leaf) + 3.0;
        }
        if (!(nv < 2147483647.0)) return false;
    }
    return true;
}

static bool all_bucket(const std::vector<Batch> &bts) {
    if (bts.size() != 1 || bts[0].k == 0) return false;
    for (int i = 0; i < bts[0].k; ++i)
        if (!bts[0].jb.j[i].bk) return false;
    return true;
}

static int enqueue_all(pcp_ctx *ctx, const std::vector<Batch> &bts, uint32_t *res,
                       float4 *emit_out, hipStream_t st) {
    if (all_bucket(bts)) return enqueue_bucket(ctx, bts[0], res, st, emit_out);
    if (!emit_out && bts.size() == 1) {   // pcp_crop_voxel's fast chain (run_single)
        bool fast = bts[0].k > 0;
        for (int i = 0; i < bts[0].k; ++i) fast = fast && bts[0].jb.j[i].fast;
        if (fast) return enqueue_fast(ctx, bts[0], res, st, nullptr);
    }
    if (emit_out && emit_in_centroid(bts)) {
        bool fast = true;
        for (int i = 0; i < bts[0].k; ++i) fast = fast && bts[0].jb.j[i].fast;
        return fast ? enqueue_fast(ctx, bts[0], res, st, emit_out)
                    : enqueue_chain(ctx, bts[0], res, st, emit_out);
    }
    for (const Batch &bt : bts) {
        int rc = enqueue_chain(ctx, bt, res, st);
        if (rc) return rc;
    }
    if (emit_out)
        for (const Batch &bt : bts) {
            int rc = enqueue_emit(ctx, bt, res, emit_out, st);
            if (rc) return rc;
        }
    return PCP_OK;
}

static int stage_cloud(pcp_ctx *ctx, const pcp_cloud_view &v, bool device_in, DevBuf &buf,
                       size_t off, CloudIn &c) {
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
    unsigned char *dst = buf.as<unsigned char>() + off;
    // message-sized clouds through the pinned ring (no wait on the stream), C3-sized ones
    // straight from pageable memory (the link, not the wait, sets their rate)
    if (int rc = upload_async(ctx, dst, v.data, bytes, ctx->stream)) return rc;
    c.raw = dst;
    return PCP_OK;
}

struct ResultInfo {
    uint32_t n;          // result points
    uint32_t m;          // points after the crop
    uint32_t overflow;
};

static int read_results(pcp_ctx *ctx, const uint32_t *res_d, int k, ResultInfo *ri,
                        bool landed = false, uint32_t *redo = nullptr) {
    // pinned landing buffer: the per-frame size readback is one small DMA, no staging copy;
    // landed: the kernels stored the sizes in pinned memory themselves (res_d is host memory)
    uint32_t *buf;
    if (landed) {
        buf = const_cast<uint32_t *>(res_d);
    } else {
        PCP_HIP(ctx, ctx->res_host.ensure(kResWords * sizeof(uint32_t)));
        buf = ctx->res_host.as<uint32_t>();
        PCP_HIP(ctx, hipMemcpyAsync(buf, res_d, kResWords * sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, ctx->stream));
    }
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    for (int i = 0; i < k; ++i) {
        ri[i].n = buf[i];
        ri[i].m = buf[kMaxClouds + 2 * i];
        ri[i].overflow = buf[kMaxClouds + 2 * i + 1];
    }
    if (redo) *redo = buf[3 * kMaxClouds];
    return PCP_OK;
}

// one host cloud through crop [-> voxel] (slot 0); results stay in ctx->fbuf[0]
// fast_ok: the caller wants the centroids only (pcp_crop_voxel) -- a finite box then takes the
// fast chain, whose centroid kernel stores the voxels and the result sizes straight into
// pinned memory (J.out4 is then HOST memory): one round trip for the call
static int run_single(pcp_ctx *ctx, const pcp_cloud_view *in, const Box &b, float leaf,
                      bool want_idx, CloudJob &J, ResultInfo &ri, bool fast_ok = false) {
    VoxParams *vp;
    uint32_t *res;
    int rc = ensure_misc(ctx, vp, res);
    if (rc) return rc;
    if (ctx->fbuf.empty()) ctx->fbuf.resize(1);
    CloudIn c;
    // a message-sized cloud on the fast chain: read in place from the pinned ring (no DMA)
    const uint64_t in_bytes = in->n * (uint64_t)in->point_step;
    const bool zc = fast_ok && ctx->zc_in && ctx->fm_fast && in_bytes <= kPinDirectMax;
    if (zc) {
        if ((rc = stage_cloud(ctx, *in, true, ctx->f_in, 0, c))) return rc;   // fields only
        const HostPiece pc{0, in->data, in_bytes};
        const void *dv = nullptr;
        if ((rc = pin_stage(ctx, &pc, 1, in_bytes, &dv))) return rc;
        c.raw = static_cast<const unsigned char *>(dv);
    } else {
        PCP_HIP(ctx, ctx->f_in.ensure(in_bytes + 256));
        if ((rc = stage_cloud(ctx, *in, false, ctx->f_in, 0, c))) return rc;
    }
    std::vector<CloudJob> jobs(1);
    if ((rc = make_job(ctx, 0, c, b, leaf, want_idx, Rigid{}, vp, jobs[0]))) return rc;
    // the bucket chain (PCP_FM_FAST 2), else the LSD fast chain; a bucket chain that set its redo
    // flag runs again on the LSD chain (the input stays where it was staged until then)
    for (int mode = ctx->fm_fast; fast_ok && !want_idx && mode > 0; --mode) {
        CloudJob F = jobs[0];
        const bool geo = mode == 2 ? bucket_geometry(ctx, 0, F) : fast_geometry(ctx, 0, F);
        if (!geo) continue;
        const uint64_t ncap = c.n ? c.n : 1;
        const size_t res_b = align256(kResWords * sizeof(uint32_t));
        PCP_HIP(ctx, ctx->cv_host.ensure(res_b + (ncap + 1) * sizeof(float4) + (2 * ncap + 8) * 4 + 256));
        uint32_t *res_h = ctx->cv_host.as<uint32_t>();
        F.out4 = reinterpret_cast<float4 *>(ctx->cv_host.as<char>() + res_b);
        F.vidx = reinterpret_cast<uint32_t *>(F.out4 + ncap + 1);
        F.vcnt = F.vidx + ncap + 1;
        std::vector<CloudJob> fj(1, F);
        if ((rc = enqueue_all(ctx, batches_of(fj), res_h, nullptr, ctx->stream))) return rc;
        uint32_t redo = 0;
        if ((rc = read_results(ctx, res_h, 1, &ri, true, &redo))) return rc;
        if (mode == 2 && redo) {
            prof_count(ctx, PCP_K_VOXEL_REDO);
            continue;
        }
        if (zc) pin_release(ctx, ctx->stream);
        J = F;
        return PCP_OK;
    }
    if ((rc = enqueue_all(ctx, batches_of(jobs), res, nullptr, ctx->stream))) return rc;
    if (zc) pin_release(ctx, ctx->stream);
    J = jobs[0];
    return read_results(ctx, res, 1, &ri);
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
    const Box b{box[0], box[1], box[2], box[3], box[4], box[5]};
    CloudJob J;
    ResultInfo ri;
    if ((rc = run_single(ctx, in, b, 0.0f, kept_idx != nullptr, J, ri))) return rc;
    *n_kept = ri.m;
    if ((kept_idx || out_xyz16) && ri.m > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_crop_box: need %u, cap %llu", ri.m,
                       (unsigned long long)cap);
    }
    if (kept_idx && ri.m)
        PCP_HIP(ctx, hipMemcpyAsync(kept_idx, J.kept_idx, (size_t)ri.m * 4, hipMemcpyDeviceToHost,
                                    ctx->stream));
    if (out_xyz16 && ri.m)
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, J.xyz, (size_t)ri.m * 16, hipMemcpyDeviceToHost,
                                    ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

static int crop_voxel_impl(pcp_ctx *ctx, const pcp_cloud_view *in, const Box &b, float leaf,
                           float *out_xyz16, uint32_t *voxel_idx, uint32_t *voxel_count,
                           uint64_t cap, uint64_t *n_out, uint64_t *n_cropped,
                           int32_t *passthrough) {
    CloudJob J;
    ResultInfo ri;
    const bool fast_ok = voxel_idx == nullptr && voxel_count == nullptr;
    int rc = run_single(ctx, in, b, leaf, false, J, ri, fast_ok);
    if (rc) return rc;
    const bool vox = leaf > 0.0f && !ri.overflow;
    if (passthrough) *passthrough = (leaf > 0.0f && ri.overflow) ? 1 : 0;
    if (n_cropped) *n_cropped = ri.m;
    *n_out = ri.n;
    if (ri.n > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "voxel output needs %u points, cap %llu", ri.n,
                       (unsigned long long)cap);
    }
    if (J.fast || J.bk) {   // the fast chains (LSD or bucket) stored the voxels straight into
                            // pinned memory (synchronised by read_results): a host copy only
        if (ri.n) host_copy(ctx, out_xyz16, J.out4, (size_t)ri.n * 16);
        prof_resolve(ctx);
        return PCP_OK;
    }
    if (ri.n) {
        const void *src = vox ? (const void *)J.out4 : (const void *)J.xyz;
        PCP_HIP(ctx, hipMemcpyAsync(out_xyz16, src, (size_t)ri.n * 16, hipMemcpyDeviceToHost,
                                    ctx->stream));
        if (vox && voxel_idx)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_idx, J.vidx, (size_t)ri.n * 4,
                                        hipMemcpyDeviceToHost, ctx->stream));
        if (vox && voxel_count)
            PCP_HIP(ctx, hipMemcpyAsync(voxel_count, J.vcnt, (size_t)ri.n * 4,
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
    std::vector<size_t> soff(k + 1, 0);
    for (int i = 0; i < k; ++i)
        soff[i + 1] = soff[i] + align256(clouds[i].n * (uint64_t)clouds[i].point_step);
    if (ctx->zc_in && k <= kXfMax && soff[k] <= kPinDirectMax) {
        // message-sized: every cloud read in place from one pinned slot, one launch, the
        // records stored straight into pinned memory -- no DMA either way, one synchronisation
        std::vector<HostPiece> pc(k);
        for (int i = 0; i < k; ++i)
            pc[i] = HostPiece{soff[i], clouds[i].data, clouds[i].n * (uint64_t)clouds[i].point_step};
        ctx->fm_land_valid = false;   // (tc_host rewritten)
        PCP_HIP(ctx, ctx->tc_host.ensure(total * 32 + 256));
        float4 *o = ctx->tc_host.as<float4>();
        const void *dv = nullptr;
        if (int rc = pin_stage(ctx, pc.data(), k, soff[k], &dv)) return rc;
        XformBatch B{};
        B.k = k;
        uint64_t base = 0;
        uint32_t tiles = 0;
        for (int i = 0; i < k; ++i) {
            CloudIn &c = B.c[i];
            c.n = clouds[i].n;
            c.step = clouds[i].point_step;
            c.ox = clouds[i].off_x;
            c.oy = clouds[i].off_y;
            c.oz = clouds[i].off_z;
            c.raw = static_cast<const unsigned char *>(dv) + soff[i];
            B.r[i] = make_rigid(tf[i], rgb + 3 * i);
            B.base[i] = base;
            B.tile0[i] = tiles;
            base += c.n;
            tiles += (uint32_t)((c.n + kFT - 1) / kFT);
        }
        B.tile0[k] = tiles;
        {
            ProfScope ps(ctx, PCP_K_TRANSFORM);
            hipLaunchKernelGGL(k_xform_batch, dim3(tiles), dim3(kFT), 0, ctx->stream, B, o);
            PCP_CHECK_LAUNCH(ctx);
        }
        pin_release(ctx, ctx->stream);
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        host_copy(ctx, out, o, total * 32);
        prof_resolve(ctx);
        return PCP_OK;
    }
    PCP_HIP(ctx, ctx->out_d.ensure(total * 32));
    float4 *o = ctx->out_d.as<float4>();
    // every cloud staged in its own region of f_in: all uploads and launches in flight, one
    // synchronisation for the call
    PCP_HIP(ctx, ctx->f_in.ensure(soff[k] + 256));
    uint64_t base = 0;
    for (int i = 0; i < k; ++i) {
        if (clouds[i].n == 0) continue;
        CloudIn c;
        int rc = stage_cloud(ctx, clouds[i], false, ctx->f_in, soff[i], c);
        if (rc) return rc;
        const Rigid r = make_rigid(tf[i], rgb + 3 * i);
        {
            ProfScope ps(ctx, PCP_K_TRANSFORM);
            hipLaunchKernelGGL(k_xform_raw, dim3((unsigned)((c.n + kFT - 1) / kFT)), dim3(kFT), 0,
                               ctx->stream, c, r, o + 2 * base);
            PCP_CHECK_LAUNCH(ctx);
        }
        base += c.n;
    }
    PCP_HIP(ctx, hipMemcpyAsync(out, o, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

// key of a captured filter_merge graph: everything baked into its nodes and its job table
static std::vector<uint8_t> fm_key(int k, const pcp_cloud_view *clouds, const double *boxes,
                                   float leaf, const pcp_rigid *tf, const uint8_t *rgb,
                                   const void *out, uint64_t cap,
                                   const std::vector<CloudJob> &jobs) {
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
    put(jobs.data(), jobs.size() * sizeof(CloudJob));   // every scratch pointer, the results
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
    *n_out = 0;
    if (k == 0) return PCP_OK;
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
    VoxParams *vp;
    uint32_t *res;
    int rc = ensure_misc(ctx, vp, res);
    if (rc) return rc;
    // staging (host input): one region per cloud
    std::vector<size_t> soff(k + 1, 0);
    for (int i = 0; i < k; ++i)
        soff[i + 1] = soff[i] + (dev_in ? 0 : align256(clouds[i].n * clouds[i].point_step));
    if (!dev_in) PCP_HIP(ctx, ctx->f_in.ensure(soff[k] + 256));
    if ((int)ctx->fbuf.size() < k) ctx->fbuf.resize(k);
    std::vector<CloudJob> jobs(k);
    for (int i = 0; i < k; ++i) {
        CloudIn c;
        if ((rc = stage_cloud(ctx, clouds[i], dev_in, ctx->f_in, soff[i], c))) return rc;
        const double *bx = boxes + 6 * i;
        const Box b{bx[0], bx[1], bx[2], bx[3], bx[4], bx[5]};
        if ((rc = make_job(ctx, i, c, b, leaf, false, make_rigid(tf[i], rgb + 3 * i), vp, jobs[i])))
            return rc;
    }
    std::vector<Batch> bts = batches_of(jobs);
    // the emit needs the sizes first when the output might not fit (device output only)
    const bool emit_now = !(dev_out && upper > cap);
    // every cloud certainly voxelises: the fast chain (PCP_FM_FAST=0: the general chain)
    // (2: the bucket chain, the LSD fast chain when a bucket chain frame has to be redone)
    const std::vector<CloudJob> plain = jobs;
    auto lsd_jobs = [&]() {
        std::vector<CloudJob> fj = plain;
        bool all = true;
        for (int i = 0; i < k && all; ++i) all = fast_geometry(ctx, i, fj[i], k);
        return all ? fj : plain;
    };
    bool bucket = false;
    if (emit_now && ctx->fm_fast && emit_in_centroid(bts)) {
        std::vector<CloudJob> fj = plain;
        bucket = ctx->fm_fast == 2;
        for (int i = 0; i < k && bucket; ++i) bucket = bucket_geometry(ctx, i, fj[i], k);
        jobs = bucket ? fj : lsd_jobs();
        bts = batches_of(jobs);
    }
    const bool graphable = dev_in && dev_out && emit_now && ctx->use_graphs;
    // the centroid kernel emits the records itself: no kernel reads the sizes back, so they
    // are stored straight into pinned memory (no D2H copy per frame; PCP_FM_HOST_OUT)
    const bool landed = emit_now && ctx->fm_host_out && emit_in_centroid(bts);
    if (landed) {
        PCP_HIP(ctx, ctx->fm_res_host.ensure(kResWords * sizeof(uint32_t)));
        res = ctx->fm_res_host.as<uint32_t>();
    }
    if (graphable) {
        std::vector<uint8_t> key = fm_key(k, clouds, boxes, leaf, tf, rgb, out, cap, jobs);
        key.insert(key.end(), reinterpret_cast<const uint8_t *>(&res),
                   reinterpret_cast<const uint8_t *>(&res) + sizeof(res));
        if (!ctx->fm_exec || key != ctx->fm_key) {
            if (ctx->fm_exec) (void)hipGraphExecDestroy(ctx->fm_exec);
            if (ctx->fm_graph) (void)hipGraphDestroy(ctx->fm_graph);
            ctx->fm_exec = nullptr;
            ctx->fm_graph = nullptr;
            ctx->fm_key.clear();
            PCP_HIP(ctx, hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
            ctx->capturing = true;
            rc = enqueue_all(ctx, bts, res, obuf, ctx->stream);
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
        rc = enqueue_all(ctx, bts, res, emit_now ? obuf : nullptr, ctx->stream);
        if (rc) return rc;
    }
    std::vector<ResultInfo> ri(k);
    uint32_t redo = 0;
    if ((rc = read_results(ctx, res, k, ri.data(), landed, &redo))) return rc;
    if (bucket && redo) {   // a bucket past its LDS capacity: the frame again on the LSD chain
        prof_count(ctx, PCP_K_VOXEL_REDO);
        jobs = lsd_jobs();
        bts = batches_of(jobs);
        {
            ProfScope ps(ctx, PCP_K_FILTER_MERGE);
            if ((rc = enqueue_all(ctx, bts, res, obuf, ctx->stream))) return rc;
        }
        if ((rc = read_results(ctx, res, k, ri.data(), landed))) return rc;
    }
    uint64_t total = 0;
    for (int i = 0; i < k; ++i) {
        const uint64_t ni = clouds[i].n ? ri[i].n : 0;
        if (n_per_cloud) n_per_cloud[i] = ni;
        total += ni;
    }
    *n_out = total;
    if (total > cap) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_filter_merge: need %llu, cap %llu",
                       (unsigned long long)total, (unsigned long long)cap);
    }
    if (!emit_now && total)   // deferred until the size was known to fit
        for (const Batch &bt : bts)
            if ((rc = enqueue_emit(ctx, bt, res, obuf, ctx->stream))) return rc;
    if (!dev_out && total)
        PCP_HIP(ctx, hipMemcpyAsync(out, obuf, total * 32, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

// The launch file's filter node (both sensors) and merger node composed in one process
// (the C5 chain): each cloud cropped + voxelised, its centroids in its own frame
// (the /filtered_points message, PointXYZ 16-B stride) AND the concatenated transformed + coloured
// records (the merged PointXYZRGB message), one batch of launches and ONE synchronisation.  The
// clouds are read in place from the pinned ring, the results are stored by the kernels into
// pinned memory (host output only).
int pcp_filter_merge_nodes(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds,
                           const double *boxes, float leaf, const pcp_rigid *tf,
                           const uint8_t *rgb, void *out, uint64_t cap, uint64_t *n_out,
                           uint64_t *n_per_cloud, float *const *filtered, uint64_t *n_cropped) {
    if (!ctx) return PCP_E_INVALID;
    if (k < 0 || k > kBatch || (k && (!clouds || !boxes || !tf || !rgb || !filtered)) || !n_out)
        return set_err(ctx, PCP_E_INVALID, "pcp_filter_merge_nodes: bad argument");
    uint64_t upper = 0, in_bytes = 0;
    for (int i = 0; i < k; ++i) {
        int rc = check_view(ctx, &clouds[i], "pcp_filter_merge_nodes");
        if (rc) return rc;
        upper += clouds[i].n;
        in_bytes += clouds[i].n * (uint64_t)clouds[i].point_step;
    }
    *n_out = 0;
    if (k == 0) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    VoxParams *vp;
    uint32_t *res;
    int rc = ensure_misc(ctx, vp, res);
    if (rc) return rc;
    if ((int)ctx->fbuf.size() < k) ctx->fbuf.resize(k);
    // inputs: one pinned-ring slot holding every cloud (message-sized), else DMA'd staging
    const bool zc = ctx->zc_in && in_bytes <= kPinDirectMax;
    std::vector<size_t> soff(k + 1, 0);
    for (int i = 0; i < k; ++i)
        soff[i + 1] = soff[i] + align256(clouds[i].n * clouds[i].point_step);
    std::vector<CloudIn> cin(k);
    if (zc) {
        std::vector<HostPiece> pc;
        for (int i = 0; i < k; ++i) {
            if ((rc = stage_cloud(ctx, clouds[i], true, ctx->f_in, 0, cin[i]))) return rc;   // fields
            if (clouds[i].n) pc.push_back(HostPiece{soff[i], clouds[i].data,
                                                    clouds[i].n * (uint64_t)clouds[i].point_step});
        }
        const void *dv = nullptr;
        if (!pc.empty()) {
            if ((rc = pin_stage(ctx, pc.data(), (int)pc.size(), soff[k], &dv))) return rc;
            for (int i = 0; i < k; ++i)
                if (clouds[i].n) cin[i].raw = static_cast<const unsigned char *>(dv) + soff[i];
        }
    } else {
        PCP_HIP(ctx, ctx->f_in.ensure(soff[k] + 256));
        for (int i = 0; i < k; ++i)
            if ((rc = stage_cloud(ctx, clouds[i], false, ctx->f_in, soff[i], cin[i]))) return rc;
    }
    std::vector<CloudJob> jobs(k);
    for (int i = 0; i < k; ++i) {
        const double *bx = boxes + 6 * i;
        const Box b{bx[0], bx[1], bx[2], bx[3], bx[4], bx[5]};
        if ((rc = make_job(ctx, i, cin[i], b, leaf, false, make_rigid(tf[i], rgb + 3 * i), vp,
                           jobs[i])))
            return rc;
    }
    // landing (pinned): [result words | merged records | each cloud's centroids]
    ctx->fm_land_valid = false;
    const size_t res_b = align256(kResWords * sizeof(uint32_t));
    const size_t mrg_b = align256((upper + 1) * 32);
    std::vector<size_t> koff(k + 1, 0);
    for (int i = 0; i < k; ++i) koff[i + 1] = koff[i] + align256((clouds[i].n + 1) * 16);
    PCP_HIP(ctx, ctx->tc_host.ensure(res_b + mrg_b + koff[k] + 256));
    char *land = ctx->tc_host.as<char>();
    uint32_t *res_h = reinterpret_cast<uint32_t *>(land);
    float4 *mrg = reinterpret_cast<float4 *>(land + res_b);
    auto keep = [&](int i) { return reinterpret_cast<float4 *>(land + res_b + mrg_b + koff[i]); };
    std::vector<ResultInfo> ri(k);
    bool done = false;
    // the bucket chain with the emit writing both outputs (every cloud certainly voxelises)
    std::vector<Batch> bts = batches_of(jobs);
    if (ctx->fm_fast == 2 && emit_in_centroid(bts)) {
        std::vector<CloudJob> fj = jobs;
        bool bucket = true;
        for (int i = 0; i < k && bucket; ++i) bucket = bucket_geometry(ctx, i, fj[i], k);
        if (bucket) {
            for (int i = 0; i < k; ++i) fj[i].keep16 = keep(i);
            {
                ProfScope ps(ctx, PCP_K_FILTER_MERGE);
                if ((rc = enqueue_all(ctx, batches_of(fj), res_h, mrg, ctx->stream))) return rc;
            }
            uint32_t redo = 0;
            if ((rc = read_results(ctx, res_h, k, ri.data(), true, &redo))) return rc;
            if (redo) prof_count(ctx, PCP_K_VOXEL_REDO);
            done = !redo;
        }
    }
    if (!done) {   // the general chain: each cloud's result, then the transform + concat
        std::vector<CloudJob> gj = jobs;
        for (int i = 0; i < k; ++i) gj[i].bk = 0;
        bts = batches_of(gj);
        {
            ProfScope ps(ctx, PCP_K_FILTER_MERGE);
            for (const Batch &bt : bts)
                if ((rc = enqueue_chain(ctx, bt, res, ctx->stream))) return rc;
            for (const Batch &bt : bts)
                if ((rc = enqueue_emit(ctx, bt, res, mrg, ctx->stream))) return rc;
        }
        if ((rc = read_results(ctx, res, k, ri.data()))) return rc;
        // each cloud's result (centroids, or the cropped points of a passthrough cloud) down
        for (int i = 0; i < k; ++i) {
            if (!ri[i].n) continue;
            VoxParams v;
            PCP_HIP(ctx, hipMemcpyAsync(&v, gj[i].vp, sizeof(v), hipMemcpyDeviceToHost, ctx->stream));
            PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
            const float4 *src = (v.do_voxel && !v.overflow) ? gj[i].out4 : gj[i].xyz;
            PCP_HIP(ctx, hipMemcpyAsync(keep(i), src, (size_t)ri[i].n * 16, hipMemcpyDeviceToHost,
                                        ctx->stream));
        }
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (zc) pin_release(ctx, ctx->stream);
    uint64_t total = 0;
    for (int i = 0; i < k; ++i) {
        const uint64_t ni = clouds[i].n ? ri[i].n : 0;
        if (n_per_cloud) n_per_cloud[i] = ni;
        if (n_cropped) n_cropped[i] = clouds[i].n ? ri[i].m : 0;
        total += ni;
    }
    *n_out = total;
    prof_resolve(ctx);
    if (out && total > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_filter_merge_nodes: need %llu, cap %llu",
                       (unsigned long long)total, (unsigned long long)cap);
    if (total && out) host_copy(ctx, out, mrg, total * 32);
    for (int i = 0; i < k; ++i)
        if (clouds[i].n && ri[i].n && filtered[i]) host_copy(ctx, filtered[i], keep(i), (size_t)ri[i].n * 16);
    ctx->fm_land_merged = mrg;
    ctx->fm_land_filtered.resize(k);
    for (int i = 0; i < k; ++i) ctx->fm_land_filtered[i] = reinterpret_cast<const float *>(keep(i));
    ctx->fm_land_k = k;
    ctx->fm_land_valid = true;
    return PCP_OK;
}

int pcp_filter_merge_landed(pcp_ctx *ctx, int k, const void **merged, const float **filtered) {
    if (!ctx) return PCP_E_INVALID;
    if (!ctx->fm_land_valid || k != ctx->fm_land_k)
        return set_err(ctx, PCP_E_STATE, "pcp_filter_merge_landed: no pcp_filter_merge_nodes "
                                         "result of %d clouds in place", k);
    if (merged) *merged = ctx->fm_land_merged;
    if (filtered)
        for (int i = 0; i < k; ++i) filtered[i] = ctx->fm_land_filtered[i];
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
