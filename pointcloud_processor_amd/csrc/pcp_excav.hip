// pcp_excav.hip -- virtual_lidar.cpp's excavation-area setup on gfx950:
// excavationAreaCallback (:164-178) -> computeTerrainNormals (:209-234) and
// generateExcavationGrid3D (:236-287) with isPointNearExcavation (:289-299) and
// computeCellSurfaceNormal (:301-340).  The resulting cells become the context's scoring
// cells (what pcp_set_cells would hold).
//
//  area normals : one block per area point; the 1.5 m neighbours (FLANN predicate) of the
//                 point's stencil in a uniform grid sized for r = 1.5; shifted second moments in
//                 double, covariance rounded to float, pcl::eigen33 restated in float,
//                 viewpoint (0,0,0) flip, then the reference's flip to normal_z >= 0
//  cell lattice : one thread per (i, j, k) lattice point, exact radius test (r = 1.5 res) on a
//                 grid sized for that radius; one block compacts the hits in loop order
//  cell normals : one block per cell; double-double sums of the neighbours' finite normals
//                 (the reference's sequential double sum when that sum is exact, which it is
//                 for these magnitudes), normalised when the norm exceeds 1e-6
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>
#include <vector>

#include "pcp_internal.hpp"
#include "pcp_libm.h"
#include "pcp_stencil.hpp"

namespace pcp {

constexpr double kNormalRadius = 1.5;   // NORMAL_SEARCH_RADIUS (virtual_lidar.cpp:110)
constexpr int kXT = 256;

// the 2x2x2 stencil of q as 4 contiguous point ranges [lo, hi) (rows of 2 adjacent x-cells)
__device__ __forceinline__ bool stencil_ranges(const GridView &g, float qx, float qy, float qz,
                                               uint32_t (&lo)[4], uint32_t (&hi)[4]) {
    uint32_t ix, iy, iz;
    if (!stencil_cell3_f(g, qx, qy, qz, ix, iy, iz)) return false;
    const uint32_t nx = (uint32_t)g.nx, nxy = nx * (uint32_t)g.ny;
    const uint32_t lin = ix + nx * iy + nxy * iz;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t row = lin + (r & 1) * nx + (r >> 1) * nxy;
        lo[r] = g.start[row];
        hi[r] = g.start[row + 2];
    }
    return true;
}

// ---- pcl::eigen33, smallest eigenvalue's eigenvector (float, as PCL's Scalar) ---------------
// Every libm call and every float division / square root as the reference's platform computes
// them (pcp_libm.h: glibc 2.35's atan2f / cosf / sinf restated, correctly rounded sqrt and
// division), so the same covariance gives the same normal bits as the oracle (glibc)
__device__ __forceinline__ void roots2(float b, float c, float r[3]) {
    r[0] = 0.0f;
    float d = (float)(b * b - 4.0 * c);
    if (d < 0.0f) d = 0.0f;
    const float sd = pcp_lm_sqrt(d);
    r[2] = 0.5f * (b + sd);
    r[1] = 0.5f * (b - sd);
}

__device__ __forceinline__ void roots3(const float m[3][3], float r[3]) {
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
    const float s_sqrt3 = pcp_lm_sqrt(3.0f);
    const float c2_over_3 = c2 * s_inv3;
    float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
    if (a_over_3 > 0.0f) a_over_3 = 0.0f;
    const float half_b = 0.5f * (c0 + c2_over_3 * (2.0f * c2_over_3 * c2_over_3 - c1));
    float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
    if (q > 0.0f) q = 0.0f;
    const float rho = pcp_lm_sqrt(-a_over_3);
    const float theta = pcp_atan2f(pcp_lm_sqrt(-q), half_b) * s_inv3;
    const float ct = pcp_cosf(theta), st = pcp_sinf(theta);
    r[0] = c2_over_3 + 2.0f * rho * ct;
    r[1] = c2_over_3 - rho * (ct + s_sqrt3 * st);
    r[2] = c2_over_3 - rho * (ct - s_sqrt3 * st);
    float t;
    if (r[0] >= r[1]) {
        t = r[0]; r[0] = r[1]; r[1] = t;
    }
    if (r[1] >= r[2]) {
        t = r[1]; r[1] = r[2]; r[2] = t;
        if (r[0] >= r[1]) {
            t = r[0]; r[0] = r[1]; r[1] = t;
        }
    }
    if (r[0] <= 0.0f) roots2(c2, c1, r);
}

__device__ __forceinline__ void cross3(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ void eigen33_min(const float cov[3][3], float ev[3]) {
    float scale = 0.0f;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) scale = fmaxf(scale, fabsf(cov[i][j]));
    if (scale <= FLT_MIN) scale = 1.0f;
    float m[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m[i][j] = pcp_lm_div(cov[i][j], scale);
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
    const float *v = v3;
    float l = l3;
    if (l1 >= l2 && l1 >= l3) {
        v = v1;
        l = l1;
    } else if (l2 >= l1 && l2 >= l3) {
        v = v2;
        l = l2;
    }
    const float s = pcp_lm_sqrt(l);
    for (int a = 0; a < 3; ++a) ev[a] = pcp_lm_div(v[a], s);
}

// the normal of one area point from its covariance: eigen33, flipNormalTowardsViewpoint with
// the viewpoint (0, 0, 0) (scalar PCL overload: ((vx nx + vy ny) + vz nz)), then the
// reference's flip to normal_z >= 0 (virtual_lidar.cpp:223-229)
__device__ __forceinline__ void normal_from_cov(const float cov[3][3], float qx, float qy,
                                                float qz, float *o) {
    float ev[3];
    eigen33_min(cov, ev);
    const float ct = (0.0f - qx) * ev[0] + (0.0f - qy) * ev[1] + (0.0f - qz) * ev[2];
    if (ct < 0.0f)
        for (int a = 0; a < 3; ++a) ev[a] = -ev[a];
    if (ev[2] < 0.0f)
        for (int a = 0; a < 3; ++a) ev[a] = -ev[a];
    o[0] = ev[0];
    o[1] = ev[1];
    o[2] = ev[2];
}

// double-double accumulation (TwoSum): exact sums of these float addends
struct DD {
    double hi, lo;
};
__device__ __forceinline__ void dd_add(DD &a, double x) {
    const double s = a.hi + x;
    const double bb = s - a.hi;
    const double err = (a.hi - (s - bb)) + (x - bb);
    a.hi = s;
    a.lo += err;
}
__device__ __forceinline__ DD dd_merge(DD a, DD b) {
    dd_add(a, b.hi);
    a.lo += b.lo;
    return a;
}

// computeTerrainNormals: block per point (sorted index order; .w = input index).  The shifted
// second moments are summed as 64-bit fixed point (each double term rounded once to a multiple
// of 2^-32, far below the float covariance's own rounding): integer sums are associative, so
// the result does not depend on the (atomic) order of the points in a cell or on the reduction
// tree -- deterministic run to run -- for fewer instructions than the double-double sums this
// replaced (|term| <= 2.25 m^2 within the 1.5 m radius: 9e8 neighbours fit in int64).
constexpr double kMomScale = 4294967296.0;   // 2^32
// round-to-nearest-even of t * 2^32 to an integer, as the bit pattern of 1.5 * 2^52 + that
// integer: one FMA instead of the emulated double -> int64 conversion.  |t * 2^32| < 2^51, so
// the sum stays in [2^52, 2^53) where the double's ulp is 1 and the bits are linear in the
// integer; the accumulated 1.5 * 2^52 terms come off once at the end (count * kMagicBits)
constexpr double kMagic = 6755399441055744.0;   // 1.5 * 2^52
constexpr unsigned long long kMagicBits = 0x4338000000000000ull;
__device__ __forceinline__ unsigned long long fx_bits(double t) {
    return (unsigned long long)__double_as_longlong(fma(t, kMomScale, kMagic));
}
// the raw input (the index holds its finite points only): the blocks past the index's points
// give the non-finite ones their NaN normal
struct RawIn {
    const unsigned char *raw;
    uint64_t n;
    uint32_t step, ox, oy, oz;
};
__global__ void __launch_bounds__(kXT) k_area_normals(GridView g, float r2, float *__restrict__ out,
                                                      RawIn in) {
    const uint32_t qi = blockIdx.x;
    if (qi >= g.n_pts) {
        const uint64_t i = (uint64_t)(qi - g.n_pts) * kXT + threadIdx.x;
        if (i >= in.n) return;
        const unsigned char *p = in.raw + i * in.step;
        const float x = *reinterpret_cast<const float *>(p + in.ox),
                    y = *reinterpret_cast<const float *>(p + in.oy),
                    z = *reinterpret_cast<const float *>(p + in.oz);
        if (!(isfinite(x) && isfinite(y) && isfinite(z)))
            out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = NAN;
        return;
    }
    const float4 q = g.pts[qi];
    const uint32_t orig = __float_as_uint(q.w);
    uint32_t lo[4], hi[4];
    unsigned long long acc[10];   // xx xy xz yy yz zz x y z (biased bits) count
    for (int a = 0; a < 10; ++a) acc[a] = 0;
    if (stencil_ranges(g, q.x, q.y, q.z, lo, hi)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            for (uint32_t k = lo[r] + threadIdx.x; k < hi[r]; k += kXT) {
                const P3 p = ld_p3(g.pts, k);
                if (!flann_within(q.x, q.y, q.z, p, r2)) continue;
                // shifted by K = the first (nearest) neighbour = the query point itself; the
                // products of two float-valued doubles are exact
                const double x = (double)(p.x - q.x), y = (double)(p.y - q.y),
                             z = (double)(p.z - q.z);
                acc[0] += fx_bits(x * x);
                acc[1] += fx_bits(x * y);
                acc[2] += fx_bits(x * z);
                acc[3] += fx_bits(y * y);
                acc[4] += fx_bits(y * z);
                acc[5] += fx_bits(z * z);
                acc[6] += fx_bits(x);
                acc[7] += fx_bits(y);
                acc[8] += fx_bits(z);
                acc[9] += 1;
            }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int a = 0; a < 10; ++a) acc[a] += __shfl_xor(acc[a], o, 64);
    __shared__ unsigned long long lds[10][kXT / 64];
    if (lane == 0)
        for (int a = 0; a < 10; ++a) lds[a][wid] = acc[a];
    __syncthreads();
    if (threadIdx.x != 0) return;
    double v[10];
    unsigned long long cnt = 0;
    for (int w = 0; w < kXT / 64; ++w) cnt += lds[9][w];
    for (int a = 0; a < 10; ++a) {
        unsigned long long t = lds[a][0];
        for (int w = 1; w < kXT / 64; ++w) t += lds[a][w];
        // modulo-2^64 sums: the bias comes off exactly
        v[a] = a == 9 ? (double)t : (double)(long long)(t - cnt * kMagicBits) / kMomScale;
    }
    float *o = out + 3 * (size_t)orig;
    if (v[9] < 3.0) {   // computePointNormal: < 3 neighbours -> NaN
        o[0] = o[1] = o[2] = NAN;
        return;
    }
    double acc2[9];
    for (int a = 0; a < 9; ++a) acc2[a] = v[a] / v[9];
    float cov[3][3];
    cov[0][0] = (float)(acc2[0] - acc2[6] * acc2[6]);
    cov[0][1] = (float)(acc2[1] - acc2[6] * acc2[7]);
    cov[0][2] = (float)(acc2[2] - acc2[6] * acc2[8]);
    cov[1][1] = (float)(acc2[3] - acc2[7] * acc2[7]);
    cov[1][2] = (float)(acc2[4] - acc2[7] * acc2[8]);
    cov[2][2] = (float)(acc2[5] - acc2[8] * acc2[8]);
    cov[1][0] = cov[0][1];
    cov[2][0] = cov[0][2];
    cov[2][1] = cov[1][2];
    normal_from_cov(cov, q.x, q.y, q.z, o);
}

// ---- the reference's neighbour order (the default path) --------------------------------------
// PCL sums each covariance in float, and each cell normal in double, over the radius search's
// result in FLANN's order: ascending (float distance, index) (RadiusResultSet, sorted = true;
// the oracle's radius_search).  Float sums depend on that order, so the default path builds the
// sorted neighbour list of every query and then sums it sequentially:
//  k_nb_lists : blocks loop over the queries: one pass over the stencil counts the points
//               within r (FLANN predicate) into 2,048 distance buckets of LDS (bucket =
//               (uint)(d * 2048 / r2): monotone in d, so buckets are ordered) and appends their
//               64-bit keys (distance bits << 32 | input index) to LDS; a block scan, the keys
//               grouped by bucket, each key placed at its bucket's start + its rank among the
//               bucket's keys; the list (input indices) goes to the block's own region of the
//               list buffer
//  k_nb_sums  : a block per QB queries; waves 1-3 gather the listed points (by input index)
//               64 steps at a time and form the summands (lane-parallel), wave 0 adds them in
//               list order, one lane per (query, summand) -- the only sequential part, ~1 add
//               per step.  The gathers of a chunk are issued one chunk ahead, its list entries
//               two chunks ahead.
//  k_cell_sums_exact : the cells' double sums in any order where an exponent bound makes
//               every order equal; the cells it leaves take k_nb_lists / k_nb_sums in order
#ifndef PCP_NB_BUCKETS
#define PCP_NB_BUCKETS 1792   // distance buckets of k_nb_lists (build knob, A/B; 7 per thread)
#endif
#ifndef PCP_NB_LDS
#define PCP_NB_LDS 4096       // keys sorted in LDS (build knob, A/B)
#endif
constexpr int kNbBuckets = PCP_NB_BUCKETS;
constexpr int kNbLds = PCP_NB_LDS;   // keys sorted in LDS (32 KB); longer lists sort in global memory
constexpr int kNbT = 256;
constexpr int kNbBlocks = 2048;        // k_nb_lists grid (blocks loop over the queries)
constexpr int kNbU = 8;                // k_nb_lists candidates in flight per thread

__device__ __forceinline__ uint32_t nb_wave_incl_scan(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// FLANN's L2 (acc = 0; acc += d0 d0; acc += d1 d1; acc += d2 d2, each op rounded; 0 + d0 d0
// is d0 d0 exactly).  x and y as one packed pair: v_pk_add / v_pk_mul round each half like the
// scalar ops, one instruction for two
typedef float nb_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float flann_d2(float qx, float qy, float qz, const float4 &p) {
    const nb_f2 q2 = {qx, qy}, p2 = {p.x, p.y};
    const nb_f2 d01 = q2 - p2;
    const nb_f2 s01 = d01 * d01;
    const float d2 = qz - p.z;
    float acc = s01.x + s01.y;
    acc = acc + d2 * d2;
    return acc;
}

// diagnostic build only (make stamps): per (block, query round) phase times of k_nb_lists and
// per block of k_nb_sums, s_memrealtime (100 MHz)
#ifdef PCP_STAMPS
constexpr int kNbStampBlocks = 2048, kNbStampQ = 4, kNbStampPh = 8;
__device__ unsigned long long g_nb_stamps[2][kNbStampBlocks * kNbStampQ * kNbStampPh];
#define NB_STAMP(k, q, ph)                                                                    \
    do {                                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < kNbStampBlocks && (q) < kNbStampQ)               \
            g_nb_stamps[k][(blockIdx.x * kNbStampQ + (q)) * kNbStampPh + (ph)] =              \
                __builtin_amdgcn_s_memrealtime();                                             \
    } while (0)
#else
#define NB_STAMP(k, q, ph) \
    do {                   \
    } while (0)
#endif

struct NbLists {
    uint32_t *list;                 // entries: input indices of the neighbours, sorted
    uint2 *meta;                    // per query: {base, m}
    uint32_t *need;                 // the largest words one block needed (zero before the launch)
    uint32_t *overflow;             // set when a list fit neither its block's region nor the pool
    uint32_t per_block;             // words of each block's region (block b: [b pb, (b + 1) pb))
    uint32_t *pool_cursor;          // the shared spill pool's cursor (zero before the launch)
    uint64_t pool_base, pool_words; // the pool: words [pool_base, pool_base + pool_words)
};

// the stencil's points of query q within r2, 4 loads in flight per thread: f(k, p, d)
template <class F>
__device__ __forceinline__ void nb_for_within(const GridView &g, const uint32_t (&lo)[4],
                                              const uint32_t (&hi)[4], float qx, float qy,
                                              float qz, float r2, F f) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
        for (uint32_t k0 = lo[r] + threadIdx.x; k0 < hi[r]; k0 += 4 * kNbT) {
            float4 p[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + (uint32_t)u * kNbT;
                p[u] = g.pts[k < hi[r] ? k : hi[r] - 1];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + (uint32_t)u * kNbT;
                if (k >= hi[r]) break;
                const float d = flann_d2(qx, qy, qz, p[u]);
                if (d < r2) f(p[u], d);
            }
        }
}

// a workgroup barrier ordering the LDS only.  __syncthreads() also fences global memory: it
// waits for every load in flight (the sums' prefetched gathers) and for every store's
// acknowledgement (the lists' entries) -- microseconds per barrier
__device__ __forceinline__ void nb_lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// queries: the index's own points (CELLS false: area normals, nq = g.n_pts) or the cells
// (double xyz rounded to float, nq = *n_dev).  One pass over the stencil counts the neighbours
// into the distance buckets and appends their 64-bit keys (distance bits << 32 | input index)
// to LDS in any order; the keys are then grouped by bucket (indices into the appended array)
// and each key's rank among its bucket's keys places it in the list.  A query with more than
// kNbLds neighbours takes a second stencil pass that scatters its keys into global memory.
// SMALL (an area below 2^16 points): the keys' indices as 16 bits, ~40 KB of LDS -- four
// blocks per CU instead of three
template <bool CELLS, bool SMALL>
__global__ void __launch_bounds__(kNbT)
k_nb_lists(GridView g, float r2, float bscale, const double *__restrict__ cells,
           const uint32_t *__restrict__ n_dev, NbLists L, const uint32_t *__restrict__ sel) {
    using IdxT = typename std::conditional<SMALL, uint16_t, uint32_t>::type;
    __shared__ uint32_t cnt[kNbBuckets];
    __shared__ uint32_t kd[kNbLds];   // appended keys: the distance's bits
    __shared__ IdxT ki[kNbLds];       //   and the input index
    __shared__ uint16_t grp[kNbLds];  // the keys' positions grouped by bucket
    // a key as one 64-bit value ordered as FLANN orders neighbours: (distance, index)
    auto key = [&](uint32_t j) { return ((unsigned long long)kd[j] << 32) | (uint32_t)ki[j]; };
    __shared__ uint32_t wsum[kNbT / 64];
    __shared__ uint32_t sh_base, sh_ok, sh_pos, sh_m, sh_need;
    // CELLS with sel: only the cells sel[1 ..= sel[0]] (those k_cell_sums_exact left to the
    // ordered path), their lists at the compact positions
    const uint32_t nq = CELLS ? (sel ? *sel : *n_dev) : g.n_pts;
    if (threadIdx.x == 0) sh_pos = sh_need = 0;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    auto bucket_of = [&](float d) { return min((uint32_t)(d * bscale), kNbBuckets - 1u); };
    uint32_t qround = 0;
    for (uint32_t qi = blockIdx.x; qi < nq; qi += gridDim.x, ++qround) {
        if (!CELLS) NB_STAMP(0, qround, 0);
        float qx, qy, qz;
        if (CELLS) {
            const uint32_t ci = sel ? sel[1 + qi] : qi;
            qx = (float)cells[3 * (size_t)ci];
            qy = (float)cells[3 * (size_t)ci + 1];
            qz = (float)cells[3 * (size_t)ci + 2];
        } else {
            const float4 q = g.pts[qi];
            qx = q.x;
            qy = q.y;
            qz = q.z;
        }
        for (int b = threadIdx.x; b < kNbBuckets; b += kNbT) cnt[b] = 0;
        if (threadIdx.x == 0) sh_m = 0;
        nb_lds_barrier();
        if (!CELLS) NB_STAMP(0, qround, 1);
        uint32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
        stencil_ranges(g, qx, qy, qz, lo, hi);   // (false: empty ranges)
        // the one pass over the stencil's four row ranges, kNbU candidates in flight per thread,
        // one LDS append per wave and round.  (The ranges as one flat index space with 8 in
        // flight measured slower: 66 vs 45 us per C1 frame -- the range selects cost more VALU
        // than the partial rounds cost latency)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            for (uint32_t k0 = lo[r] + threadIdx.x; k0 < hi[r]; k0 += kNbU * kNbT) {
                float4 p[kNbU];
#pragma unroll
                for (int u = 0; u < kNbU; ++u) {
                    const uint32_t k = k0 + (uint32_t)u * kNbT;
                    p[u] = g.pts[k < hi[r] ? k : hi[r] - 1];
                }
                bool in[kNbU];
                float dd[kNbU];
                uint64_t bal[kNbU];
                uint32_t tot = 0;
#pragma unroll
                for (int u = 0; u < kNbU; ++u) {
                    dd[u] = flann_d2(qx, qy, qz, p[u]);
                    in[u] = k0 + (uint32_t)u * kNbT < hi[r] && dd[u] < r2;
                    if (in[u]) atomicAdd(&cnt[bucket_of(dd[u])], 1u);
                    bal[u] = __ballot(in[u]);
                    tot += (uint32_t)__popcll(bal[u]);
                }
                if (tot) {   // (uniform)
                    const int leader = __ffsll((unsigned long long)__ballot(1)) - 1;
                    uint32_t base = 0;
                    if (lane == leader) base = atomicAdd(&sh_m, tot);
                    base = (uint32_t)__shfl((int)base, leader);
#pragma unroll
                    for (int u = 0; u < kNbU; ++u) {
                        const uint32_t pos =
                            base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[u] >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal[u], 0u));
                        if (in[u] && pos < (uint32_t)kNbLds) {
                            kd[pos] = __float_as_uint(dd[u]);
                            ki[pos] = (IdxT)__float_as_uint(p[u].w);
                        }
                        base += (uint32_t)__popcll(bal[u]);
                    }
                }
            }
        nb_lds_barrier();
        if (!CELLS) NB_STAMP(0, qround, 2);
        // exclusive scan of the buckets: thread t owns buckets [8 t, 8 t + 8)
        constexpr int kPer = kNbBuckets / kNbT;
        uint32_t v[kPer], run = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            v[j] = cnt[kPer * threadIdx.x + j];
            run += v[j];
        }
        const uint32_t incl = nb_wave_incl_scan(run);
        if (lane == 63) wsum[wid] = incl;
        nb_lds_barrier();
        uint32_t ex = incl - run, m = 0;
#pragma unroll
        for (int w = 0; w < kNbT / 64; ++w) {
            ex += w < wid ? wsum[w] : 0u;
            m += wsum[w];
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
            cnt[kPer * threadIdx.x + j] = ex;   // bucket start
            ex += v[j];
        }
        const bool big = m > (uint32_t)kNbLds;
        if (threadIdx.x == 0) {
            // the list's words from the block's own region of the list buffer (no device
            // atomics: those on one shared cursor serialise across the XCDs).  A list past the LDS sorts its 64-bit
            // keys in global memory, after its entries: m + 1 + 2 m words.  A list its region
            // cannot hold spills to the shared pool behind the regions (one device atomic per
            // spilled list: the dense blocks of a streamed area, not every block); one that
            // fits neither marks the list empty and the overflow.  The block's use (region +
            // spills) goes to the host, which then regrows the buffer and runs the normals again.
            const uint32_t words = big ? 3 * m + 1 : m;
            uint32_t ok = (uint64_t)sh_pos + words <= L.per_block;
            uint64_t b = (uint64_t)L.per_block * blockIdx.x + sh_pos;
            if (ok) {
                sh_pos += words;
            } else {
                const uint32_t at = atomicAdd(L.pool_cursor, words);
                ok = (uint64_t)at + words <= L.pool_words;
                b = L.pool_base + at;
                if (!ok) atomicOr(L.overflow, 1u);
            }
            sh_base = (uint32_t)b;
            sh_ok = ok;
            sh_need += words;   // (counted on: the host's regrow size)
            L.meta[qi] = make_uint2(sh_base, ok ? m : 0u);
        }
        nb_lds_barrier();
        if (!CELLS) NB_STAMP(0, qround, 3);
        const uint32_t base = sh_base;
        if (sh_ok && m) {
            uint32_t *out = L.list + base;
            if (!big) {
                // group the appended keys by bucket (cnt[b] becomes the bucket's end).  Four keys
                // per thread at a time: the loops are chains of LDS round trips, and few waves
                // share a CU (48 KB of LDS per block)
                constexpr int G4 = 4;
                for (uint32_t i0 = threadIdx.x; i0 < m; i0 += G4 * kNbT) {
                    uint32_t bk[G4];
#pragma unroll
                    for (int u = 0; u < G4; ++u) {
                        const uint32_t i = min(i0 + (uint32_t)u * kNbT, m - 1);
                        bk[u] = bucket_of(__uint_as_float(kd[i]));
                    }
                    uint32_t pos[G4];
#pragma unroll
                    for (int u = 0; u < G4; ++u)
                        if (i0 + (uint32_t)u * kNbT < m) pos[u] = atomicAdd(&cnt[bk[u]], 1u);
#pragma unroll
                    for (int u = 0; u < G4; ++u)
                        if (i0 + (uint32_t)u * kNbT < m) grp[pos[u]] = (uint16_t)(i0 + (uint32_t)u * kNbT);
                }
                nb_lds_barrier();
                if (!CELLS) NB_STAMP(0, qround, 4);
                // each key's place = its bucket's start + its rank among the bucket's keys (the
                // keys are distinct: distinct indices; a bucket holds a distance's exact ties, 2.4
                // keys on average in C1).  Four grouped positions per thread, in lockstep
                for (uint32_t i0 = threadIdx.x; i0 < m; i0 += G4 * kNbT) {
                    unsigned long long kv[G4];
                    uint32_t s0[G4], len[G4], rank[G4], lmax = 0;
#pragma unroll
                    for (int u = 0; u < G4; ++u) kv[u] = key(grp[min(i0 + (uint32_t)u * kNbT, m - 1)]);
#pragma unroll
                    for (int u = 0; u < G4; ++u) {
                        const uint32_t b = bucket_of(__uint_as_float((uint32_t)(kv[u] >> 32)));
                        s0[u] = b ? cnt[b - 1] : 0u;
                        len[u] = i0 + (uint32_t)u * kNbT < m ? cnt[b] - s0[u] : 0u;
                        rank[u] = 0;
                    }
#pragma unroll
                    for (int u = 0; u < G4; ++u) lmax = max(lmax, len[u]);
                    for (uint32_t jj = 0; jj < lmax; ++jj) {
                        unsigned long long o[G4];
#pragma unroll
                        for (int u = 0; u < G4; ++u)
                            o[u] = key(grp[jj < len[u] ? s0[u] + jj : s0[u]]);
#pragma unroll
                        for (int u = 0; u < G4; ++u) rank[u] += (jj < len[u]) & (o[u] < kv[u]);
                    }
#pragma unroll
                    for (int u = 0; u < G4; ++u)
                        if (i0 + (uint32_t)u * kNbT < m) out[s0[u] + rank[u]] = (uint32_t)kv[u];
                }
            } else {
                unsigned long long *K =
                    reinterpret_cast<unsigned long long *>(L.list + ((base + m + 1) & ~1u));
                // a second stencil pass scatters the keys by bucket into global memory
                nb_for_within(g, lo, hi, qx, qy, qz, r2, [&](const float4 &p, float d) {
                    K[atomicAdd(&cnt[bucket_of(d)], 1u)] =
                        ((unsigned long long)__float_as_uint(d) << 32) | __float_as_uint(p.w);
                });
                __threadfence_block();
                __syncthreads();   // (global memory: the keys)
                for (uint32_t i = threadIdx.x; i < m; i += kNbT) {
                    const unsigned long long ki = K[i];
                    const uint32_t b = bucket_of(__uint_as_float((uint32_t)(ki >> 32)));
                    const uint32_t s0 = b ? cnt[b - 1] : 0u, e = cnt[b];
                    uint32_t rank = 0;
                    for (uint32_t j = s0; j < e; ++j) rank += K[j] < ki;
                    out[s0 + rank] = (uint32_t)ki;
                }
            }
        }
        nb_lds_barrier();   // the LDS is reused by the next query
        if (!CELLS) NB_STAMP(0, qround, 5);
#ifdef PCP_STAMPS
        if (!CELLS && threadIdx.x == 0 && blockIdx.x < kNbStampBlocks && qround < kNbStampQ)
            g_nb_stamps[0][(blockIdx.x * kNbStampQ + qround) * kNbStampPh + 7] = m;
#endif
    }
    if (threadIdx.x == 0 && sh_need) atomicMax(L.need, sh_need);   // (no return value awaited)
}

// computeCellSurfaceNormal's tail (:301-340): the normalised sum of the finite neighbours'
// normals, GridCell's default (0, 0, 1) without any or below 1e-6
__device__ __forceinline__ void cell_normal_out(float *o, double sx, double sy, double sz,
                                                uint32_t nvalid) {
    o[0] = 0.0f;
    o[1] = 0.0f;
    o[2] = 1.0f;
    if (nvalid != 0) {
        const double norm = sqrt(sx * sx + sy * sy + sz * sz);
        if (norm > 1e-6) {
            o[0] = (float)(sx / norm);
            o[1] = (float)(sy / norm);
            o[2] = (float)(sz / norm);
        }
    }
}

// sequential sums over the sorted lists.  CELLS false: the 9 float moments of
// computeMeanAndCovarianceMatrix (shifted by K = the first listed point: xx xy xz yy yz zz x y
// z), then the covariance and the normal; CELLS true: the 3 double sums of the finite
// neighbours' normals (computeCellSurfaceNormal :301-340), then the cell normal.
//
// A block takes QB queries; its lists are cut into chunks of 64 steps.  Wave 0 adds the
// chunks' summands in list order, one lane per (query, summand) -- the only sequential part,
// ~1 add per step.  Waves 1-3 feed it, each element (query, step) of a chunk on one producer
// lane: chunk c + 2's list entries and chunk c + 1's records are loaded while chunk c's
// summands are formed (LDS, double-buffered).  The kernel is bound by the VALU work per
// element (producers) and the consumer's dependent adds, not by the loads.
template <bool CELLS> struct NbCfg;
template <> struct NbCfg<false> {
    using T = float;
    static constexpr int NT = 9, QB = 7;
};
template <> struct NbCfg<true> {
    using T = double;
    static constexpr int NT = 3, QB = 7;
};
constexpr int kNbSteps = 64;   // list entries per chunk
#ifndef PCP_NB_LIST_AHEAD
#define PCP_NB_LIST_AHEAD 1    // k_nb_sums: chunks of list entries in flight (build knob, A/B: 1 best)
#endif
constexpr int kNbListAhead = PCP_NB_LIST_AHEAD;


// one neighbour's gathered record: its point (area moments) or its normal (cells), 16 bytes
using NbRec = float4;

template <bool CELLS>
__global__ void __launch_bounds__(kNbT)
k_nb_sums(GridView g, const uint2 *__restrict__ meta, const uint32_t *__restrict__ list,
          const uint32_t *__restrict__ n_dev, const float4 *__restrict__ recs,
          float *__restrict__ out, float4 *__restrict__ out4, uint32_t *ctl,
          uint32_t *__restrict__ ctl_host, const uint32_t *__restrict__ sel) {
    // the lists' largest block uses and overflow word (final: every k_nb_lists ran before this launch)
    // to the caller's pinned landing, one plain store each, then cleared for the next call (no
    // memset launch in front of its k_nb_lists)
    if (ctl_host && blockIdx.x == 0 && threadIdx.x < 5) {
        ctl_host[threadIdx.x] = ctl[threadIdx.x];
        ctl[threadIdx.x] = 0;   // (ctl is written: neither const nor restrict)
    }
    using Cfg = NbCfg<CELLS>;
    using T = typename Cfg::T;
    constexpr int NT = Cfg::NT, QB = Cfg::QB, S = kNbSteps;
    static_assert(S == 64, "one wave's 64 lanes per query row");
    constexpr int PW = kNbT / 64 - 1;            // producer waves
    constexpr int PER = (QB + PW - 1) / PW;      // query rows per producer wave
    // rows of S summands padded by 16 bytes: the consumer lanes' 16-byte reads start 4 banks
    // apart (conflict-free per 16 lanes)
    constexpr int SP = S + 16 / (int)sizeof(T);
    __shared__ __attribute__((aligned(16))) T buf[2][QB][NT][SP];
    __shared__ uint2 qm[QB];
    __shared__ float4 qk[QB];          // K (area) per query
    __shared__ uint32_t valid[QB];     // finite neighbour normals (cells)
    __shared__ T accs[QB][NT];
    const uint32_t nq = CELLS ? (sel ? *sel : *n_dev) : g.n_pts;   // (sel: as k_nb_lists)
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t qround = 0;
    for (uint32_t q0 = blockIdx.x * QB; q0 < nq; q0 += gridDim.x * QB, ++qround) {
        if (!CELLS) NB_STAMP(1, qround, 0);
        if (threadIdx.x < QB) {
            const uint32_t qi = q0 + threadIdx.x;
            const uint2 mt = qi < nq ? meta[qi] : make_uint2(0u, 0u);
            qm[threadIdx.x] = mt;
            valid[threadIdx.x] = 0;
            if (!CELLS) qk[threadIdx.x] = mt.y ? recs[list[mt.x]] : make_float4(0, 0, 0, 0);
        }
        nb_lds_barrier();
        uint32_t maxm = 0;
#pragma unroll
        for (int q = 0; q < QB; ++q) maxm = max(maxm, qm[q].y);
        const uint32_t nch = (maxm + S - 1) / S;
        // producer wave w (1..3) owns the query rows j = w - 1 + PW * i (i < PER): element
        // (row j, step c * S + lane).  Every load unconditional (clamped to entry 0, the value
        // discarded under the mask): a load under a branch, or a select right after it, waits
        auto row = [&](int i) { return min(wid - 1 + PW * i, QB - 1); };
        auto row_ok = [&](int i) { return wid > 0 && wid - 1 + PW * i < QB; };
        auto load_list = [&](uint32_t c, uint32_t (&kk)[PER]) {
            uint32_t mk = 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const uint2 mt = qm[max(row(i), 0)];
                const uint32_t st = c * S + (uint32_t)lane;
                const bool ok = row_ok(i) && st < mt.y;
                kk[i] = list[ok ? mt.x + st : 0u];
                mk |= (ok ? 1u : 0u) << i;
            }
            return mk;
        };
        auto gather = [&](const uint32_t (&kk)[PER], uint32_t mk, NbRec (&rr)[PER]) {
#pragma unroll
            for (int i = 0; i < PER; ++i) rr[i] = recs[(mk >> i & 1u) ? kk[i] : 0u];
        };
        // the list entries of chunks c + 1 .. c + LA in flight (a streamed list misses the
        // caches: one chunk ahead left each chunk waiting ~1 us for its entries), the records
        // of chunk c + 1 (the points / normals: cache-resident)
        constexpr int LA = kNbListAhead;
        uint32_t KA[LA][PER], MA[LA];
        NbRec R0[PER];                               // records of chunk c
        uint32_t M0 = 0;
        if (wid > 0) {
            M0 = load_list(0, KA[0]);
            gather(KA[0], M0, R0);
#pragma unroll
            for (int d = 0; d < LA; ++d) MA[d] = load_list(1 + d, KA[d]);
        }
        T acc = 0;
        const int cq = lane / NT, ca = lane % NT;   // the consumer lane's (query, summand)
        for (uint32_t c = 0; c <= nch; ++c) {
            if (wid > 0 && c < nch) {
                NbRec rc[PER];
                const uint32_t mc = M0;
#pragma unroll
                for (int i = 0; i < PER; ++i) rc[i] = R0[i];
                // chunk c + 1's records, then chunk c + 1 + LA's list entries
                gather(KA[0], MA[0], R0);
                M0 = MA[0];
#pragma unroll
                for (int d = 0; d + 1 < LA; ++d) {
                    MA[d] = MA[d + 1];
#pragma unroll
                    for (int i = 0; i < PER; ++i) KA[d][i] = KA[d + 1][i];
                }
                MA[LA - 1] = load_list(c + 1 + LA, KA[LA - 1]);
                T (*B)[NT][SP] = buf[c & 1];
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    if (!row_ok(i)) continue;   // (uniform per wave)
                    const int j = row(i);
                    T tv[NT];
#pragma unroll
                    for (int a = 0; a < NT; ++a) tv[a] = 0;
                    const NbRec r = rc[i];
                    if (CELLS) {
                        const bool fin = (mc >> i & 1u) && isfinite(r.x) && isfinite(r.y) &&
                                         isfinite(r.z);
                        if (fin) {
                            tv[0] = (T)r.x;
                            tv[1] = (T)r.y;
                            tv[2 % NT] = (T)r.z;
                        }
                        const uint32_t nv = (uint32_t)__popcll(__ballot(fin));
                        if (lane == 0) valid[j] += nv;
                    } else if (mc >> i & 1u) {
                        const float4 K = qk[j];
                        const float x = r.x - K.x, y = r.y - K.y, z = r.z - K.z;
                        tv[0] = (T)(x * x);
                        tv[1] = (T)(x * y);
                        tv[2 % NT] = (T)(x * z);
                        tv[3 % NT] = (T)(y * y);
                        tv[4 % NT] = (T)(y * z);
                        tv[5 % NT] = (T)(z * z);
                        tv[6 % NT] = (T)x;
                        tv[7 % NT] = (T)y;
                        tv[8 % NT] = (T)z;
                    }
#pragma unroll
                    for (int a = 0; a < NT; ++a) B[j][a][lane] = tv[a];
                }
            }
            if (wid == 0 && c > 0 && cq < QB) {
                // acc + 0 == acc for these sums (they start at +0 and never become -0): the
                // zero padding past a query's list is exact
                if (CELLS) {
                    const double2 *v =
                        reinterpret_cast<const double2 *>(&buf[(c - 1) & 1][cq][ca][0]);
#pragma unroll 8
                    for (int t = 0; t < S / 2; ++t) {
                        const double2 w = v[t];
                        acc = acc + (T)w.x;
                        acc = acc + (T)w.y;
                    }
                } else {
                    const float4 *v =
                        reinterpret_cast<const float4 *>(&buf[(c - 1) & 1][cq][ca][0]);
#pragma unroll 8
                    for (int t = 0; t < S / 4; ++t) {
                        const float4 w = v[t];
                        acc = acc + (T)w.x;
                        acc = acc + (T)w.y;
                        acc = acc + (T)w.z;
                        acc = acc + (T)w.w;
                    }
                }
            }
            nb_lds_barrier();
        }
        if (!CELLS) NB_STAMP(1, qround, 1);
#ifdef PCP_STAMPS
        if (!CELLS && threadIdx.x == 0 && blockIdx.x < kNbStampBlocks && qround < kNbStampQ)
            g_nb_stamps[1][(blockIdx.x * kNbStampQ + qround) * kNbStampPh + 7] = maxm;
#endif
        if (wid == 0 && cq < QB) accs[cq][ca] = acc;
        __syncthreads();
        if (threadIdx.x < QB && q0 + threadIdx.x < nq) {
            const int q = threadIdx.x;
            const uint32_t qi = q0 + q;
            const uint32_t m = qm[q].y;
            if (CELLS) {
                cell_normal_out(out + 3 * (size_t)(sel ? sel[1 + qi] : qi), (double)accs[q][0],
                                (double)accs[q][1], (double)accs[q][2 % NT], valid[q]);
            } else {
                const float4 qp = g.pts[qi];
                float *o = out + 3 * (size_t)__float_as_uint(qp.w);
                if (m < 3) {   // computePointNormal: < 3 neighbours -> NaN
                    o[0] = o[1] = o[2] = NAN;
                } else {
                    float a[9];
                    const float fm = (float)m;
#pragma unroll
                    for (int k = 0; k < 9; ++k) a[k] = pcp_lm_div((float)accs[q][k % NT], fm);
                    float cov[3][3];
                    cov[0][0] = a[0] - a[6] * a[6];
                    cov[0][1] = a[1] - a[6] * a[7];
                    cov[0][2] = a[2] - a[6] * a[8];
                    cov[1][1] = a[3] - a[7] * a[7];
                    cov[1][2] = a[4] - a[7] * a[8];
                    cov[2][2] = a[5] - a[8] * a[8];
                    cov[1][0] = cov[0][1];
                    cov[2][0] = cov[0][2];
                    cov[2][1] = cov[1][2];
                    normal_from_cov(cov, qp.x, qp.y, qp.z, o);
                }
                // (the cells' sums gather the normals as 16-byte records)
                out4[__float_as_uint(qp.w)] = make_float4(o[0], o[1], o[2], 0.0f);
            }
        }
        nb_lds_barrier();   // (LDS reuse; the stores need no acknowledgement here)
    }
}

// The cells' sums where their order cannot matter.  computeCellSurfaceNormal adds the finite
// neighbours' float normals as doubles.  Let E_min / E_max be the smallest / largest exponent
// of their nonzero components and n their count: every component is a multiple of
// U = 2^(E_min - 23), every partial sum -- of any subset, in any order -- a multiple of U below
// n 2^(E_max + 1) in magnitude, so when n 2^(E_max + 1) <= 2^53 U, i.e.
// E_min - E_max >= ceil(log2 n) - 29, every addition is exact and the sum is the same in every
// order: FLANN's included.  One block per cell sums its stencil's neighbours in any order (no
// list, no sort) and checks the bound; a cell that fails it (a component below ~2^-17 of the
// largest, a subnormal) goes to sel for the ordered path (k_nb_lists / k_nb_sums over sel).
__global__ void __launch_bounds__(kNbT)
k_cell_sums_exact(GridView g, float r2, const double *__restrict__ cells,
                  const uint32_t *__restrict__ n_dev, const float4 *__restrict__ nrm4,
                  float *__restrict__ out, uint32_t *__restrict__ sel, int all_ordered) {
    __shared__ double rs[3][kNbT / 64];
    __shared__ uint32_t rc[kNbT / 64], rmin[kNbT / 64], rmax[kNbT / 64];
    const uint32_t nq = *n_dev;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (uint32_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
        const float qx = (float)cells[3 * (size_t)qi], qy = (float)cells[3 * (size_t)qi + 1],
                    qz = (float)cells[3 * (size_t)qi + 2];
        uint32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
        stencil_ranges(g, qx, qy, qz, lo, hi);   // (false: empty ranges)
        double sx = 0.0, sy = 0.0, sz = 0.0;
        uint32_t cnt = 0, emin = 255, emax = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            for (uint32_t k0 = lo[r] + threadIdx.x; k0 < hi[r]; k0 += kNbU * kNbT) {
                float4 p[kNbU];
#pragma unroll
                for (int u = 0; u < kNbU; ++u) {
                    const uint32_t k = k0 + (uint32_t)u * kNbT;
                    p[u] = g.pts[k < hi[r] ? k : hi[r] - 1];
                }
                bool in[kNbU];
                float4 v[kNbU];
#pragma unroll
                for (int u = 0; u < kNbU; ++u) {
                    in[u] = k0 + (uint32_t)u * kNbT < hi[r] && flann_d2(qx, qy, qz, p[u]) < r2;
                    v[u] = nrm4[in[u] ? __float_as_uint(p[u].w) : 0u];   // (unconditional)
                }
#pragma unroll
                for (int u = 0; u < kNbU; ++u) {
                    if (!(in[u] && isfinite(v[u].x) && isfinite(v[u].y) && isfinite(v[u].z)))
                        continue;
                    sx += (double)v[u].x;
                    sy += (double)v[u].y;
                    sz += (double)v[u].z;
                    ++cnt;
                    const uint32_t b[3] = {__float_as_uint(v[u].x) & 0x7fffffffu,
                                           __float_as_uint(v[u].y) & 0x7fffffffu,
                                           __float_as_uint(v[u].z) & 0x7fffffffu};
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        if (b[a]) {   // (a subnormal has exponent field 0: emin 0 fails the bound)
                            emin = min(emin, b[a] >> 23);
                            emax = max(emax, b[a] >> 23);
                        }
                }
            }
        // any-order reduction (exact whenever the bound holds; discarded otherwise)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            sx += __shfl_xor(sx, o);
            sy += __shfl_xor(sy, o);
            sz += __shfl_xor(sz, o);
            cnt += (uint32_t)__shfl_xor((int)cnt, o);
            emin = min(emin, (uint32_t)__shfl_xor((int)emin, o));
            emax = max(emax, (uint32_t)__shfl_xor((int)emax, o));
        }
        if (lane == 0) {
            rs[0][wid] = sx;
            rs[1][wid] = sy;
            rs[2][wid] = sz;
            rc[wid] = cnt;
            rmin[wid] = emin;
            rmax[wid] = emax;
        }
        nb_lds_barrier();
        if (threadIdx.x == 0) {
            double tx = 0.0, ty = 0.0, tz = 0.0;
            uint32_t n = 0, e0 = 255, e1 = 0;
            for (int w = 0; w < kNbT / 64; ++w) {
                tx += rs[0][w];
                ty += rs[1][w];
                tz += rs[2][w];
                n += rc[w];
                e0 = min(e0, rmin[w]);
                e1 = max(e1, rmax[w]);
            }
            const int lg = n <= 1 ? 0 : 32 - __clz((int)(n - 1));   // ceil(log2 n)
            const bool exact = n == 0 || (e0 > 0 && (e0 == 255 || (int)e0 - (int)e1 >= lg - 29));
            if (exact && !all_ordered) {   // (all_ordered: PCP_CELLS_ORDER_FREE=0, A/B)
                cell_normal_out(out + 3 * (size_t)qi, tx, ty, tz, n);
            } else {   // sel[0]: the count (zeroed by k_area_prep), sel[1 + i]: the cells
                const uint32_t pos = atomicAdd(&sel[0], 1u);
                sel[1 + pos] = qi;
            }
        }
        nb_lds_barrier();   // (the LDS is reused by the next cell)
    }
}

// the raw input's points by input index (the sums gather them by the lists' indices) and the
// non-finite points' NaN normals (they are in no list), one thread per input point
__global__ void __launch_bounds__(kXT) k_area_prep(RawIn in, float4 *__restrict__ pts_in,
                                                   float *__restrict__ out, uint32_t *sel) {
    if (sel && blockIdx.x == 0 && threadIdx.x == 0) sel[0] = 0;   // (k_cell_sums_exact's count)
    const uint64_t i = (uint64_t)blockIdx.x * kXT + threadIdx.x;
    if (i >= in.n) return;
    const unsigned char *p = in.raw + i * in.step;
    const float x = *reinterpret_cast<const float *>(p + in.ox),
                y = *reinterpret_cast<const float *>(p + in.oy),
                z = *reinterpret_cast<const float *>(p + in.oz);
    pts_in[i] = make_float4(x, y, z, 0.0f);
    if (!(isfinite(x) && isfinite(y) && isfinite(z)))
        out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = NAN;
}


struct Lattice {
    double x0, y0, z0, res, z_step;
    int32_t gw, gh, layers;
    uint32_t total;
};

__device__ __forceinline__ void lattice_xyz(const Lattice &L, uint32_t li, double &x, double &y,
                                            double &z) {
    const uint32_t k = li % (uint32_t)L.layers;
    const uint32_t ij = li / (uint32_t)L.layers;
    const uint32_t j = ij % (uint32_t)L.gw, i = ij / (uint32_t)L.gw;
    x = L.x0 + (int)j * L.res;
    y = L.y0 + (int)i * L.res;
    z = L.z0 + (int)k * L.z_step + L.z_step / 2.0;
}

// isPointNearExcavation (radiusSearch(r) > 0) of every lattice point; linear index =
// (i * gw + j) * layers + k, i.e. the reference's loop order.  One wave per lattice point: the
// lanes split the block's candidate points and stop at the first round that finds one (a point
// far from the area would otherwise walk hundreds of candidates on one lane)
constexpr int kLatWaves = kXT / 64;
__global__ void __launch_bounds__(kXT)
k_lattice_flags(GridView g, float r2, Lattice L, uint8_t *__restrict__ flags) {
    const uint32_t li = blockIdx.x * kLatWaves + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (li >= L.total) return;   // uniform per wave
    double x, y, z;
    lattice_xyz(L, li, x, y, z);
    const float qx = (float)x, qy = (float)y, qz = (float)z;
    uint32_t lo[4], hi[4];
    bool hit = false;
    if (stencil_ranges(g, qx, qy, qz, lo, hi)) {
        for (int r = 0; r < 4 && !hit; ++r)
            for (uint32_t k0 = lo[r]; k0 < hi[r] && !hit; k0 += 64) {
                const uint32_t k = k0 + lane;
                const bool w = k < hi[r] && flann_within(qx, qy, qz, ld_p3(g.pts, k), r2);
                hit = __ballot(w) != 0ull;
            }
    }
    if (lane == 0) flags[li] = hit ? 1 : 0;
}

// one block: the flagged lattice points in order -> cells (double xyz); *n_out = count.  Each
// thread takes 4 consecutive lattice points per round (one 4-byte load of their flags), so a
// round covers 4,096 points: a quarter of the dependent rounds of one point per thread
__global__ void __launch_bounds__(1024)
k_lattice_compact(const uint8_t *__restrict__ flags, Lattice L, double *__restrict__ cells,
                  uint32_t cap, uint32_t *__restrict__ n_out, uint32_t *__restrict__ n_host,
                  uint32_t *__restrict__ sel) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (sel && threadIdx.x == 0) sel[0] = 0;   // (k_cell_sums_exact's count, after this launch)
    __shared__ uint32_t wc[16];
    uint32_t run = 0;
    for (uint32_t base = 0; base < L.total; base += 4096) {
        const uint32_t li0 = base + 4 * threadIdx.x;
        uint32_t f4 = 0;
        if (li0 + 3 < L.total) {
            f4 = *reinterpret_cast<const uint32_t *>(flags + li0);   // 4-aligned: base, 4 t
        } else {
            for (int j = 0; j < 4; ++j)
                if (li0 + j < L.total && flags[li0 + j]) f4 |= 1u << (8 * j);
        }
        uint32_t fl = 0;   // bit j: lattice point li0 + j flagged
#pragma unroll
        for (int j = 0; j < 4; ++j) fl |= ((f4 >> (8 * j)) & 0xFFu) ? (1u << j) : 0u;
        const uint32_t c = (uint32_t)__popc(fl);
        // exclusive scan of c over the block: within the wave, then the waves' totals
        uint32_t inc = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(inc, o, 64);
            if (lane >= o) inc += v;
        }
        if (lane == 63) wc[wid] = inc;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            pre += w < wid ? wc[w] : 0u;
            tot += wc[w];
        }
        uint32_t d = run + pre + inc - c;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if ((fl >> j) & 1u) {
                if (d < cap) {
                    double x, y, z;
                    lattice_xyz(L, li0 + j, x, y, z);
                    cells[3 * (size_t)d] = x;
                    cells[3 * (size_t)d + 1] = y;
                    cells[3 * (size_t)d + 2] = z;
                }
                ++d;
            }
        }
        run += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *n_out = run;
        if (n_host) *n_host = run;   // the pinned landing: no readback copy
    }
}

// computeCellSurfaceNormal: a block per cell (block-strided over the cells; their count is
// read on the device, so the host never waits for the lattice), neighbours within 1.5 m of
// the float cell position
__global__ void __launch_bounds__(kXT)
k_cell_normals(GridView g, float r2, const double *__restrict__ cells,
               const float *__restrict__ area_nrm, const uint32_t *__restrict__ n_cells,
               float *__restrict__ out) {
    const uint32_t nc = *n_cells;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ DD lds[3][kXT / 64];
    __shared__ uint32_t lv[kXT / 64];
    for (uint32_t c = blockIdx.x; c < nc; c += gridDim.x) {
        const float qx = (float)cells[3 * (size_t)c], qy = (float)cells[3 * (size_t)c + 1],
                    qz = (float)cells[3 * (size_t)c + 2];
        DD s[3] = {{0, 0}, {0, 0}, {0, 0}};
        uint32_t valid = 0;
        uint32_t lo[4], hi[4];
        if (stencil_ranges(g, qx, qy, qz, lo, hi)) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                for (uint32_t k = lo[r] + threadIdx.x; k < hi[r]; k += kXT) {
                    const float4 p = g.pts[k];
                    if (!flann_within(qx, qy, qz, p, r2)) continue;
                    const float *n = area_nrm + 3 * (size_t)__float_as_uint(p.w);
                    const float nx = n[0], ny = n[1], nz = n[2];
                    if (!(isfinite(nx) && isfinite(ny) && isfinite(nz))) continue;
                    dd_add(s[0], (double)nx);
                    dd_add(s[1], (double)ny);
                    dd_add(s[2], (double)nz);
                    ++valid;
                }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                DD t{__shfl_xor(s[a].hi, o, 64), __shfl_xor(s[a].lo, o, 64)};
                s[a] = dd_merge(s[a], t);
            }
            valid += __shfl_xor(valid, o, 64);
        }
        if (lane == 0) {
            for (int a = 0; a < 3; ++a) lds[a][wid] = s[a];
            lv[wid] = valid;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            DD t[3];
            uint32_t nv = 0;
            for (int a = 0; a < 3; ++a) {
                t[a] = lds[a][0];
                for (int w = 1; w < kXT / 64; ++w) t[a] = dd_merge(t[a], lds[a][w]);
            }
            for (int w = 0; w < kXT / 64; ++w) nv += lv[w];
            float *o = out + 3 * (size_t)c;
            o[0] = 0.0f;   // GridCell's default surface normal
            o[1] = 0.0f;
            o[2] = 1.0f;
            if (nv != 0) {
                const double sx = t[0].hi + t[0].lo, sy = t[1].hi + t[1].lo,
                             sz = t[2].hi + t[2].lo;
                const double norm = sqrt(sx * sx + sy * sy + sz * sz);
                if (norm > 1e-6) {
                    o[0] = (float)(sx / norm);
                    o[1] = (float)(sy / norm);
                    o[2] = (float)(sz / norm);
                }
            }
        }
        __syncthreads();
    }
}

}  // namespace pcp

namespace pcp {

// the exact normals' two phases over the device-resident setup (pcp_set_excavation_area):
// the area's sorted lists + ordered sums, and the cells' (order-free exact sums, then the lists
// and sums of the cells they leave).  Everything they read is on the device: the indices
// (exc_norm), the points by input index (nb_pts), the lattice and its count (cells_xyz,
// cells_n_d), so an overflow can rerun them long after the raw records are gone.
// a list buffer as the grid's regions (3/4 of its words; PCP_NB_REGION_PCT) and the spill pool
// behind them.  ctl
// words: [0] / [1] the area's / cells' largest block use, [2] the overflow, [3] / [4] their pool
// cursors -- landed in area_host[1 .. 5] and cleared by k_nb_sums<true>
static NbLists nb_lists_view(const pcp_ctx *ctx, const DevBuf &list, const DevBuf &meta,
                             uint32_t *need, uint32_t *overflow, uint32_t *cursor, uint32_t grid) {
    const uint64_t words = std::min<uint64_t>(list.cap / 4, 0xffffffffull);
    const uint32_t per_block = (uint32_t)(words * (uint64_t)ctx->nb_region_pct / 100 / grid);
    const uint64_t pool_base = (uint64_t)per_block * grid;
    return NbLists{list.as<uint32_t>(), meta.as<uint2>(), need, overflow,
                   per_block, cursor, pool_base, words - pool_base};
}

static void nb_area_launch(pcp_ctx *ctx, hipStream_t st) {
    const GridView gn = ctx->exc_norm.view();
    const float r2n = (float)(kNormalRadius * kNormalRadius), bscale = (float)kNbBuckets / r2n;
    const uint32_t grid_a = ctx->area_grid_a, npts = ctx->area_npts;
    const uint64_t n = ctx->area_n;
    uint32_t *ctl = ctx->nb_ctl.as<uint32_t>();
    const NbLists La = nb_lists_view(ctx, ctx->nb_list, ctx->nb_meta, ctl, ctl + 2, ctl + 3, grid_a);
    if (n <= 65536 && ctx->nb_small)   // (input indices in 16 bits)
        hipLaunchKernelGGL((k_nb_lists<false, true>), dim3(grid_a), dim3(kNbT), 0, st, gn, r2n,
                           bscale, (const double *)nullptr, (const uint32_t *)nullptr, La,
                           (const uint32_t *)nullptr);
    else
        hipLaunchKernelGGL((k_nb_lists<false, false>), dim3(grid_a), dim3(kNbT), 0, st, gn, r2n,
                           bscale, (const double *)nullptr, (const uint32_t *)nullptr, La,
                           (const uint32_t *)nullptr);
    hipLaunchKernelGGL(k_nb_sums<false>, dim3((npts + NbCfg<false>::QB - 1) / NbCfg<false>::QB),
                       dim3(kNbT), 0, st, gn, (const uint2 *)La.meta, (const uint32_t *)La.list,
                       (const uint32_t *)nullptr, (const float4 *)ctx->nb_pts.as<float4>(),
                       ctx->area_nrm.as<float>(), ctx->nb_pts.as<float4>() + n, ctl,
                       (uint32_t *)nullptr, (const uint32_t *)nullptr);
}
static void nb_cells_launch(pcp_ctx *ctx, hipStream_t st) {
    const GridView gn = ctx->exc_norm.view();
    const float r2n = (float)(kNormalRadius * kNormalRadius), bscale = (float)kNbBuckets / r2n;
    const uint32_t grid_c = ctx->area_grid_c;
    const uint64_t total = ctx->area_total;
    uint32_t *ctl = ctx->nb_ctl.as<uint32_t>();
    uint32_t *sel = ctx->nb_sel.as<uint32_t>();
    const uint32_t *n_d = ctx->cells_n_d.as<uint32_t>();
    const float4 *nrm4 = ctx->nb_pts.as<float4>() + ctx->area_n;
    uint32_t *n_h = ctx->area_host.as<uint32_t>();
    const NbLists Lc = nb_lists_view(ctx, ctx->nb_list_c, ctx->nb_meta_c, ctl + 1, ctl + 2, ctl + 4, grid_c);
    if (total) {
        hipLaunchKernelGGL(k_cell_sums_exact, dim3(grid_c), dim3(kNbT), 0, st, gn, r2n,
                           (const double *)ctx->cells_xyz.as<double>(), n_d, nrm4,
                           ctx->cells_nrm.as<float>(), sel, ctx->cells_all_ordered ? 1 : 0);
        if (ctx->area_n <= 65536 && ctx->nb_small)
            hipLaunchKernelGGL((k_nb_lists<true, true>), dim3(grid_c), dim3(kNbT), 0, st, gn, r2n,
                               bscale, (const double *)ctx->cells_xyz.as<double>(), n_d, Lc,
                               (const uint32_t *)sel);
        else
            hipLaunchKernelGGL((k_nb_lists<true, false>), dim3(grid_c), dim3(kNbT), 0, st, gn,
                               r2n, bscale, (const double *)ctx->cells_xyz.as<double>(), n_d, Lc,
                               (const uint32_t *)sel);
    }
    // launched for an empty selection too: it lands both lists' uses and the overflow word in
    // area_host[1..3], and clears the control words
    constexpr int QB = NbCfg<true>::QB;
    hipLaunchKernelGGL(k_nb_sums<true>,
                       dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((total + QB - 1) / QB,
                                                                                4096))),
                       dim3(kNbT), 0, st, gn, (const uint2 *)Lc.meta, (const uint32_t *)Lc.list,
                       n_d, nrm4, ctx->cells_nrm.as<float>(), (float4 *)nullptr, ctl, n_h + 1,
                       (const uint32_t *)(total ? sel : nullptr));
}

bool area_overflowed(const pcp_ctx *ctx) {
    return ctx->area_host.p && ctx->area_host.as<const uint32_t>()[3] != 0u;
}

void area_join(pcp_ctx *ctx) {
    if (!ctx->area_forked) return;
    (void)hipStreamWaitEvent(ctx->stream, ctx->area_join_ev, 0);
    ctx->area_forked = false;
}

int area_finish(pcp_ctx *ctx, bool stream_synced) {
    if (ctx->area_forked) stream_synced = false;   // (its join is enqueued below)
    area_join(ctx);
    if (!ctx->area_pending) return PCP_OK;
    hipStream_t st = ctx->stream;
    if (!stream_synced) PCP_HIP(ctx, hipStreamSynchronize(st));
    uint32_t *n_h = ctx->area_host.as<uint32_t>();
    if (n_h[3]) {
        // a list buffer too small (first frames, or a denser area): regrow both to their largest
        // block's use x the grid and run the normals again (the lattice and the records stand;
        // the cells' order-free pass too, over the new area normals)
        ctx->nb_need = std::max<uint64_t>(ctx->nb_need, (uint64_t)n_h[1] * ctx->area_grid_a);
        ctx->nb_need_c = std::max<uint64_t>(ctx->nb_need_c, (uint64_t)n_h[2] * ctx->area_grid_c);
        if (std::max(ctx->nb_need, ctx->nb_need_c) > 0xffffffffull) {
            ctx->area_pending = false;
            return set_err(ctx, PCP_E_CAPACITY, "pcp_set_excavation_area: %llu neighbour list "
                           "words (32-bit list offsets)",
                           (unsigned long long)std::max(ctx->nb_need, ctx->nb_need_c));
        }
        // twice the measured need: a streamed area keeps changing (the carve), and each regrow
        // is a free + malloc + a second pass of the normals inside one frame
        PCP_HIP(ctx, ctx->nb_list.ensure(ctx->nb_need * 8 + 64));
        PCP_HIP(ctx, ctx->nb_list_c.ensure(ctx->nb_need_c * 8 + 64));
        ctx->normals_regrown++;
        n_h[1] = n_h[2] = n_h[3] = n_h[4] = n_h[5] = 0;   // (ctl: cleared by k_nb_sums<true>)
        PCP_HIP(ctx, hipMemsetAsync(ctx->nb_sel.p, 0, sizeof(uint32_t), st));
        nb_area_launch(ctx, st);
        PCP_CHECK_LAUNCH(ctx);
        nb_cells_launch(ctx, st);
        PCP_CHECK_LAUNCH(ctx);
        PCP_HIP(ctx, hipStreamSynchronize(st));
        if (n_h[3]) {
            ctx->area_pending = false;
            return set_err(ctx, PCP_E_CAPACITY, "pcp_set_excavation_area: neighbour lists "
                                                "overflowed after regrowing");
        }
    }
    // (nb_need / nb_need_c move only on an overflow: a frame the spill pool absorbed keeps the
    // buffers, a later setup does not grow them for it)
    ctx->nb_ctl_zero = true;   // k_nb_sums<true> (always launched on this path) cleared them
    ctx->n_cells = n_h[0];
    ctx->area_pending = false;
    prof_resolve(ctx);
    return PCP_OK;
}

// pcp_set_excavation_area (defer = false: settled before the return) and its _async form;
// raw_pre: the records already device-readable (pcp_excavate_area_async's landing), else staged
int area_setup_from(pcp_ctx *ctx, const pcp_cloud_view *area, double grid_resolution,
                    int32_t vertical_layers, double grid_bbox[6], uint64_t *n_cells, bool defer,
                    const unsigned char *raw_pre) {
    if (!ctx) return PCP_E_INVALID;
    int rc = check_view(ctx, area, "pcp_set_excavation_area");
    if (rc) return rc;
    if (!(grid_resolution > 0.0))
        return set_err(ctx, PCP_E_INVALID, "pcp_set_excavation_area: grid_resolution must be > 0");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    // a setup still pending is settled first (its lists may need a rerun)
    if ((rc = area_finish(ctx))) return rc;
    if (n_cells) *n_cells = defer ? ctx->cells_cap : ctx->n_cells;
    if (area->n == 0) return PCP_OK;   // :168, nothing is rebuilt; the previous cells stay
    ProfScope prof(ctx, PCP_K_EXCAV_SETUP);
    const double r_near = grid_resolution * 1.5;
    // both indices read the same staged bytes (staged once)
    const unsigned char *raw = raw_pre;
    const uint64_t n = area->n;
    PCP_HIP(ctx, ctx->area_nrm.ensure(n * 3 * sizeof(float) + 16));
    // the exact path: both grids from one pass over the records, which also lays out the points
    // by input index for the sums and the non-finite points' NaN normals (k_area_prep's work)
    bool paired = false;
    if (ctx->normals_exact) {
        PCP_HIP(ctx, ctx->nb_pts.ensure(2 * n * sizeof(float4) + 64));
        if ((rc = build_index_pair(ctx, ctx->exc_norm, kNormalRadius, ctx->exc_near, r_near,
                                   *area, &raw, ctx->nb_pts.as<float4>(),
                                   ctx->area_nrm.as<float>(), &paired)))
            return rc;
    }
    if (!paired) {
        if ((rc = build_index(ctx, ctx->exc_norm, *area, kNormalRadius, false, false, &raw)))
            return rc;
        rc = build_index(ctx, ctx->exc_near, *area, r_near, false, false, &raw);
        if (rc) return rc;   // (a held slot is drained by the next pin_stage)
    } else {
        pin_release(ctx, ctx->stream);   // (the pair's extraction read the records last)
    }
    ctx->area_n = n;
    if (ctx->exc_norm.n_pts == 0) {   // no finite point: no lattice bounds, no cells
        PCP_HIP(ctx, hipMemsetAsync(ctx->area_nrm.p, 0xff, n * 3 * sizeof(float), ctx->stream));
        pin_release(ctx, ctx->stream);
        ctx->n_cells = 0;
        ctx->cells_cap = 0;
        if (n_cells) *n_cells = 0;
        return PCP_OK;
    }
    const GridView gn = ctx->exc_norm.view(), gq = ctx->exc_near.view();
    const float r2n = (float)(kNormalRadius * kNormalRadius), r2q = (float)(r_near * r_near);
    // non-finite points are not in the index: PCL gives them a NaN normal
    const RawIn rin{raw, n, area->point_step, area->off_x, area->off_y, area->off_z};
    const uint32_t npts = (uint32_t)ctx->exc_norm.n_pts;
    // grid bounds (:239-256): min/max of the float coordinates as doubles, then the margin
    const double *bmin = ctx->exc_norm.bmin, *bmax = ctx->exc_norm.bmax;
    Lattice L;
    const double x0 = bmin[0] - grid_resolution, x1 = bmax[0] + grid_resolution;
    const double y0 = bmin[1] - grid_resolution, y1 = bmax[1] + grid_resolution;
    const double z0 = bmin[2] - grid_resolution, z1 = bmax[2] + grid_resolution;
    L.x0 = x0;
    L.y0 = y0;
    L.z0 = z0;
    L.res = grid_resolution;
    L.gw = (int)std::ceil((x1 - x0) / grid_resolution) + 1;
    L.gh = (int)std::ceil((y1 - y0) / grid_resolution) + 1;
    L.layers = vertical_layers;
    L.z_step = (z1 - z0) / std::max(1, vertical_layers);
    if (grid_bbox) {
        const double bb[6] = {x0, x1, y0, y1, z0, z1};
        for (int a = 0; a < 6; ++a) grid_bbox[a] = bb[a];
    }
    const uint64_t total = vertical_layers > 0 ? (uint64_t)L.gw * L.gh * vertical_layers : 0;
    if (total >= (1ull << 31))
        return set_err(ctx, PCP_E_CAPACITY, "pcp_set_excavation_area: %llu lattice points",
                       (unsigned long long)total);
    L.total = (uint32_t)total;
    const bool exact = ctx->normals_exact;
    defer = defer && exact;   // (the order-free A/B kernels settle before the return)
    PCP_HIP(ctx, ctx->area_host.ensure(64));
    uint32_t *n_h = ctx->area_host.as<uint32_t>();
    n_h[1] = n_h[2] = n_h[3] = n_h[4] = n_h[5] = 0;   // the lists' uses, overflow, pool cursors
    PCP_HIP(ctx, ctx->cells_n_d.ensure(64));
    uint32_t *n_d = ctx->cells_n_d.as<uint32_t>();
    // the lattice of candidate cells (:258-298) on stream st (its per-point flags in lat_flags)
    auto lattice = [&](hipStream_t st) -> int {
        PCP_HIP(ctx, ctx->lat_flags.ensure(total + 64));
        PCP_HIP(ctx, ctx->cells_xyz.ensure(total * 3 * sizeof(double) + 16));
        PCP_HIP(ctx, ctx->cells_nrm.ensure(total * 3 * sizeof(float) + 16));
        if (total) {
            hipLaunchKernelGGL(k_lattice_flags,
                               dim3((unsigned)((total + kLatWaves - 1) / kLatWaves)), dim3(kXT), 0,
                               st, gq, r2q, L, ctx->lat_flags.as<uint8_t>());
            PCP_CHECK_LAUNCH(ctx);
        }
        hipLaunchKernelGGL(k_lattice_compact, dim3(1), dim3(1024), 0, st,
                           (const uint8_t *)ctx->lat_flags.as<uint8_t>(), L,
                           ctx->cells_xyz.as<double>(), (uint32_t)total, n_d, n_h,
                           exact ? ctx->nb_sel.as<uint32_t>() : (uint32_t *)nullptr);
        PCP_CHECK_LAUNCH(ctx);
        return PCP_OK;
    };
    if (!exact) {
        // order-free fixed-point moments (A/B: PCP_NORMALS_EXACT=0), NaN for the non-finite
        // points by the blocks past the index's points; one stream
        hipLaunchKernelGGL(k_area_normals, dim3((unsigned)(npts + (n + kXT - 1) / kXT)), dim3(kXT),
                           0, ctx->stream, gn, r2n, ctx->area_nrm.as<float>(), rin);
        PCP_CHECK_LAUNCH(ctx);
        pin_release(ctx, ctx->stream);   // the normals read the raw records last
        if (int rcl = lattice(ctx->stream)) return rcl;
        if (total) {
            hipLaunchKernelGGL(k_cell_normals, dim3((unsigned)std::min<uint64_t>(total, 8192)),
                               dim3(kXT), 0, ctx->stream, gn, r2n,
                               (const double *)ctx->cells_xyz.as<double>(),
                               (const float *)ctx->area_nrm.as<float>(), (const uint32_t *)n_d,
                               ctx->cells_nrm.as<float>());
            PCP_CHECK_LAUNCH(ctx);
        }
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        ctx->n_cells = n_h[0];
        ctx->cells_cap = total;
        if (n_cells) *n_cells = ctx->n_cells;
        prof_resolve(ctx);
        return PCP_OK;
    }
    // The sorted neighbour lists: the area's (nb_list / nb_meta) and the cells' (nb_list_c /
    // nb_meta_c), one region per k_nb_lists block, words as the previous call needed (first
    // guess n x min(n, 4096)), regrown on overflow to the largest block's use x the grid (by
    // area_finish).  The cells go through k_cell_sums_exact first (any order where no order can
    // change the sums); only those it leaves in nb_sel take the ordered lists.  Every buffer is
    // sized before the launches.
    const uint32_t nbb = ctx->nb_blocks > 0 ? (uint32_t)ctx->nb_blocks : (uint32_t)kNbBlocks;
    ctx->area_grid_a = std::min<uint32_t>(npts, nbb);
    ctx->area_grid_c = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(total, nbb));
    ctx->area_npts = npts;
    ctx->area_total = total;
    const uint64_t per_pt = std::min<uint64_t>(npts, 4096);
    const uint64_t guess_a = std::min<uint64_t>((uint64_t)npts * per_pt, ctx->nb_guess_max);
    const uint64_t guess_c = std::min<uint64_t>(std::max<uint64_t>(total, 1) * per_pt, ctx->nb_guess_max);
    PCP_HIP(ctx, ctx->nb_list.ensure(std::max<uint64_t>(guess_a, ctx->nb_need) * 4 + 64));
    PCP_HIP(ctx, ctx->nb_list_c.ensure(std::max<uint64_t>(guess_c, ctx->nb_need_c) * 4 + 64));
    PCP_HIP(ctx, ctx->nb_meta.ensure((size_t)npts * sizeof(uint2) + 64));
    PCP_HIP(ctx, ctx->nb_meta_c.ensure((size_t)total * sizeof(uint2) + 64));
    PCP_HIP(ctx, ctx->nb_sel.ensure(((size_t)total + 2) * sizeof(uint32_t)));
    bool ctl_dirty = !ctx->nb_ctl_zero || !ctx->nb_ctl.p;   // control words not known zero
    PCP_HIP(ctx, ctx->nb_ctl.ensure(64));
    ctx->nb_ctl_zero = false;   // set again once k_nb_sums<true> has cleared them
    // nb_pts: the points by input index, then their normals as float4 (the sums' records)
    PCP_HIP(ctx, ctx->nb_pts.ensure(2 * n * sizeof(float4) + 64));
    uint32_t *ctl = ctx->nb_ctl.as<uint32_t>();
    uint32_t *sel = ctx->nb_sel.as<uint32_t>();
    hipStream_t st = ctx->stream;
    // deferred: the rest on the side stream, forked here (the indices above are its inputs) and
    // joined by the scoring / area_finish.  Everything it writes is its own (nb_*, area_nrm,
    // cells_*, lat_flags, area_host) and nothing on ctx->stream reads those before the join
    // (not when the raw records sit in ctx->stage: a large area's, DMA'd there, which the next
    // upload on ctx->stream may overwrite while k_area_prep still reads them)
    const bool side = defer && ctx->area_side && (paired || raw != ctx->stage.as<unsigned char>());
    if (side) {
        if (!ctx->area_stream)
            PCP_HIP(ctx, hipStreamCreateWithFlags(&ctx->area_stream, hipStreamNonBlocking));
        if (!ctx->area_fork_ev)
            PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->area_fork_ev, hipEventDisableTiming));
        if (!ctx->area_join_ev)
            PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->area_join_ev, hipEventDisableTiming));
        PCP_HIP(ctx, hipEventRecord(ctx->area_fork_ev, st));
        PCP_HIP(ctx, hipStreamWaitEvent(ctx->area_stream, ctx->area_fork_ev, 0));
        st = ctx->area_stream;
    }
    // the control words are zero: cleared by the previous call's last k_nb_sums<true> (or, on a
    // fresh buffer, by this memset)
    if (ctl_dirty) PCP_HIP(ctx, hipMemsetAsync(ctl, 0, 32, st));
    // first: the input points by input index for the sums' gathers, the non-finite points' NaN
    // normals (k_area_prep is the raw records' last reader; the exact kernels never write those
    // entries, so a rerun keeps them), and sel's count cleared
    if (!paired) {   // (paired: done by the pair's extraction; sel's count by k_lattice_compact)
        hipLaunchKernelGGL(k_area_prep, dim3((unsigned)((n + kXT - 1) / kXT)), dim3(kXT), 0, st,
                           rin, ctx->nb_pts.as<float4>(), ctx->area_nrm.as<float>(), sel);
        PCP_CHECK_LAUNCH(ctx);
        pin_release(ctx, st);
    }
    nb_area_launch(ctx, st);
    PCP_CHECK_LAUNCH(ctx);
    if (int rcl = lattice(st)) return rcl;
    nb_cells_launch(ctx, st);
    PCP_CHECK_LAUNCH(ctx);
    if (side) {
        PCP_HIP(ctx, hipEventRecord(ctx->area_join_ev, st));
        ctx->area_forked = true;
    }
    ctx->cells_cap = total;
    ctx->area_pending = true;
    if (defer) {   // the count (<= cells_cap) is settled by the next call that needs it
        if (n_cells) *n_cells = total;
        return PCP_OK;
    }
    if ((rc = area_finish(ctx))) return rc;
    if (n_cells) *n_cells = ctx->n_cells;
    return PCP_OK;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_set_excavation_area(pcp_ctx *ctx, const pcp_cloud_view *area, double grid_resolution,
                            int32_t vertical_layers, double grid_bbox[6], uint64_t *n_cells) {
    return area_setup_from(ctx, area, grid_resolution, vertical_layers, grid_bbox, n_cells, false,
                           nullptr);
}

int pcp_set_excavation_area_async(pcp_ctx *ctx, const pcp_cloud_view *area,
                                  double grid_resolution, int32_t vertical_layers,
                                  double grid_bbox[6], uint64_t *cells_cap) {
    return area_setup_from(ctx, area, grid_resolution, vertical_layers, grid_bbox, cells_cap, true,
                           nullptr);
}

int pcp_cells_count(pcp_ctx *ctx, uint64_t *n_cells) {
    if (!ctx) return PCP_E_INVALID;
    if (!n_cells) return set_err(ctx, PCP_E_INVALID, "pcp_cells_count: null n_cells");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (int rc = area_finish(ctx)) return rc;
    *n_cells = ctx->n_cells;
    return PCP_OK;
}

int pcp_get_cells(pcp_ctx *ctx, double *xyz, float *normals, uint64_t cap, uint64_t *n_cells) {
    if (!ctx) return PCP_E_INVALID;
    if (!n_cells) return set_err(ctx, PCP_E_INVALID, "pcp_get_cells: null n_cells");
    if (int rc = area_finish(ctx)) return rc;
    *n_cells = ctx->n_cells;
    if (ctx->n_cells > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_get_cells: %llu cells, cap %llu",
                       (unsigned long long)ctx->n_cells, (unsigned long long)cap);
    if (!ctx->n_cells) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (xyz)
        PCP_HIP(ctx, hipMemcpyAsync(xyz, ctx->cells_xyz.p, ctx->n_cells * 3 * sizeof(double),
                                    hipMemcpyDeviceToHost, ctx->stream));
    if (normals)
        PCP_HIP(ctx, hipMemcpyAsync(normals, ctx->cells_nrm.p, ctx->n_cells * 3 * sizeof(float),
                                    hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_get_area_normals(pcp_ctx *ctx, float *normals, uint64_t cap, uint64_t *n) {
    if (!ctx) return PCP_E_INVALID;
    if (!n) return set_err(ctx, PCP_E_INVALID, "pcp_get_area_normals: null n");
    if (int rc = area_finish(ctx)) return rc;
    *n = ctx->area_n;
    if (ctx->area_n > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_get_area_normals: %llu points, cap %llu",
                       (unsigned long long)ctx->area_n, (unsigned long long)cap);
    if (!ctx->area_n || !normals) return PCP_OK;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, hipMemcpyAsync(normals, ctx->area_nrm.p, ctx->area_n * 3 * sizeof(float),
                                hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

#ifdef PCP_STAMPS
// diagnostic build only: the stamps of the last k_nb_lists<false> (which 0) / k_nb_sums<false>
// (which 1) launches: [block][query round][phase], phase 7 = the list length (sums: the longest)
int pcp_diag_nb_stamps(pcp_ctx *ctx, int which, unsigned long long *out, size_t n) {
    PCP_HIP(ctx, hipDeviceSynchronize());
    const size_t per = (size_t)kNbStampBlocks * kNbStampQ * kNbStampPh;
    n = std::min<size_t>(n, per);
    PCP_HIP(ctx, hipMemcpyFromSymbol(out, HIP_SYMBOL(g_nb_stamps), n * 8,
                                     (size_t)(which ? 1 : 0) * per * 8, hipMemcpyDeviceToHost));
    return PCP_OK;
}
#endif

}  // extern "C"
