// pcp_carve.hip -- excavated_surface_generator.cpp (ExcavationTerrainGenerator) on gfx950:
// matchedCloudCallback (:259-326) -> processExcavation (:451-485) + generateExcavatedSurface
// (:487-584) + generateExcavationArea (:350-455).
//
// Every getTerrainHeight (:183-226) -- which the reference answers by building a fresh
// KdTreeFLANN over the whole cloud, once per input point -- is a GPU query against ONE uniform
// grid of the input (r = terrain_search_radius):
//   3-D radius search from (x, y, 0) with FLANN's float predicate, the 2-D distance filter in
//   double, the mean z (double-double sum: the reference's sequential double sum, exact for
//   these magnitudes), else the nearest point's z (brute force, smallest float distance, lowest
//   index on a tie), else 0.
// Per input point, the pit test needs a height only where the point can be inside a box
// widened by the largest slope offset; all other points are kept without a query (exact).
// The pose / lattice / wall geometry is O(lattice) double arithmetic on the host (glibc), the
// reference's own expressions.
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "pcp_internal.hpp"
#include "pcp_stencil.hpp"

namespace pcp {

constexpr int kCT = 256;
constexpr int kKeepItems = 16;   // most points per thread of a keep tile (large clouds)
// points per thread of the keep tiles for n points: message-sized clouds (C5: ~10 k) get at
// least kKeepMinTiles tiles -- the emit is a chain of per-item load rounds, and 3 tiles of 16
// items left it latency-bound (21 us)
constexpr int kKeepMinTiles = 64;
static inline int keep_items(uint64_t n) {
    const uint64_t per = (n + (uint64_t)kCT * kKeepMinTiles - 1) / ((uint64_t)kCT * kKeepMinTiles);
    return (int)std::min<uint64_t>(std::max<uint64_t>(per, 1), kKeepItems);
}

struct ExcBox {
    double cx, cy, len, wid, min_x, max_x, min_y, max_y;
};

struct CarveArgs {
    const unsigned char *raw;   // the input records (device copy)
    uint64_t n;
    uint32_t step, ox, oy, oz;
    int32_t has_rgb;
    double cx, cy;              // excavation centre (map)
    double cos_my, sin_my;      // cos(-yaw), sin(-yaw), glibc on the host
    double depth, slope_offset;
    ExcBox box[2];
    int32_t nbox;
};

__device__ __forceinline__ void load_p(const CarveArgs &a, uint64_t i, float &x, float &y,
                                       float &z) {
    const unsigned char *p = a.raw + i * a.step;
    x = *reinterpret_cast<const float *>(p + a.ox);
    y = *reinterpret_cast<const float *>(p + a.oy);
    z = *reinterpret_cast<const float *>(p + a.oz);
}

// double-double (TwoSum) accumulation
struct DDs {
    double hi, lo;
};
__device__ __forceinline__ void dds_add(DDs &a, double x) {
    const double s = a.hi + x;
    const double bb = s - a.hi;
    const double err = (a.hi - (s - bb)) + (x - bb);
    a.hi = s;
    a.lo += err;
}

// candidates of the pit test: points inside some box widened by the largest slope offset
// (isInsideExcavationArea's offset is slope_offset * (depth + z_rel) / depth <= slope_offset
// for every z_rel it accepts).  Writes the query (x, y) and the point index.
// Also presets each keep tile's count (tile_pts points per tile) to its size: k_carve_decide
// takes the carved points off, so k_keep_emit finds the kept counts without a counting pass.
__global__ void __launch_bounds__(kCT)
k_carve_cand(CarveArgs a, double2 *__restrict__ qxy, uint32_t *__restrict__ qidx,
             uint32_t *__restrict__ count, uint32_t qbase, uint8_t *__restrict__ removed,
             uint32_t *__restrict__ tcount, uint32_t tile_pts) {
    const uint64_t i = (uint64_t)blockIdx.x * kCT + threadIdx.x;
    bool cand = false;
    float x = 0.f, y = 0.f, z = 0.f;
    if (i < a.n && i % tile_pts == 0)
        tcount[i / tile_pts] = (uint32_t)min((uint64_t)tile_pts, a.n - i);
    if (i < a.n) {
        removed[i] = 0;   // (k_carve_decide sets the carved ones)
        load_p(a, i, x, y, z);
        const double dx = (double)x - a.cx, dy = (double)y - a.cy;
        const double xl = dx * a.cos_my - dy * a.sin_my;
        const double yl = dx * a.sin_my + dy * a.cos_my;
        for (int k = 0; k < a.nbox; ++k)
            if (fabs(xl - a.box[k].cx) <= a.box[k].len / 2.0 + a.slope_offset &&
                fabs(yl - a.box[k].cy) <= a.box[k].wid / 2.0 + a.slope_offset)
                cand = true;
    }
    // one atomic per wave: slots in lane order
    const uint64_t bal = __ballot(cand);
    if (!bal) return;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == __builtin_ctzll(bal)) base = atomicAdd(count, (uint32_t)__popcll(bal));
    base = __shfl(base, __builtin_ctzll(bal), 64);
    if (cand) {
        const uint32_t s = qbase + base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
        qxy[s] = make_double2((double)x, (double)y);
        qidx[s - qbase] = (uint32_t)i;
    }
}

// getTerrainHeight for queries [0, nq): radius part; queries without a valid neighbour go to
// the nearest-point list
__global__ void __launch_bounds__(kCT)
k_heights(GridView g, float r2, double radius, const double2 *__restrict__ qxy,
          const uint32_t *__restrict__ nq_dev, uint32_t nq_fixed, double *__restrict__ h,
          uint32_t *__restrict__ fb_list, uint32_t *__restrict__ fb_count) {
    // one wave per query: the lanes split the stencil's candidate points (a query used to walk
    // hundreds of them on one lane).  The z sum is double-double, exact at these magnitudes, so
    // the lanes' partial sums merge to the same value in any order.
    const uint32_t nq = nq_fixed + (nq_dev ? *nq_dev : 0u);
    const uint32_t q = blockIdx.x * (kCT / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (q >= nq) return;   // uniform per wave
    const double2 xy = qxy[q];
    const float qx = (float)xy.x, qy = (float)xy.y, qz = 0.0f;
    DDs s{0.0, 0.0};
    uint32_t valid = 0;
    uint32_t ix, iy, iz;
    if (g.n_pts && stencil_cell3_f(g, qx, qy, qz, ix, iy, iz)) {
        const uint32_t nx = (uint32_t)g.nx, nxy = nx * (uint32_t)g.ny;
        const uint32_t lin = ix + nx * iy + nxy * iz;
        uint32_t lo4[4], hi4[4];   // the 4 rows' ranges first: 8 independent loads
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t row = lin + (r & 1) * nx + (r >> 1) * nxy;
            lo4[r] = g.start[row];
            hi4[r] = g.start[row + 2];
        }
        for (int r = 0; r < 4; ++r) {
            const uint32_t lo = lo4[r], hi = hi4[r];
            for (uint32_t k = lo + lane; k < hi; k += 64) {
                const P3 p = ld_p3(g.pts, k);
                if (!flann_within(qx, qy, qz, p, r2)) continue;
                const double dx = (double)p.x - xy.x, dy = (double)p.y - xy.y;
                if (sqrt(dx * dx + dy * dy) <= radius) {
                    dds_add(s, (double)p.z);
                    ++valid;
                }
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double oh = __shfl_xor(s.hi, o, 64), ol = __shfl_xor(s.lo, o, 64);
        dds_add(s, oh);
        s.lo += ol;
        valid += __shfl_xor(valid, o, 64);
    }
    if (lane != 0) return;
    if (valid > 0) {
        h[q] = (s.hi + s.lo) / (double)valid;
    } else {
        h[q] = 0.0;   // no point at all (g.n_pts == 0); else replaced by the nearest point's z
        if (g.n_pts) fb_list[atomicAdd(fb_count, 1u)] = q;
    }
}

// nearestKSearch(k = 1) for the listed queries: one block each, brute force over the index
__global__ void __launch_bounds__(kCT)
k_nearest(GridView g, const double2 *__restrict__ qxy, const uint32_t *__restrict__ fb_list,
          const uint32_t *__restrict__ fb_count, double *__restrict__ h) {
    const uint32_t nfb = *fb_count;
    __shared__ float sd[kCT / 64];
    __shared__ uint32_t si[kCT / 64], sk[kCT / 64];
    for (uint32_t f = blockIdx.x; f < nfb; f += gridDim.x) {
        const uint32_t q = fb_list[f];
        const double2 xy = qxy[q];
        const float qx = (float)xy.x, qy = (float)xy.y, qz = 0.0f;
        float bd = INFINITY;
        uint32_t bi = UINT32_MAX, bk = 0;
        // sixteen independent loads in flight per step (the minimum of (distance, index) does not
        // depend on the order the points are taken in)
        constexpr int kU = 16;
        for (uint32_t k0 = threadIdx.x; k0 < g.n_pts; k0 += kU * kCT) {
            float4 pu[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint32_t k = k0 + u * kCT;
                pu[u] = g.pts[k < g.n_pts ? k : k0];
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint32_t k = k0 + u * kCT;
                const float4 p = pu[u];
                const float d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
                float acc = 0.0f;
                acc = acc + d0 * d0;
                acc = acc + d1 * d1;
                acc = acc + d2 * d2;
                const uint32_t oi = __float_as_uint(p.w);
                if (k < g.n_pts && (acc < bd || (acc == bd && oi < bi))) {
                    bd = acc;
                    bi = oi;
                    bk = k;
                }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float od = __shfl_xor(bd, o, 64);
            const uint32_t oi = __shfl_xor(bi, o, 64), ok = __shfl_xor(bk, o, 64);
            if (od < bd || (od == bd && oi < bi)) {
                bd = od;
                bi = oi;
                bk = ok;
            }
        }
        if ((threadIdx.x & 63) == 0) {
            sd[threadIdx.x >> 6] = bd;
            si[threadIdx.x >> 6] = bi;
            sk[threadIdx.x >> 6] = bk;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float d = sd[0];
            uint32_t i = si[0], kk = sk[0];
            for (int w = 1; w < kCT / 64; ++w)
                if (sd[w] < d || (sd[w] == d && si[w] < i)) {
                    d = sd[w];
                    i = si[w];
                    kk = sk[w];
                }
            if (i != UINT32_MAX) h[q] = (double)g.pts[kk].z;
        }
        __syncthreads();
    }
}

// isInsideExcavationArea (:328-348) for each candidate: removed[point] = 1 when inside
__global__ void __launch_bounds__(kCT)
k_carve_decide(CarveArgs a, const uint32_t *__restrict__ qidx, const uint32_t *__restrict__ count,
               const double *__restrict__ h, uint8_t *__restrict__ removed,
               uint32_t *__restrict__ tcount, uint32_t tile_pts) {
    const uint32_t c = blockIdx.x * kCT + threadIdx.x;
    if (c >= *count) return;
    const uint32_t i = qidx[c];
    float x, y, z;
    load_p(a, i, x, y, z);
    const double dx = (double)x - a.cx, dy = (double)y - a.cy;
    const double xl = dx * a.cos_my - dy * a.sin_my;
    const double yl = dx * a.sin_my + dy * a.cos_my;
    const double zr = (double)z - h[c];
    bool inside = false;
    if (!(zr < -a.depth || zr > 0)) {
        const double slope_factor = (a.depth + zr) / a.depth;
        const double cur = a.slope_offset * slope_factor;
        for (int k = 0; k < a.nbox; ++k) {
            const double ddx = xl - a.box[k].cx, ddy = yl - a.box[k].cy;
            const double hl = a.box[k].len / 2.0 + cur, hw = a.box[k].wid / 2.0 + cur;
            if (fabs(ddx) <= hl && fabs(ddy) <= hw) inside = true;
        }
    }
    if (inside) {
        removed[i] = 1;
        atomicSub(&tcount[i / tile_pts], 1u);   // (its keep tile's count, preset by k_carve_cand)
    }
}

struct GenPoint {    // a generated point: position, height query, z recipe (reference order)
    double x, y;
    int32_t q;       // height query index
    int32_t kind;    // 0: h - v   1: (h - depth) + v   (v as below)
    double v;
    float rgb;
};

// the generated records (generateExcavatedSurface / generateExcavationArea) from their height
// queries, in the host's double expressions: record k at out + 2 * (base + k), base = *base_d
// (the kept count, the generated surface goes after the kept points) or 0
__global__ void __launch_bounds__(kCT)
k_gen_emit(const GenPoint *__restrict__ gp, uint32_t ns, uint32_t na, const double *__restrict__ h,
           double depth, const uint32_t *__restrict__ base_d, float4 *__restrict__ out_s,
           float4 *__restrict__ out_a, const uint32_t *__restrict__ ctr,
           uint32_t *__restrict__ sm_host, uint32_t *__restrict__ ctr_next) {
    // the surface records (gp[0 .. ns): after the kept points) and the area's (gp[ns ..)), one
    // launch
    const uint32_t k = blockIdx.x * kCT + threadIdx.x;
    // the counters and the centre height into the pinned landing (in place of two small DMAs);
    // every kernel that writes them ran before this one
    if (sm_host && k == 0) {
        for (int w = 0; w < 4; ++w) sm_host[w] = ctr[w];
        const double h0 = h[0];
        __builtin_memcpy(sm_host + 4, &h0, sizeof(double));
    }
    if (ctr_next && k < 4) ctr_next[k] = 0u;   // the next call's counters (the other set)
    if (k >= ns + na) return;
    const GenPoint g = gp[k];
    const double z = g.kind == 0 ? h[g.q] - g.v : (h[g.q] - depth) + g.v;
    const bool surf = k < ns;
    float4 *out = surf ? out_s : out_a;
    const size_t o = surf ? (size_t)(base_d ? *base_d : 0u) + k : (size_t)(k - ns);
    out[2 * o] = make_float4((float)g.x, (float)g.y, (float)z, 1.0f);
    out[2 * o + 1] = make_float4(g.rgb, 0.0f, 0.0f, 0.0f);
}

// kept points in input order as PointXYZRGB records (x, y, z, 1, rgb, 0, 0, 0)
__global__ void __launch_bounds__(kCT)
k_keep_emit(CarveArgs a, const uint8_t *__restrict__ removed, const uint32_t *__restrict__ counts,
            float4 *__restrict__ out, uint32_t *__restrict__ n_out, int items) {
    const uint64_t base = (uint64_t)blockIdx.x * kCT * items;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __shared__ uint32_t wc[kCT / 64];
    uint32_t pre_t = 0;
    for (uint32_t t = threadIdx.x; t < blockIdx.x; t += kCT) pre_t += counts[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pre_t += __shfl_xor(pre_t, o, 64);
    if (lane == 0) wc[wid] = pre_t;
    __syncthreads();
    uint32_t run = wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_out = run + counts[blockIdx.x];
    for (int j = 0; j < items; ++j) {
        const uint64_t i = base + (uint64_t)j * kCT + threadIdx.x;
        const bool keep = i < a.n && !removed[i];
        const uint64_t bal = __ballot(keep);
        if (lane == 0) wc[wid] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < kCT / 64; ++w) {
            pre += w < wid ? wc[w] : 0u;
            tot += wc[w];
        }
        if (keep) {
            const uint32_t d = run + pre + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            float x, y, z;
            load_p(a, i, x, y, z);
            const float rgb = a.has_rgb ? *reinterpret_cast<const float *>(a.raw + i * a.step + 16)
                                        : 0.0f;
            out[2 * (size_t)d] = make_float4(x, y, z, 1.0f);
            out[2 * (size_t)d + 1] = make_float4(rgb, 0.f, 0.f, 0.f);
        }
        run += tot;
        __syncthreads();
    }
}

// ---- host geometry (the reference's double expressions) ---------------------------------------
static int exc_boxes(const pcp_excavation_params &p, ExcBox b[2]) {
    if (p.l_shape_enabled) {   // getExcavationBoxes (:138-181)
        b[0].cx = 0.0;
        b[0].cy = -p.arm1_length / 2.0;
        b[0].len = p.arm1_width;
        b[0].wid = p.arm1_length;
        b[1].cx = p.arm2_length / 2.0;
        b[1].cy = -p.arm1_length + p.arm2_width / 2.0;
        b[1].len = p.arm2_length;
        b[1].wid = p.arm2_width;
        for (int k = 0; k < 2; ++k) {
            b[k].min_x = b[k].cx - b[k].len / 2.0;
            b[k].max_x = b[k].cx + b[k].len / 2.0;
            b[k].min_y = b[k].cy - b[k].wid / 2.0;
            b[k].max_y = b[k].cy + b[k].wid / 2.0;
        }
        return 2;
    }
    b[0].cx = 0.0;
    b[0].cy = 0.0;
    b[0].len = p.length;
    b[0].wid = p.width;
    b[0].min_x = -p.length / 2.0;
    b[0].max_x = p.length / 2.0;
    b[0].min_y = -p.width / 2.0;
    b[0].max_y = p.width / 2.0;
    return 1;
}

static bool inside_any(double x, double y, const ExcBox *b, int nb) {   // :229-237
    for (int k = 0; k < nb; ++k)
        if (x >= b[k].min_x && x <= b[k].max_x && y >= b[k].min_y && y <= b[k].max_y) return true;
    return false;
}

static bool outer_edge(double x, double y, const ExcBox *b, int nb, double tol) {   // :240-258
    if (!inside_any(x, y, b, nb)) return false;
    bool out = false;
    if (!inside_any(x + tol, y, b, nb)) out = true;
    if (!inside_any(x - tol, y, b, nb)) out = true;
    if (!inside_any(x, y + tol, b, nb)) out = true;
    if (!inside_any(x, y - tol, b, nb)) out = true;
    return out;
}

static float pack_rgb(unsigned r, unsigned g, unsigned b) {
    const uint32_t v = b | (g << 8) | (r << 16) | (255u << 24);
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}

// the carve (pcp_excavate).  xl non-null (pcp_excavate_area_async): the records land in
// ctx->exc_land (pinned, device-readable, kept until the next such call) when they fit, and are
// NOT copied to terrain_out / area_out here -- xl->terr / xl->area point at them and the caller
// copies them out after enqueueing their consumers.  xl->keep (null outputs): the records land
// there whatever their size and stay (pcp_excavate_landed); no capacity or null-output check
struct ExcLand {
    bool keep = false;
    bool landed = false;
    const unsigned char *terr = nullptr, *area = nullptr;
};

static int excavate_impl(pcp_ctx *ctx, const pcp_cloud_view *in, const pcp_excavation_params *p,
                         const pcp_rigid *zx120_base, void *terrain_out, uint64_t terrain_cap,
                         uint64_t *n_terrain, void *area_out, uint64_t area_cap, uint64_t *n_area,
                         double pose_out[4], ExcLand *xl) {
    if (!ctx) return PCP_E_INVALID;
    if (!p || !zx120_base || !n_terrain || !n_area)
        return set_err(ctx, PCP_E_INVALID, "pcp_excavate: null argument");
    ctx->exc_keep_valid = false;   // (exc_land is rewritten below)
    int rc = check_view(ctx, in, "pcp_excavate");
    if (rc) return rc;
    if (!(p->point_density > 0.0) || !(p->depth > 0.0) || !(p->terrain_search_radius > 0.0))
        return set_err(ctx, PCP_E_INVALID, "pcp_excavate: density, depth, radius must be > 0");
    if (in->n >= (1ull << 31)) return set_err(ctx, PCP_E_INVALID, "pcp_excavate: cloud too large");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    ProfScope prof(ctx, PCP_K_EXCAVATE);
    hipStream_t st = ctx->stream;
    // ---- pose: tf2 Transform * (offset_x, offset_y, 0), Matrix3x3::getRPY (solution 1)
    const double qx = zx120_base->q[0], qy = zx120_base->q[1], qz = zx120_base->q[2],
                 qw = zx120_base->q[3];
    const double d = qx * qx + qy * qy + qz * qz + qw * qw;
    const double s = 2.0 / d;
    const double xs = qx * s, ys = qy * s, zs = qz * s;
    const double wx = qw * xs, wy = qw * ys, wz = qw * zs;
    const double xx = qx * xs, xy = qx * ys, xz = qx * zs;
    const double yy = qy * ys, yz = qy * zs, zz = qz * zs;
    const double m[3][3] = {{1.0 - (yy + zz), xy - wz, xz + wy},
                            {xy + wz, 1.0 - (xx + zz), yz - wx},
                            {xz - wy, yz + wx, 1.0 - (xx + yy)}};
    const double ox = p->offset_x, oy = p->offset_y, oz = 0.0;
    const double cx = (m[0][0] * ox + m[0][1] * oy + m[0][2] * oz) + zx120_base->t[0];
    const double cy = (m[1][0] * ox + m[1][1] * oy + m[1][2] * oz) + zx120_base->t[1];
    double yaw = 0.0;
    if (!(std::fabs(m[2][0]) >= 1)) {
        const double pitch = -std::asin(m[2][0]);
        yaw = std::atan2(m[1][0] / std::cos(pitch), m[0][0] / std::cos(pitch));
    }
    ExcBox box[2];
    const int nbox = exc_boxes(*p, box);
    const double slope_rad = p->slope_angle_deg * M_PI / 180.0;
    const double slope_offset = p->depth / std::tan(slope_rad);
    // ---- generated points (surface bottom + walls, area bottom + walls) and their queries
    double mnx = DBL_MAX, mxx = -DBL_MAX, mny = DBL_MAX, mxy = -DBL_MAX;
    for (int k = 0; k < nbox; ++k) {
        mnx = std::fmin(mnx, box[k].min_x);
        mxx = std::fmax(mxx, box[k].max_x);
        mny = std::fmin(mny, box[k].min_y);
        mxy = std::fmax(mxy, box[k].max_y);
    }
    const double dens = p->point_density;
    const int n_x = (int)((mxx - mnx) / dens) + 1;
    const int n_y = (int)((mxy - mny) / dens) + 1;
    const double cyaw = std::cos(yaw), syaw = std::sin(yaw);
    const uint64_t n = in->n;
    // the generated lattice is a function of these alone (the excavation pose and the
    // parameters): an unchanged key reuses the device copy of the last call
    const double key[16] = {p->depth, p->slope_angle_deg, p->offset_x, p->offset_y, dens,
                            (double)p->l_shape_enabled, p->arm1_length, p->arm1_width,
                            p->arm2_length, p->arm2_width, p->width, p->length, cx, cy, yaw, 0.0};
    auto gen_bytes = [n](uint64_t g, uint64_t ns, uint64_t na, size_t &gpb, size_t &qxb) {
        gpb = ((ns + na) * sizeof(GenPoint) + 255) & ~(size_t)255;
        qxb = ((g + n) * sizeof(double2) + 255) & ~(size_t)255;
        return gpb + qxb + na * 32 + 256;
    };
    size_t gpb = 0, qxb = 0;
    bool gen_hit = ctx->carve_gen_ok && std::memcmp(key, ctx->carve_key, sizeof(key)) == 0 &&
                   ctx->carve_gen.cap >= gen_bytes(ctx->carve_G, ctx->carve_nsurf,
                                                   ctx->carve_narea, gpb, qxb);
    std::vector<double2> qv;          // 0: the centre; then the lattice bottoms; then walls
    std::vector<GenPoint> surf, area;
    if (!gen_hit) {
        qv.push_back(make_double2(cx, cy));
        const float rgb_bottom = pack_rgb(0, 139, 0), rgb_slope = pack_rgb(144, 238, 144);
        const float rgb_abot = pack_rgb(255, 255, 0), rgb_aslope = pack_rgb(200, 200, 0);
        const int n_slope = (int)(slope_offset / dens) + 1;
        const int n_depth = (int)(p->depth / dens);
        auto wall_offset = [&](double xl, double yl, double off, double &ofx, double &ofy) {
            ofx = 0.0;
            ofy = 0.0;
            if (!inside_any(xl + dens, yl, box, nbox)) ofx = off;
            else if (!inside_any(xl - dens, yl, box, nbox)) ofx = -off;
            if (!inside_any(xl, yl + dens, box, nbox)) ofy = off;
            else if (!inside_any(xl, yl - dens, box, nbox)) ofy = -off;
        };
        for (int i = 0; i <= n_x; ++i)   // generateExcavatedSurface bottom (:518-535) + area (:367-)
            for (int j = 0; j <= n_y; ++j) {
                const double xl = mnx + i * dens, yl = mny + j * dens;
                if (!inside_any(xl, yl, box, nbox)) continue;
                const double xg = cx + xl * cyaw - yl * syaw;
                const double yg = cy + xl * syaw + yl * cyaw;
                const int q = (int)qv.size();
                qv.push_back(make_double2(xg, yg));
                surf.push_back(GenPoint{xg, yg, q, 0, p->depth, rgb_bottom});   // h - depth
                area.push_back(GenPoint{xg, yg, q, 0, p->depth, rgb_abot});
                if (!outer_edge(xl, yl, box, nbox, dens)) continue;
                for (int k = 1; k < n_depth; ++k) {   // area walls use the lattice point's height
                    const double z_ratio = (double)k / n_depth;
                    double ofx, ofy;
                    wall_offset(xl, yl, slope_offset * z_ratio, ofx, ofy);
                    const double xs2 = xl + ofx, ys2 = yl + ofy;
                    area.push_back(GenPoint{cx + xs2 * cyaw - ys2 * syaw, cy + xs2 * syaw + ys2 * cyaw,
                                            q, 1, k * dens, rgb_aslope});   // (h - depth) + k*dens
                }
            }
        for (int i = 0; i <= n_x; ++i)   // generateExcavatedSurface walls (:538-583)
            for (int j = 0; j <= n_y; ++j) {
                const double xl = mnx + i * dens, yl = mny + j * dens;
                if (!outer_edge(xl, yl, box, nbox, dens)) continue;
                for (int k = 0; k <= n_slope; ++k) {
                    const double z_ratio = (double)k / n_slope;
                    double ofx, ofy;
                    wall_offset(xl, yl, slope_offset * z_ratio, ofx, ofy);
                    const double xs2 = xl + ofx, ys2 = yl + ofy;
                    const double xg = cx + xs2 * cyaw - ys2 * syaw;
                    const double yg = cy + xs2 * syaw + ys2 * cyaw;
                    const int q = (int)qv.size();
                    qv.push_back(make_double2(xg, yg));
                    surf.push_back(GenPoint{xg, yg, q, 0, p->depth * (1.0 - z_ratio), rgb_slope});
                }
            }
    }
    const uint32_t G = gen_hit ? ctx->carve_G : (uint32_t)qv.size();
    const uint64_t nsurf = gen_hit ? ctx->carve_nsurf : surf.size();
    const uint64_t narea = gen_hit ? ctx->carve_narea : area.size();
    // ---- index of the input (radius = terrain_search_radius); the raw records stay staged
    // (build_index's pinned slot or ctx->stage) for the per-point passes below, the slot held
    // until the last of them is enqueued
    // (DMA'd, not read in place: three passes below re-read the records, which over the host
    // link cost more than the copy -- k_keep_emit 16 -> 36 us measured)
    const unsigned char *raw = nullptr;
    unsigned char *raw_copy = nullptr;
    if (n) {
        const size_t raw_b = n * (size_t)in->point_step;
        PCP_HIP(ctx, ctx->stage.ensure(raw_b));
        // composed (xl): a view into the merger's landing (pcp_filter_merge_landed) is pinned,
        // device-readable memory -- copied into ctx->stage by the index's extraction on its way
        // through (no copy launch, no host staging copy; the non-composed call may regrow that
        // landing for its own records before the copy ran: staged)
        const uintptr_t d0 = reinterpret_cast<uintptr_t>(in->data),
                        l0 = reinterpret_cast<uintptr_t>(ctx->tc_host.p);
        if (xl && ctx->tc_host.p && d0 >= l0 && d0 + raw_b <= l0 + ctx->tc_host.cap) {
            raw = static_cast<const unsigned char *>(in->data);
            raw_copy = ctx->stage.as<unsigned char>();
            if (!ctx->carve_fuse_copy) {   // (A/B: the copy launch first)
                if (int rc0 = copy_pinned_async(ctx, raw_copy, raw, raw_b, st)) return rc0;
                raw = raw_copy;
                raw_copy = nullptr;
            }
        } else {
            if (int rc0 = upload_async(ctx, ctx->stage.p, in->data, raw_b, st)) return rc0;
            raw = ctx->stage.as<unsigned char>();
        }
    }
    if ((rc = build_index(ctx, ctx->carve, *in, p->terrain_search_radius, false, false, &raw,
                          raw_copy)))
        return rc;
    const GridView g = ctx->carve.view();
    CarveArgs a{};
    a.raw = raw;
    a.n = n;
    a.step = in->point_step;
    a.ox = in->off_x;
    a.oy = in->off_y;
    a.oz = in->off_z;
    a.has_rgb = in->point_step >= 20 ? 1 : 0;
    a.cx = cx;
    a.cy = cy;
    a.cos_my = std::cos(-yaw);
    a.sin_my = std::sin(-yaw);
    a.depth = p->depth;
    a.slope_offset = slope_offset;
    a.box[0] = box[0];
    a.box[1] = box[1];
    a.nbox = nbox;
    // device scratch: candidate indices (n), heights, fallback list, removed flags, tile
    // counts, kept records (the queries live in carve_gen)
    const uint64_t nq_max = G + n;
    const int kitems = keep_items(n);
    const uint32_t nb = (uint32_t)((n + (uint64_t)kCT * kitems - 1) / ((uint64_t)kCT * kitems));
    const size_t qb = 0;
    const size_t ib = (n * 4 + 256) & ~(size_t)255;
    const size_t hb = (nq_max * 8 + 255) & ~(size_t)255;
    const size_t fb = (nq_max * 4 + 256) & ~(size_t)255;
    const size_t rb = (n + 256) & ~(size_t)255;
    const size_t cb = ((size_t)(nb + 1) * 4 + 256) & ~(size_t)255;
    PCP_HIP(ctx, ctx->carve_buf.ensure(qb + ib + hb + fb + rb + cb + 256));
    char *base = ctx->carve_buf.as<char>();
    uint32_t *qidx = reinterpret_cast<uint32_t *>(base + qb);
    double *h = reinterpret_cast<double *>(base + qb + ib);
    uint32_t *fb_list = reinterpret_cast<uint32_t *>(base + qb + ib + hb);
    uint8_t *removed = reinterpret_cast<uint8_t *>(base + qb + ib + hb + fb);
    uint32_t *tcount = reinterpret_cast<uint32_t *>(base + qb + ib + hb + fb + rb);
    // the counters: this call's set of two (cleared by the previous call's k_gen_emit, or here)
    const size_t cap0 = ctx->carve_ctr.cap;
    PCP_HIP(ctx, ctx->carve_ctr.ensure(64));
    if (ctx->carve_ctr.cap != cap0) ctx->carve_ctr_clean[0] = ctx->carve_ctr_clean[1] = false;
    const int cs = ctx->carve_ctr_sel;
    uint32_t *ctr = ctx->carve_ctr.as<uint32_t>() + 4 * cs;
    uint32_t *ctr_next = ctx->carve_ctr.as<uint32_t>() + 4 * (1 - cs);
    // the records: straight into pinned memory for message-sized results (the kernels store
    // them there, no D2H copy), else a device buffer copied out
    const size_t land_b = (n + nsurf + narea) * 32;
    const bool land = (ctx->zc_in && land_b <= kPinDirectMax * 8) || (xl && xl->keep);
    float4 *kept;
    if (land && xl) {
        PCP_HIP(ctx, ctx->exc_land.ensure(land_b + 256));
        kept = ctx->exc_land.as<float4>();
    } else if (land) {
        ctx->fm_land_valid = false;   // (tc_host rewritten)
        PCP_HIP(ctx, ctx->tc_host.ensure(land_b + 256));
        kept = ctx->tc_host.as<float4>();
    } else {
        PCP_HIP(ctx, ctx->out_d.ensure((n + nsurf) * 32 + 64));
        kept = ctx->out_d.as<float4>();
    }
    const size_t gen_need = gen_bytes(G, nsurf, narea, gpb, qxb);
    if (!gen_hit) {   // surface + area records and the generated queries: one DMA
        ctx->carve_gen_ok = false;
        PCP_HIP(ctx, ctx->carve_gen.ensure(gen_need));
        const HostPiece pc[3] = {{0, surf.data(), nsurf * sizeof(GenPoint)},
                                 {nsurf * sizeof(GenPoint), area.data(), narea * sizeof(GenPoint)},
                                 {gpb, qv.data(), G * sizeof(double2)}};
        if (int rc0 = upload_pieces(ctx, ctx->carve_gen.p, pc, 3, gpb + G * sizeof(double2), st))
            return rc0;
        std::memcpy(ctx->carve_key, key, sizeof(key));
        ctx->carve_G = G;
        ctx->carve_nsurf = nsurf;
        ctx->carve_narea = narea;
        ctx->carve_gen_ok = true;
    }
    char *gbase = ctx->carve_gen.as<char>();
    GenPoint *gp = reinterpret_cast<GenPoint *>(gbase);
    double2 *qxy = reinterpret_cast<double2 *>(gbase + gpb);
    float4 *area_d = land ? kept + 2 * (n + nsurf) : reinterpret_cast<float4 *>(gbase + gpb + qxb);
    if (!ctx->carve_ctr_clean[cs]) PCP_HIP(ctx, hipMemsetAsync(ctr, 0, 16, st));
    ctx->carve_ctr_clean[cs] = false;
    ctx->carve_ctr_sel = 1 - cs;
    const float r2 = (float)(p->terrain_search_radius * p->terrain_search_radius);
    const unsigned gn = (unsigned)((n + kCT - 1) / kCT);
    if (n) {
        hipLaunchKernelGGL(k_carve_cand, dim3(gn), dim3(kCT), 0, st, a, qxy, qidx, ctr, G, removed,
                           tcount, (uint32_t)kCT * (uint32_t)kitems);
        PCP_CHECK_LAUNCH(ctx);
    }
    const unsigned gq = (unsigned)((nq_max + kCT / 64 - 1) / (kCT / 64));   // a wave per query
    hipLaunchKernelGGL(k_heights, dim3(gq), dim3(kCT), 0, st, g, r2, p->terrain_search_radius,
                       (const double2 *)qxy, (const uint32_t *)ctr, G, h, fb_list, ctr + 1);
    PCP_CHECK_LAUNCH(ctx);
    // (one block per fallback query, up to 4,096 at once: the count is on the device, the
    // blocks past it return at once)
    hipLaunchKernelGGL(k_nearest, dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nq_max, 4096))),
                       dim3(kCT), 0, st, g, (const double2 *)qxy,
                       (const uint32_t *)fb_list, (const uint32_t *)(ctr + 1), h);
    PCP_CHECK_LAUNCH(ctx);
    if (n) {
        hipLaunchKernelGGL(k_carve_decide, dim3(gn), dim3(kCT), 0, st, a, (const uint32_t *)qidx,
                           (const uint32_t *)ctr, (const double *)(h + G), removed, tcount,
                           (uint32_t)kCT * (uint32_t)kitems);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_keep_emit, dim3(nb), dim3(kCT), 0, st, a, (const uint8_t *)removed,
                           (const uint32_t *)tcount, kept, ctr + 2, kitems);
        PCP_CHECK_LAUNCH(ctx);
    }
    pin_release(ctx, st);   // k_keep_emit was the raw records' last reader
    // the generated surface (after the kept points) and area records, on the device
    PCP_HIP(ctx, ctx->small_host.ensure(4096));
    char *sm = ctx->small_host.as<char>();
    // landed: the first k_gen_emit stores the counters and the centre height too
    uint32_t *sm_k = land ? reinterpret_cast<uint32_t *>(sm) : nullptr;
    if (nsurf + narea) {
        hipLaunchKernelGGL(k_gen_emit, dim3((unsigned)((nsurf + narea + kCT - 1) / kCT)), dim3(kCT),
                           0, st, (const GenPoint *)gp, (uint32_t)nsurf, (uint32_t)narea,
                           (const double *)h, p->depth, n ? (const uint32_t *)(ctr + 2) : nullptr,
                           kept, area_d, (const uint32_t *)ctr, sm_k, ctr_next);
        PCP_CHECK_LAUNCH(ctx);
        ctx->carve_ctr_clean[1 - cs] = true;
        sm_k = nullptr;
    }
    // the kept count and the centre height land in pinned memory; when the caller's buffers
    // hold the worst case (n kept + the surface, pcp_excavate_bounds), the records go out in the
    // same round trip: one synchronisation for the call
    if (!land || sm_k) {   // not stored by a kernel above
        PCP_HIP(ctx, hipMemcpyAsync(sm, ctr, 16, hipMemcpyDeviceToHost, st));
        PCP_HIP(ctx, hipMemcpyAsync(sm + 16, h, sizeof(double), hipMemcpyDeviceToHost, st));
    }
    const bool one_trip = !land && terrain_out && terrain_cap >= n + nsurf &&
                          (area_out || !narea) && area_cap >= narea;
    if (one_trip) {
        if (n + nsurf)
            PCP_HIP(ctx, hipMemcpyAsync(terrain_out, kept, (n + nsurf) * 32, hipMemcpyDeviceToHost,
                                        st));
        if (narea)
            PCP_HIP(ctx, hipMemcpyAsync(area_out, area_d, narea * 32, hipMemcpyDeviceToHost, st));
    }
    PCP_HIP(ctx, hipStreamSynchronize(st));
    uint32_t cnt[4];
    std::memcpy(cnt, sm, 16);
    double h0;
    std::memcpy(&h0, sm + 16, sizeof(double));
    const uint64_t nkept = n ? cnt[2] : 0;
    if (pose_out) {
        pose_out[0] = cx;
        pose_out[1] = cy;
        pose_out[2] = h0;
        pose_out[3] = yaw;
    }
    *n_terrain = nkept + nsurf;
    *n_area = narea;
    const bool keep = xl && xl->keep;
    if (!keep && (*n_terrain > terrain_cap || *n_area > area_cap)) {
        prof_resolve(ctx);
        return set_err(ctx, PCP_E_CAPACITY, "pcp_excavate: need %llu / %llu records, cap %llu / %llu",
                       (unsigned long long)*n_terrain, (unsigned long long)*n_area,
                       (unsigned long long)terrain_cap, (unsigned long long)area_cap);
    }
    if (!keep && ((*n_terrain && !terrain_out) || (*n_area && !area_out)))
        return set_err(ctx, PCP_E_INVALID, "pcp_excavate: null output");
    if (land && xl) {   // the caller copies them out
        xl->landed = true;
        xl->terr = reinterpret_cast<const unsigned char *>(kept);
        xl->area = reinterpret_cast<const unsigned char *>(area_d);
    } else if (land) {   // the records sit in pinned memory already
        if (*n_terrain) host_copy(ctx, terrain_out, kept, *n_terrain * 32);
        if (narea) host_copy(ctx, area_out, area_d, narea * 32);
    } else if (!one_trip) {   // exact-size buffers: the records follow the sizes
        if (*n_terrain)
            PCP_HIP(ctx, hipMemcpyAsync(terrain_out, kept, *n_terrain * 32, hipMemcpyDeviceToHost,
                                        st));
        if (narea)
            PCP_HIP(ctx, hipMemcpyAsync(area_out, area_d, narea * 32, hipMemcpyDeviceToHost, st));
        PCP_HIP(ctx, hipStreamSynchronize(st));
    }
    prof_resolve(ctx);
    return PCP_OK;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_excavate(pcp_ctx *ctx, const pcp_cloud_view *in, const pcp_excavation_params *p,
                 const pcp_rigid *zx120_base, void *terrain_out, uint64_t terrain_cap,
                 uint64_t *n_terrain, void *area_out, uint64_t area_cap, uint64_t *n_area,
                 double pose_out[4]) {
    return excavate_impl(ctx, in, p, zx120_base, terrain_out, terrain_cap, n_terrain, area_out,
                         area_cap, n_area, pose_out, nullptr);
}

int pcp_excavate_area_async(pcp_ctx *ctx, const pcp_cloud_view *in,
                            const pcp_excavation_params *p, const pcp_rigid *zx120_base,
                            void *terrain_out, uint64_t terrain_cap, uint64_t *n_terrain,
                            void *area_out, uint64_t area_cap, uint64_t *n_area,
                            double pose_out[4], double grid_resolution, int32_t vertical_layers,
                            double grid_bbox[6], uint64_t *n_cells) {
    if (!ctx) return PCP_E_INVALID;
    if (!n_cells) return set_err(ctx, PCP_E_INVALID, "pcp_excavate_area_async: null argument");
    // a setup still in flight may read the landing this carve rewrites
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (int rc = area_finish(ctx)) return rc;
    ExcLand xl;
    xl.keep = !terrain_out && !area_out;   // the records stay landed (pcp_excavate_landed)
    if (int rc = excavate_impl(ctx, in, p, zx120_base, terrain_out, terrain_cap, n_terrain,
                               area_out, area_cap, n_area, pose_out, &xl))
        return rc;
    // the carve's records as the two messages' views (xyz at 0 / 4 / 8 of 32-byte records)
    auto rec_view = [](const void *d, uint64_t n) {
        pcp_cloud_view v{};
        v.data = n ? d : nullptr;
        v.n = n;
        v.point_step = 32;
        v.off_x = 0;
        v.off_y = 4;
        v.off_z = 8;
        return v;
    };
    if (!xl.landed) {   // records past the landing's size: the two calls over the copies
        const pcp_cloud_view va = rec_view(area_out, *n_area), vt = rec_view(terrain_out, *n_terrain);
        if (int rc = pcp_set_excavation_area_async(ctx, &va, grid_resolution, vertical_layers,
                                                   grid_bbox, n_cells))
            return rc;
        return pcp_set_terrain(ctx, &vt);
    }
    // the landed records feed the setup and the terrain index in place (device-readable pinned
    // memory: no staging copy, no upload); the messages' copies follow the launches
    const pcp_cloud_view va = rec_view(xl.area, *n_area), vt = rec_view(xl.terr, *n_terrain);
    if (int rc = area_setup_from(ctx, &va, grid_resolution, vertical_layers, grid_bbox, n_cells,
                                 true, xl.area))
        return rc;
    if (int rc = set_terrain_from(ctx, &vt, xl.terr)) return rc;
    if (xl.keep) {   // read in place by the caller (its own consumers enqueued first)
        ctx->exc_keep_terr = xl.terr;
        ctx->exc_keep_area = xl.area;
        ctx->exc_keep_valid = true;
        return PCP_OK;
    }
    if (*n_terrain) host_copy(ctx, terrain_out, xl.terr, *n_terrain * 32);
    if (*n_area) host_copy(ctx, area_out, xl.area, *n_area * 32);
    return PCP_OK;
}

int pcp_excavate_landed(pcp_ctx *ctx, const void **terrain, const void **area) {
    if (!ctx) return PCP_E_INVALID;
    if (!ctx->exc_keep_valid)
        return set_err(ctx, PCP_E_STATE, "pcp_excavate_landed: no pcp_excavate_area_async result "
                                         "left in place");
    if (terrain) *terrain = ctx->exc_keep_terr;
    if (area) *area = ctx->exc_keep_area;
    return PCP_OK;
}

int pcp_excavate_bounds(const pcp_excavation_params *p, uint64_t n_in, uint64_t *terrain_cap,
                        uint64_t *area_cap) {
    if (!p || !terrain_cap || !area_cap || !(p->point_density > 0.0) || !(p->depth > 0.0))
        return PCP_E_INVALID;
    ExcBox box[2];
    const int nbox = exc_boxes(*p, box);
    double mnx = DBL_MAX, mxx = -DBL_MAX, mny = DBL_MAX, mxy = -DBL_MAX;
    for (int k = 0; k < nbox; ++k) {
        mnx = std::fmin(mnx, box[k].min_x);
        mxx = std::fmax(mxx, box[k].max_x);
        mny = std::fmin(mny, box[k].min_y);
        mxy = std::fmax(mxy, box[k].max_y);
    }
    const double dens = p->point_density;
    const uint64_t lat = (uint64_t)((int)((mxx - mnx) / dens) + 2) * (uint64_t)((int)((mxy - mny) / dens) + 2);
    const double slope_offset = p->depth / std::tan(p->slope_angle_deg * M_PI / 180.0);
    const uint64_t n_slope = (uint64_t)std::max(0, (int)(slope_offset / dens) + 1);
    const uint64_t n_depth = (uint64_t)std::max(0, (int)(p->depth / dens));
    *terrain_cap = n_in + lat * (n_slope + 2);
    *area_cap = lat * (n_depth + 1);
    return PCP_OK;
}

}  // extern "C"
