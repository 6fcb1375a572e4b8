// pcp_vlidar.hip -- virtual_lidar.cpp hot path on gfx950: candidate generation, per
// (pose, cell) visibility scoring, and the dense ray-fan occlusion march.
//
// Numerics: compiled with -ffp-contract=off (no FMA) so every double/float operation
// rounds exactly as the reference's SSE2 build.  The radius predicate restates FLANN's
// L2_Simple<float> (x, y, z accumulated in order, strict '<' against float(r*r)).
#pragma clang fp contract(off)

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include <hip/hip_ext.h>

#include "pcp_crmath.h"
#include "pcp_internal.hpp"
#include "pcp_stencil.hpp"

namespace pcp {

constexpr int kT = 256;
constexpr int kStepLds = 256;   // step tables up to this long are read from LDS (fan, cells)
#ifndef PCP_CELL_PROBES
// z-band probes issued per round in the cell-scoring march (build knob; 4 measured 130 vs 132
// us per 256-pose k_score_cells: that march is not probe-latency bound)
#define PCP_CELL_PROBES 1
#endif

// Lower-corner cell of the 2x2x2 stencil of a query (q - r - margin), as one linear index.
// False when the corner falls outside [0, n-2]^3: then the stencil holds only padding /
// outside cells and no point can be within r (exact skip, see DESIGN.md "Terrain index").
__device__ __forceinline__ bool stencil_cell(const GridView &g, float qx, float qy, float qz,
                                             uint32_t &lin) {
    uint32_t ix, iy, iz;
    const bool ok = stencil_cell3_fb(g, qx, qy, qz, ix, iy, iz);
    lin = ix + (uint32_t)g.nx * (iy + (uint32_t)g.ny * iz);
    return ok;
}

// Exact point tests of an occupied stencil: 2 x 2 rows (y, z) x 2 cells (x) = 8 runs.  Points
// of a cell are sorted by descending z, so a run ends at the first point with dz = qz - pz >= 0
// and fl(dz*dz) >= r2: FLANN's accumulator ((0 + dx^2) + dy^2) + dz^2 is >= fl(dz^2) (adding
// non-negative floats never decreases), and every later point of the run has a larger dz, so
// none of them can be within r (exact).
// Latency shape: round 1 = the 4 rows' directory entries (one 12-byte load per row: cells c,
// c+1 and the end of c+1); round 2 = the first point of all 8 runs (independent loads; an empty
// run reads point 0, one line shared by every such lane); only runs that continue are walked,
// 2 points per step.  Loads use 32-bit offsets from the kernel-argument bases.
template <bool STATS>
__device__ __forceinline__ bool scan_stencil(const GridView &g, uint32_t lin, float qx, float qy,
                                             float qz, float r2, uint32_t *cnt) {
    const uint32_t nx = (uint32_t)g.nx, nxy = nx * (uint32_t)g.ny;
    uint32_t b[4][3];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const U3 u = ld_u3o(g.start, lin + (r & 1) * nx + (r >> 1) * nxy);
        b[r][0] = u.a;
        b[r][1] = u.b;
        b[r][2] = u.c;
    }
    P3 f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t k = b[i >> 1][i & 1];
        f[i] = ld_p3o(g.pts, k < b[i >> 1][(i & 1) + 1] ? k : 0u);
    }
    uint32_t live = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t k = b[i >> 1][i & 1], e = b[i >> 1][(i & 1) + 1];
        if (k < e) {
            if (STATS) cnt[2] += 1;
            if (flann_within(qx, qy, qz, f[i], r2)) return true;
            const float dz = qz - f[i].z;
            if (!(dz >= 0.0f && dz * dz >= r2) && k + 1 < e) live |= 1u << i;
        }
    }
    if (!live) return false;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (!(live & (1u << i))) continue;
        const uint32_t e = b[i >> 1][(i & 1) + 1];
        for (uint32_t k = b[i >> 1][i & 1] + 1; k < e; k += 2) {
            const P3 p0 = ld_p3o(g.pts, k);
            const P3 p1 = ld_p3o(g.pts, min(k + 1, e - 1));
            if (STATS) cnt[2] += 1;
            if (flann_within(qx, qy, qz, p0, r2)) return true;
            float dz = qz - p0.z;
            if (dz >= 0.0f && dz * dz >= r2) break;
            if (k + 1 >= e) break;
            if (STATS) cnt[2] += 1;
            if (flann_within(qx, qy, qz, p1, r2)) return true;
            dz = qz - p1.z;
            if (dz >= 0.0f && dz * dz >= r2) break;
        }
    }
    return false;
}

// The same test over the block-major copy: the block's points are one run in descending z,
// so one directory load, then one point per step until a point lies r below q (exact: every
// later point is lower still) -- a single early exit instead of one per cell.  (2, 3 or 4
// independent loads per step measured 1-2 % slower: the loads past the exit are wasted on the
// bound vector-memory path.)
#ifndef PCP_BLK_STEP
#define PCP_BLK_STEP 1   // block-walk points per step (build knob)
#endif
// a * b + c for a, b < 2^24 as one full-rate v_mad_u32_u24 (the compiler otherwise picks the
// 64-bit multi-pass v_mad_u64_u32)
__device__ __forceinline__ uint32_t mad_u24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// a z-descending run pts[k0 .. e): the walk of one block (or one fine window)
template <bool STATS>
__device__ __forceinline__ bool scan_run(const float4 *pts, uint32_t k0, uint32_t e, float qx,
                                         float qy, float qz, float r2, uint32_t *cnt) {
    for (uint32_t k = k0; k < e; k += PCP_BLK_STEP) {
        P3 p[PCP_BLK_STEP];   // independent loads (the tail repeats the last entry)
#pragma unroll
        for (int i = 0; i < PCP_BLK_STEP; ++i) p[i] = ld_p3o(pts, min(k + i, e - 1));
#pragma unroll
        for (int i = 0; i < PCP_BLK_STEP; ++i) {
            if (i > 0 && k + i >= e) return false;
            if (STATS) cnt[2] += 1;
            if (flann_within(qx, qy, qz, p[i], r2)) return true;
            const float dz = qz - p[i].z;
            if (dz >= 0.0f && dz * dz >= r2) return false;
        }
    }
    return false;
}

// the packed (12-byte) entries' walk: the same test on x, y, z at k * 12
template <bool STATS>
__device__ __forceinline__ bool scan_window3(const float *pts, uint32_t k, float qx, float qy,
                                             float qz, float r2, float rexit, uint32_t *cnt) {
    bool within, stop;
    do {
        const float *f = reinterpret_cast<const float *>(reinterpret_cast<const char *>(pts) +
                                                         ((k << 3) + (k << 2)));
        const P3 p = P3{f[0], f[1], f[2]};
        ++k;
        if (STATS) cnt[2] += 1;
#ifdef PCP_WALK_CENSUS
        if (STATS && p.z - qz >= rexit) cnt[3] += 1;   // an entry r above q: a later start skips it
#endif
        within = flann_within(qx, qy, qz, p, r2);
        stop = within | (qz - p.z >= rexit);
    } while (!stop);
    return within;
}

// a fine window's walk from k: z-descending, ended by the window's sentinel (never within r,
// always r below), so no end index; dz >= rexit is FLANN's "fl(dz^2) >= r2" as one compare
template <bool STATS>
__device__ __forceinline__ bool scan_window(const float4 *pts, uint32_t k, float qx, float qy,
                                            float qz, float r2, float rexit, uint32_t *cnt) {
    bool within, stop;
    do {   // one exit condition: simple exec-mask bookkeeping per step
        const P3 p = ld_p3o(pts, k++);
        if (STATS) cnt[2] += 1;
#ifdef PCP_WALK_CENSUS
        if (STATS && p.z - qz >= rexit) cnt[3] += 1;
#endif
        within = flann_within(qx, qy, qz, p, r2);
        stop = within | (qz - p.z >= rexit);
    } while (!stop);
    return within;
}

template <bool STATS>
__device__ __forceinline__ bool scan_block(const GridView &g, uint32_t lin, float qx, float qy,
                                           float qz, float r2, uint32_t *cnt) {
    const uint2 se = ld_u2o(g.bstart, lin);
    return scan_run<STATS>(g.bpts, se.x, se.y, qx, qy, qz, r2, cnt);
}

template <bool STATS>
__device__ __forceinline__ bool scan_corner(const GridView &g, uint32_t lin, float qx, float qy,
                                            float qz, float r2, uint32_t *cnt) {
    if (g.bpts) return scan_block<STATS>(g, lin, qx, qy, qz, r2, cnt);
    return scan_stencil<STATS>(g, lin, qx, qy, qz, r2, cnt);
}

// KdTreeFLANN::radiusSearch(q, r) > 0 for r <= the index's stencil radius.
__device__ __forceinline__ bool stencil_any(const GridView &g, float qx, float qy, float qz,
                                            float r2) {
    uint32_t lin;
    if (!stencil_cell(g, qx, qy, qz, lin)) return false;
    if (!((ld_u32o(g.occ2, lin >> 5) >> (lin & 31)) & 1u)) return false;
    return scan_stencil<false>(g, lin, qx, qy, qz, r2, nullptr);
}

// clip_k in float (approximate reciprocal): the interval is that of a box perturbed by ~1e-5 m;
// samples it drops lie within that distance of the true clip box's outside, i.e. >= r + m -
// 1e-5 from every point (the box is the point bbox inflated by r + m + 1e-6 |coord|): empty.
__device__ __forceinline__ void clip_kf(const GridView &g, double px, double py, double pz,
                                        double dx, double dy, double dz, int K, int &klo,
                                        int &khi) {
    // branch-free slabs: a zero (or flushed denormal) direction component gives +-inf slab
    // times, so a start strictly inside the slab leaves [t0, t1] as it is and one outside
    // empties it; a start exactly on a slab face (0 * inf = NaN, dropped by fmin/fmax, the
    // other time +-inf) also empties it -- exact, since the face lies r + m + 1e-6 |coord| from
    // every point and a ray parallel to it never comes closer
    float t0 = 0.0f, t1 = FLT_MAX;
    const float p[3] = {(float)px, (float)py, (float)pz}, d[3] = {(float)dx, (float)dy, (float)dz};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float inv = __builtin_amdgcn_rcpf(d[a]);
        const float ta = (g.fb[2 * a] - p[a]) * inv, tb = (g.fb[2 * a + 1] - p[a]) * inv;
        t0 = fmaxf(t0, fminf(ta, tb));
        t1 = fminf(t1, fmaxf(ta, tb));
    }
    if (!(t0 <= t1)) {
        klo = 0;
        khi = -1;
        return;
    }
    // one sample of slack each side (s_k = 0.5 + 0.3 k to ~1e-13, t0/t1 to float rounding)
    const float inv_step = (float)(1.0 / kRayStep);
    const float kl = ceilf((t0 - 0.5f) * inv_step) - 1.0f;
    const float kh = floorf(fminf(t1, 1e30f) * inv_step - 0.5f * inv_step) + 1.0f;
    klo = (int)fminf(fmaxf(kl, 0.0f), (float)K);
    khi = (int)fminf(fmaxf(kh, -1.0f), (float)(K - 1));
}

// checkVisibilityWithRaycasting's march (virtual_lidar.cpp:765-797) from pos along unit dir:
// the samples s_k < end in order, returns the first blocked k or -1.
//  * Samples outside the clip box have no point within r (clip_kf, exact skip).
//  * Probe: sample k's stencil-corner coordinates (cell units) are A + D k, one fma per axis,
//    instead of the double query point q_k = float(p + d s_k).  Their error against the exact
//    corner arithmetic is ~1e-5 m, far inside the 1 mm query margin that already absorbs the
//    float corner: a block found empty from the approximate corner holds no point
//    within r of q_k.
//  * ZB (the z-sorted terrain index): the probe reads the corner block's z band (GridView.occz)
//    and skips q_k when it lies >= r + 2 mm above the block's highest point or below its lowest
//    -- then dz alone exceeds r for every point of the block, so FLANN's float sum does too.
//    Without ZB the probe reads the block's occupancy bit.
//  * A surviving sample computes q_k exactly (s_k is the step table entry: the table was built
//    by the same repeated additions the reference performs) and scans the block of its exact
//    corner, so every point test is the reference's test.
// STATS counts probes, scanned stencils and point tests into cnt[0..2].
//  * FN (the fine-window copy, g.frec): the probe reads the record of the sample's fine corner
//    -- its window's z band and run -- and a candidate walks that run with the exact q_k.  The
//    approximate corner's window holds every point within r of q_k (the same margin argument as
//    the block's), so no exact corner and no directory load are needed.  FN = 2 decides at run
//    time (g.frec null or not).
//  * koff, kstr: a lane of a group of kstr lanes marching one ray takes the samples
//    k = klo + koff (mod kstr) (NB-sample rounds: the rounds koff (mod kstr)); the ray is blocked
//    iff some lane finds a blocked sample -- the group's answer to "march < 0" is the same
template <bool STATS, bool ZB = true, int NB = 1, int FN = 0>
__device__ __forceinline__ int march(const GridView &g, double px, double py, double pz,
                                     double dx, double dy, double dz,
                                     const double *__restrict__ steps, int K, double end,
                                     float r2, float rexit, uint32_t *cnt = nullptr,
                                     int koff = 0, int kstr = 1) {
    if (FN == 2) {
        if (g.frec && g.ftile == 2)
            return march<STATS, ZB, NB, 8>(g, px, py, pz, dx, dy, dz, steps, K, end, r2, rexit,
                                           cnt, koff, kstr);
        if (g.frec && g.ftile)
            return march<STATS, ZB, NB, 4>(g, px, py, pz, dx, dy, dz, steps, K, end, r2, rexit,
                                           cnt, koff, kstr);
        if (g.frec)
            return march<STATS, ZB, NB, 1>(g, px, py, pz, dx, dy, dz, steps, K, end, r2, rexit,
                                           cnt, koff, kstr);
        return march<STATS, ZB, NB, 0>(g, px, py, pz, dx, dy, dz, steps, K, end, r2, rexit, cnt,
                                       koff, kstr);
    }
    int klo, khi;
    clip_kf(g, px, py, pz, dx, dy, dz, K, klo, khi);
    if (end < 1e299) {   // s_k < end: k <= (end - 0.5) / 0.3, with one sample of slack
        const double ke = floor((end - 0.5) / kRayStep) + 1.0;
        khi = (int)fmin((double)khi, fmax(ke, -1.0));
    }
    if (klo > khi) return -1;
    const float fdx = (float)dx, fdy = (float)dy, fdz = (float)dz;
    const float sc = (float)kRayStep * g.finv_c, h = 0.5f * g.finv_c;   // s_k = 0.5 + 0.3 k
    const float Dx = fdx * sc, Dy = fdy * sc, Dz = fdz * sc;
    const float Ax = ((float)px - g.flo_x) * g.finv_c + fdx * h;
    const float Ay = ((float)py - g.flo_y) * g.finv_c + fdy * h;
    const float Az = ((float)pz - g.flo_z) * g.finv_c + fdz * h;
    const uint32_t nx = (uint32_t)g.nx, ny = (uint32_t)g.ny;
    if (FN == 1 || FN == 4 || FN == 8) {
        // fine units for x, y (the fine cell of the sample, (q - o) / c_f = F (f + fzoff)),
        // coarse stencil-corner units for z; out-of-range cells are clamped: a sample outside
        // the grid has no point within r, and a clamped record can only cost a walk whose exact
        // tests all fail.  The float cell is within ~1e-5 m of the exact one, inside the margin
        // m of the window's radius r + m (pcp_fine.hip).
        const float F = g.ffine;
        const float D2x = F * Dx, D2y = F * Dy, A2x = F * (Ax + g.fzoff), A2y = F * (Ay + g.fzoff);
        const uint32_t mx = g.frx - 1, my = g.fry - 1, mz = g.frz - 1;
        const uint32_t rx = FN == 4 ? (g.frx + 3) >> 2 : FN == 8 ? (g.frx + 7) >> 3 : g.frx;
        const uint32_t ry = FN == 4 ? (g.fry + 3) >> 2 : FN == 8 ? (g.fry + 7) >> 3 : g.fry;
        for (int k = klo + koff; k <= khi; k += kstr) {
            const float kf = (float)k;
            const float fx = __builtin_fmaf(D2x, kf, A2x);
            const float fy = __builtin_fmaf(D2y, kf, A2y);
            const float fz = __builtin_fmaf(Dz, kf, Az);
            const uint32_t ix = min((uint32_t)fmaxf(fx, 0.0f), mx);
            const uint32_t iy = min((uint32_t)fmaxf(fy, 0.0f), my);
            const uint32_t iz = min((uint32_t)fmaxf(fz, 0.0f), mz);
            // 24-bit multiply-adds (full rate): build_fine caps frx, fry * frz below 2^24.
            // FN 4: records in 4 x 4 xy tiles, one 128-byte line each (a wave's arc of probes
            // touches fewer lines whatever its direction); rx, ry are then the tile counts.
            // FN 8: the split records in 8 x 8 tiles, the probe reads only the 2-byte thresholds
            // (64 per 128-byte line: a quarter of FN 4's bytes through the texture path) and a
            // candidate then its 4-byte walk start
            const uint32_t ri = FN == 8 ? (mad_u24(rx, mad_u24(ry, iz, iy >> 3), ix >> 3) << 6) |
                                              ((iy & 7u) << 3) | (ix & 7u)
                              : FN == 4 ? (mad_u24(rx, mad_u24(ry, iz, iy >> 2), ix >> 2) << 4) |
                                              ((iy & 3u) << 2) | (ix & 3u)
                                        : mad_u24(rx, mad_u24(ry, iz, iy), ix);
            uint2 R = make_uint2(0u, 0u);   // FN 8: only the thresholds (.y) come with the probe
            if (FN == 8) R.y = ld_u16o(g.fband, ri);
            else R = ld_rec(g.frec, ri);
            // height above the block floor in kZq steps against the record's thresholds
            const float us = __builtin_fmaf(fz - (float)iz, 1.0f / kZq, g.fus_off);
            const bool cand = (us < (float)((R.y >> 8) & 255u)) & (us > (float)(R.y & 255u));
            if (STATS) cnt[0] += 1;
            if (cand) {
                const double s = steps[k];
                if (!(s < end)) return -1;
                if (STATS) cnt[1] += 1;
                const float qx = (float)(px + dx * s);
                const float qy = (float)(py + dy * s);
                const float qz = (float)(pz + dz * s);
                uint32_t w0 = R.x;
                if (FN == 8) {   // skip the run's entries > r above q (pcp_fine.hip, k_frec)
                    const uint32_t ws = ld_u32o(g.fstart, ri);
                    // the thresholds are the record's double heights rounded through fzo, fzc
                    // and the fma (a few ulps of the larger magnitude): the margin grows with
                    // them, so far from the origin (|z| of km) the skip stays exact
                    if (g.fskip == 2) {
                        const float ha = __builtin_fmaf((float)iz + 1.375f, g.fzc, g.fzo);
                        const float hb = __builtin_fmaf((float)iz + 1.6875f, g.fzc, g.fzo);
                        const float marg = 1e-4f + 4.0f * FLT_EPSILON *
                                                       (fmaxf(fabsf(ha), fabsf(hb)) +
                                                        fabsf(g.fzo) + fabsf(qz));
                        const float v = qz + (rexit + marg);
                        w0 = (ws & 0x01FFFFFFu) +
                             (v < ha ? (ws >> 25) & 15u : v < hb ? ws >> 29 : 0u);
                    } else {
                        const float h2 = __builtin_fmaf((float)iz + 1.5f, g.fzc, g.fzo);
                        const float marg =
                            1e-4f + 4.0f * FLT_EPSILON * (fabsf(h2) + fabsf(g.fzo) + fabsf(qz));
                        w0 = (ws & 0x0FFFFFFFu) + (qz + (rexit + marg) < h2 ? ws >> 28 : 0u);
                    }
                }
                if (g.wpack ? scan_window3<STATS>(reinterpret_cast<const float *>(g.wpts), w0, qx,
                                                  qy, qz, r2, rexit, cnt)
                            : scan_window<STATS>(g.wpts, w0, qx, qy, qz, r2, rexit, cnt))
                    return k;
            }
        }
        return -1;
    }
    if (NB > 1 && ZB) {
        // latency-bound callers (few rays in flight): NB probes per round as independent loads,
        // then taken in sample order -- the same samples, candidates and scans as below
        for (int k0 = klo + NB * koff; k0 <= khi; k0 += NB * kstr) {
            uint32_t zz[NB], izs[NB];
            float fzs[NB];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const float kf = (float)(k0 + b);
                const float fx = __builtin_fmaf(Dx, kf, Ax);
                const float fy = __builtin_fmaf(Dy, kf, Ay);
                const float fz = __builtin_fmaf(Dz, kf, Az);
                const bool ok = (k0 + b <= khi) & (fx >= 0.0f) & (fx < g.fnx1) & (fy >= 0.0f) &
                                (fy < g.fny1) & (fz >= 0.0f) & (fz < g.fnz1);
                const uint32_t izc = ok ? (uint32_t)fz : 0u;
                const uint32_t lin = ok ? (uint32_t)fx + nx * ((uint32_t)fy + ny * izc) : 0u;
                zz[b] = ok ? ld_u16o(g.occz, lin) : 0x00FFu;
                izs[b] = izc;
                fzs[b] = fz;
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const int k = k0 + b;
                const uint32_t lo = zz[b] & 255u, hi = zz[b] >> 8;
                const float u = fzs[b] - (float)izs[b] + g.fzoff;
                const bool cand = (lo <= hi) & ((hi == 255u) | (u - (float)hi * kZq < g.fzt)) &
                                  ((lo == 0u) | ((float)lo * kZq - u < g.fzt));
                if (STATS && k <= khi) cnt[0] += 1;
                if (cand) {
                    const double s = steps[k];
                    if (!(s < end)) return -1;
                    if (STATS) cnt[1] += 1;
                    const float qx = (float)(px + dx * s);
                    const float qy = (float)(py + dy * s);
                    const float qz = (float)(pz + dz * s);
                    uint32_t l2;
                    if (stencil_cell(g, qx, qy, qz, l2) && scan_corner<STATS>(g, l2, qx, qy, qz, r2, cnt))
                        return k;
                }
            }
        }
        return -1;
    }
    for (int k = klo + koff; k <= khi; k += kstr) {
        const float kf = (float)k;
        const float fx = __builtin_fmaf(Dx, kf, Ax);
        const float fy = __builtin_fmaf(Dy, kf, Ay);
        const float fz = __builtin_fmaf(Dz, kf, Az);
        const bool ok = (fx >= 0.0f) & (fx < g.fnx1) & (fy >= 0.0f) & (fy < g.fny1) &
                        (fz >= 0.0f) & (fz < g.fnz1);
        const uint32_t izc = ok ? (uint32_t)fz : 0u;
        const uint32_t lin = ok ? (uint32_t)fx + nx * ((uint32_t)fy + ny * izc) : 0u;
        bool cand;
        if (ZB) {
            const uint32_t zz = ok ? ld_u16o(g.occz, lin) : 0x00FFu;
            const uint32_t lo = zz & 255u, hi = zz >> 8;
            const float u = fz - (float)izc + g.fzoff;          // (q_z - block floor) / c
            cand = (lo <= hi) & ((hi == 255u) | (u - (float)hi * kZq < g.fzt)) &
                   ((lo == 0u) | ((float)lo * kZq - u < g.fzt));
        } else {
            const uint32_t word = ok ? ld_u32o(g.occ2, lin >> 5) : 0u;
            cand = (word >> (lin & 31u)) & 1u;
        }
        if (STATS) cnt[0] += 1;
        if (cand) {
            const double s = steps[k];
            if (!(s < end)) return -1;       // every later sample is beyond end too
            if (STATS) cnt[1] += 1;
            const float qx = (float)(px + dx * s);
            const float qy = (float)(py + dy * s);
            const float qz = (float)(pz + dz * s);
            uint32_t l2;
            if (stencil_cell(g, qx, qy, qz, l2) && scan_corner<STATS>(g, l2, qx, qy, qz, r2, cnt))
                return k;
        }
    }
    return -1;
}

// ---------------------------------------------------------------------------------------
// cell scoring (evaluateCellScore, virtual_lidar.cpp:656-714)
// ---------------------------------------------------------------------------------------
struct VisEnv {
    GridView terrain;
    GridView aux;
    int terrain_present;   // terrain_kdtree_ non-null
    int aux_present;       // zx120 tree non-null and cloud non-empty
    double max_distance;
    const double *steps;
    int K;
    float r2_ray, r2_relaxed;
    float rexit_ray;       // exit_dist(r2_ray)
};

// evaluateCellScore's score of a visible cell (:689-700): the cosine d = |dot| clamped to
// [0, 1] gives sin(pi / 2 - acos(d)) (score_sin_part), then + 1 / L and the clamp at 0
// (score_finish).  glibc's acos and sin, which the reference calls, round correctly but for
// rare near ties: ocml's first results, then the midpoint tests / one rounding of pcp_crmath.h
// (ocml alone left 9 % of the cell scores off by 1-8 ulps, test_parity_bar_per_cell)
__device__ __forceinline__ double score_sin_part(double ad) {
#ifdef PCP_SCORE_OCML   // A/B build only (tools/r6_cr_ab.sh): ocml's acos / sin as they come
    return sin(kPi / 2 - acos(ad));
#else
    return pcp_score_sin_part(ad, acos(ad), nullptr);   // (two phases, pcp_crmath.h)
#endif
}

__device__ __forceinline__ double score_finish(double sin_part, double L, int cell) {
    const double score = 1.0 * sin_part + 1.0 * (1.0 / L);
#if PCP_SCORE_ULP   // parity-bar check builds only: the score of every PCP_SCORE_ULP-th cell
                    // one ulp up (make perturb: every cell; make perturb8: every 8th)
    if (cell % PCP_SCORE_ULP == 0) return fmax(0.0, nextafter(score, INFINITY));
#else
    (void)cell;
#endif
    return fmax(0.0, score);
}

// result bits: 1 = in_range, 2 = in_fov (valid if in_range), 4 = visible (valid if both)
// G > 1: the G lanes of an aligned lane group evaluate the same (pose, cell), each marching the
// samples koff (mod G) (march's koff / kstr); every lane returns the same result
// STATS (pcp_score_poses_stats): the march's probes / walk starts / point tests into cnt[0..2]
template <int G = 1, bool STATS = false>
__device__ __forceinline__ double eval_cell(const VisEnv &E, double px, double py, double pz,
                                            double pitch, double cx, double cy, double cz,
                                            float nx, float ny, float nz, bool is_zx120,
                                            uint32_t &bits, const double *steps,
                                            uint32_t *cnt = nullptr, int cell = 0) {
    const double dx = cx - px, dy = cy - py, dz = cz - pz;
    const double L = sqrt(dx * dx + dy * dy + dz * dz);
    bits = 0;
    const bool in_range = (L >= kMinDistance && L <= E.max_distance);
    if (!in_range) return 0.0;
    bits |= 1u;
    const double fov_local = 180.0 * kPi / 180.0;
    // the FOV decision, exactly the reference's double one: a float atan2 (error < 1e-6 rad
    // including the rounding of its arguments) decides every case farther than 1e-5 rad from
    // the boundary; the double atan2 only the rest
    const double h2 = dx * dx + dy * dy;
    const double dfast = (double)atan2f((float)dz, sqrtf((float)h2)) - pitch;
    if (fabs(dfast) > fov_local / 2.0 + 1e-5) return 0.0;
    if (!(fabs(dfast) < fov_local / 2.0 - 1e-5)) {
        const double elevation = atan2(dz, sqrt(h2));
        const double elevation_diff = elevation - pitch;
        if (!(fabs(elevation_diff) <= fov_local / 2.0)) return 0.0;
    }
    bits |= 2u;
    bool visible;
    const double ndx = dx / L, ndy = dy / L, ndz = dz / L;
    const double end = L - kVisRadius;
    if (is_zx120 && E.aux_present &&
        stencil_any(E.aux, (float)cx, (float)cy, (float)cz, E.r2_relaxed)) {
        visible = true;   // checkVisibilityWithPointCloudRelaxed (:745-747)
    } else if (!E.terrain_present) {
        visible = true;   // (:721, :727, :750)
    } else {
#if defined(PCP_CELL_EXP) && PCP_CELL_EXP == 1   // A/B timing only: no march
        visible = end > 1e300;
#elif defined(PCP_CELL_EXP) && PCP_CELL_EXP == 2  // A/B timing only: probes, a candidate = hit
        visible = march<false, true, PCP_CELL_PROBES>(E.terrain, px, py, pz, ndx, ndy, ndz,
                                                      steps, E.K, end, 1e30f, 1e15f) < 0;
#else
        const int lane = threadIdx.x & 63;
        const bool clear = march<STATS, true, PCP_CELL_PROBES, 2>(
                               E.terrain, px, py, pz, ndx, ndy, ndz, steps, E.K, end, E.r2_ray,
                               E.rexit_ray, cnt, G > 1 ? lane % G : 0, G) < 0;
        if (G > 1) {   // the group's lanes all reach here (same inputs, same branches)
            const uint64_t blocked = __ballot(!clear);
            visible = ((blocked >> (lane & ~(G - 1))) & ((1ull << G) - 1)) == 0;
        } else {
            visible = clear;
        }
#endif
    }
    if (!visible) return 0.0;
    bits |= 4u;
    const double dot = ndx * (double)nx + ndy * (double)ny + ndz * (double)nz;
    const double ad = fmax(0.0, fmin(1.0, fabs(dot)));
    return score_finish(score_sin_part(ad), L, cell);
}

// one thread per (cell c, row r): rows r < P are the candidate poses (evaluatePosition's
// score_mobile, written [p][c], coalesced), row P is the pose-invariant zx120 evaluation
// (score_zx120 and its result bits) -- one launch, so the zx120 row does not run alone on a
// handful of CUs.  std::max(score_zx120, score_mobile) is applied by k_row_sum.
#ifndef PCP_SCORE_WAVES
#define PCP_SCORE_WAVES 6   // waves per SIMD of k_score_cells (build knob)
#endif
// SL: the step table in LDS (K <= kStepLds, checked by the launcher).  (Several rows per
// thread, the cell loaded once, spilled ~120 dwords: the loop hoists both GridViews' kernel
// arguments into registers.)
template <bool SL>
__global__ void __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu(PCP_SCORE_WAVES, 8)))
k_score_cells(VisEnv E, const double *__restrict__ cxyz, const float *__restrict__ cn, int C,
              const double *__restrict__ poses5, int P, const double *__restrict__ zx5,
              double *__restrict__ sm_out, uint8_t *__restrict__ mbits,
              double *__restrict__ score_z, uint8_t *__restrict__ zbits,
              int32_t *__restrict__ stats, const uint32_t *__restrict__ P_dev,
              const uint32_t *__restrict__ C_dev) {
    const int c = blockIdx.x * kT + threadIdx.x;
    // the colour-statistics slots k_cell_flags accumulates into (it runs after this kernel)
    if (stats && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) stats[threadIdx.x] = 0;
    __shared__ double s_steps[SL ? kStepLds : 1];
    if (SL) {
        for (int q = threadIdx.x; q < E.K; q += kT) s_steps[q] = E.steps[q];
        __syncthreads();
    }
    const double *steps = SL ? s_steps : E.steps;
    // C_dev: the cells' count is the device's (a setup still in flight, C = its capacity and the
    // rows' stride)
    if (c >= (C_dev ? (int)*C_dev : C)) return;
    const int p = blockIdx.y;
    const bool zrow = p == P;   // the last row (P = the rows' capacity with P_dev)
    // P_dev: the pose count is the device's (candidates generated in the same stream)
    if (P_dev && !zrow && p >= (int)*P_dev) return;
    const double *Q = zrow ? zx5 : poses5 + 5 * (size_t)p;
    uint32_t bits;
    const double s = eval_cell(E, Q[0], Q[1], Q[2], Q[3], cxyz[3 * c], cxyz[3 * c + 1],
                               cxyz[3 * c + 2], cn[3 * c], cn[3 * c + 1], cn[3 * c + 2], zrow, bits,
                               steps, nullptr, c);
    if (zrow) {
        score_z[c] = s;
        zbits[c] = (uint8_t)bits;
    } else {
        sm_out[(size_t)p * C + c] = s;
        mbits[(size_t)p * C + c] = (uint8_t)bits;
    }
}

// Diagnostic twin of k_score_cells (pcp_score_poses_stats; never timed): the same rows and the
// same march, counting per launch the gather lane-loads its visibility rays issue -- z-band
// probes (2-byte thresholds), candidates' walk starts (4 bytes), point records (12 bytes) --
// into stats[0..2] (u64, one atomic per wave and counter).  No scores are written.
template <bool SL>
__global__ void __launch_bounds__(kT)
k_score_cells_stats(VisEnv E, const double *__restrict__ cxyz, const float *__restrict__ cn,
                    int C, const double *__restrict__ poses5, int P,
                    const double *__restrict__ zx5, unsigned long long *__restrict__ stats) {
    const int c = blockIdx.x * kT + threadIdx.x;
    __shared__ double s_steps[SL ? kStepLds : 1];
    if (SL) {
        for (int q = threadIdx.x; q < E.K; q += kT) s_steps[q] = E.steps[q];
        __syncthreads();
    }
    const double *steps = SL ? s_steps : E.steps;
    uint32_t cnt[4] = {0u, 0u, 0u, 0u};
    if (c < C) {
        const int p = blockIdx.y;
        const double *Q = p == P ? zx5 : poses5 + 5 * (size_t)p;
        uint32_t bits;
        (void)eval_cell<1, true>(E, Q[0], Q[1], Q[2], Q[3], cxyz[3 * c], cxyz[3 * c + 1],
                                 cxyz[3 * c + 2], cn[3 * c], cn[3 * c + 1], cn[3 * c + 2], p == P,
                                 bits, steps, cnt, c);
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        unsigned long long v = cnt[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(&stats[i], v);
    }
}

// The same rows with G lanes per (cell, row): for launches with few rays (one candidate pose,
// C1 / C5), where one lane per ray leaves the GPU nearly empty and each ray's march is a long
// chain of dependent probes.  The G lanes split the ray's samples (march koff / kstr) and AND
// their verdicts; lane 0 of the group writes.
template <bool SL, int G>
__global__ void __launch_bounds__(kT)
k_score_cells_wide(VisEnv E, const double *__restrict__ cxyz, const float *__restrict__ cn,
                   int C, const double *__restrict__ poses5, int P,
                   const double *__restrict__ zx5, double *__restrict__ sm_out,
                   uint8_t *__restrict__ mbits, double *__restrict__ score_z,
                   uint8_t *__restrict__ zbits, int32_t *__restrict__ stats,
                   const uint32_t *__restrict__ P_dev, const uint32_t *__restrict__ C_dev) {
    static_assert(G > 1 && G <= 64 && (G & (G - 1)) == 0, "lane groups within a wave");
    const int c = (int)((blockIdx.x * kT + threadIdx.x) / G);
    if (stats && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) stats[threadIdx.x] = 0;
    __shared__ double s_steps[SL ? kStepLds : 1];
    if (SL) {
        for (int q = threadIdx.x; q < E.K; q += kT) s_steps[q] = E.steps[q];
        __syncthreads();
    }
    const double *steps = SL ? s_steps : E.steps;
    if (c >= (C_dev ? (int)*C_dev : C)) return;   // (whole groups: C * G threads, groups aligned)
    const int p = blockIdx.y;
    const bool zrow = p == P;
    if (P_dev && !zrow && p >= (int)*P_dev) return;
    const double *Q = zrow ? zx5 : poses5 + 5 * (size_t)p;
    uint32_t bits;
    const double s = eval_cell<G>(E, Q[0], Q[1], Q[2], Q[3], cxyz[3 * c], cxyz[3 * c + 1],
                                  cxyz[3 * c + 2], cn[3 * c], cn[3 * c + 1], cn[3 * c + 2], zrow,
                                  bits, steps, nullptr, c);
    if ((threadIdx.x & (G - 1)) != 0) return;
    if (zrow) {
        score_z[c] = s;
        zbits[c] = (uint8_t)bits;
    } else {
        sm_out[(size_t)p * C + c] = s;
        mbits[(size_t)p * C + c] = (uint8_t)bits;
    }
}
constexpr int kWideG = 16;               // lanes per ray of k_score_cells_wide
constexpr int kWideMaxRays = 1 << 15;    // (rows x cells) up to which the wide kernel runs

// ordered sequential sum per row (evaluatePosition :634-645): total_score += s for s > 0 in cell
// order, s = std::max(score_zx120, score_mobile) = (sz < sm) ? sm : sz for a pose row, sz for
// the zx120 row (r == P).  One wave per row: each lane holds 8 of the next 512 values in
// registers (the following 512 already loading), and the wave walks them in cell order with
// v_readlane into scalar registers, every lane carrying the same running sum -- no LDS round
// trip in the chain, which is the dependent adds alone.
constexpr int kSumChunk = 512;
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const uint64_t b = __double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ void row_sum_body(const double *__restrict__ sm,
                                             const double *__restrict__ score_z, int C, int P,
                                             double *__restrict__ total,
                                             int32_t *__restrict__ covered, int r) {
    const int lane = threadIdx.x & 63;
    const double *row = sm + (size_t)r * C;
    constexpr int kPer = kSumChunk / 64;
    double v[kPer], wz[kPer], wm[kPer];
    int32_t cov = 0;   // order-free: each lane counts its own positive values
    // raw loads only: the values they feed are formed after the chain that overlaps them
    auto load = [&](int base) {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const int c = base + q * 64 + lane;
            wz[q] = c < C ? score_z[c] : 0.0;
            wm[q] = (c < C && r < P) ? row[c] : 0.0;
        }
    };
    // x > 0 ? x : +0.0 -- adding +0.0 to the (non-negative) running sum leaves it bit-identical,
    // so the unconditional adds are the reference's `if (x > 0) total += x`
    auto form = [&]() {
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            const double sz = wz[q], m = wm[q];
            const double x = r < P ? ((sz < m) ? m : sz) : sz;
            const bool pos = x > 0;
            cov += pos ? 1 : 0;
            v[q] = pos ? x : 0.0;
        }
    };
    double acc = 0.0;
    load(0);
    form();
    for (int base = 0; base < C; base += kSumChunk) {
        const bool more = base + kSumChunk < C;
        if (more) load(base + kSumChunk);   // in flight during the chain
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            if (base + q * 64 >= C) break;   // wave-uniform; the tail's zero lanes add +0.0
#pragma unroll
            for (int l = 0; l < 64; l += 8) {   // 8 readlanes ahead of their adds
                double t[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) t[i] = readlane_f64(v[q], l + i);
#pragma unroll
                for (int i = 0; i < 8; ++i) acc += t[i];
            }
        }
        if (more) form();
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cov += __shfl_xor(cov, o, 64);
    if (lane == 0) {
        total[r] = acc;
        covered[r] = cov;
    }
}

// The same sums, one ROW PER LANE: a block of kT threads owns kSumRows rows.  Waves 1..3 load
// chunks of kSumCh cells of those rows (coalesced, one row per pass, kSumLpt cells per thread),
// form the values (the max with score_z, x > 0 ? x : +0.0, the covered counts) and stage them
// in LDS [row][cell]; lane r of wave 0 then walks row r of the chunk in cell order -- its
// chain is the dependent v_add_f64s alone (~6 clocks each on gfx950, tools/mb/chain.hip), the
// LDS reads of the next two groups of 32 values in flight under the adds of the current group,
// with no readlane traffic in front of each add (the one-wave-per-row chain above: 2 readlanes
// per add, ~19 clocks).  Three LDS buffers: the loaders fill chunk k + 2 while the chain walks
// chunk k, one barrier per chunk; their global loads run two chunks further ahead.
// k_sum_flags at 256 poses x 3,704 cells (tools/ab_libs.sh): 29.6 us one wave per row; lane
// per row with 16 / 8 / 4 / 2 rows per block 33 / 27 / 25.5 / 25.5 us (a block's loads are
// latency x concurrency bound on its CU, so few rows per block), the ring walk 20.5 us.
#ifndef PCP_SUM_ROWS
#define PCP_SUM_ROWS 4   // rows per block: few, so the loads of the rows spread over many CUs
#endif
#ifndef PCP_SUM_LPT
#define PCP_SUM_LPT 2    // cells per loader thread per chunk (chunk = 192 x this)
#endif
#ifndef PCP_SUM_BATCH
#define PCP_SUM_BATCH 16 // ds_read_b128 per group of the walk
#endif
constexpr int kSumRows = PCP_SUM_ROWS, kSumLpt = PCP_SUM_LPT, kSumCh = (kT - 64) * kSumLpt;
constexpr int kSumLd = kSumCh + 2;   // +2: b128 reads of lanes r, r + 1 four banks apart
// C: the rows' stride; Ca: the cells summed (C, or the device's count of a setup in flight)
__device__ __forceinline__ void row_group_body(const double *__restrict__ sm,
                                               const double *__restrict__ score_z, int C, int Ca,
                                               int P, double *__restrict__ total,
                                               int32_t *__restrict__ covered, int g) {
    __shared__ double s_v[3][kSumRows][kSumLd];
    __shared__ int32_t s_cov[kSumRows];
    const int tid = threadIdx.x, r0 = g * kSumRows;
    if (Ca <= 0) {   // no cells (uniform): every total is the +0.0 it starts from
        if (tid < kSumRows && r0 + tid <= P) {
            total[r0 + tid] = 0.0;
            covered[r0 + tid] = 0;
        }
        return;
    }
    const int nch = (Ca + kSumCh - 1) / kSumCh;
    if (tid < kSumRows) s_cov[tid] = 0;
    const int lt = tid - 64;   // loader thread (waves 1..3): cells lt + (kT - 64) i of a chunk
    int32_t cov[kSumRows];
#pragma unroll
    for (int q = 0; q < kSumRows; ++q) cov[q] = 0;
    // raw loads into registers, unconditional (row and cell clamped into the buffer; the
    // formation masks them), in two register sets for chunks of even / odd index: the loads
    // of chunk k + 4 go out while chunk k + 2 is formed, two chain chunks ahead of their use
    double mA[kSumLpt][kSumRows], szA[kSumLpt], mB[kSumLpt][kSumRows], szB[kSumLpt];
    auto load = [&](int k, double (&m)[kSumLpt][kSumRows], double (&sz)[kSumLpt]) {
#pragma unroll
        for (int i = 0; i < kSumLpt; ++i) {
            const int c = min(k * kSumCh + lt + (kT - 64) * i, Ca - 1);
            sz[i] = score_z[c];
#pragma unroll
            for (int q = 0; q < kSumRows; ++q)
                m[i][q] = sm[(size_t)max(min(r0 + q, P - 1), 0) * C + c];
        }
    };
    auto form = [&](int k, const double (&m)[kSumLpt][kSumRows], const double (&sz)[kSumLpt]) {
        double(*dst)[kSumLd] = s_v[k % 3];
#pragma unroll
        for (int i = 0; i < kSumLpt; ++i) {
            const int cl = lt + (kT - 64) * i;
            const bool in = k * kSumCh + cl < Ca;
#pragma unroll
            for (int q = 0; q < kSumRows; ++q) {
                const double x = r0 + q < P ? ((sz[i] < m[i][q]) ? m[i][q] : sz[i]) : sz[i];
                const bool pos = in && x > 0;   // (cells past C add +0.0)
                cov[q] += pos ? 1 : 0;
                dst[q][cl] = pos ? x : 0.0;
            }
        }
    };
    double acc = 0.0;
    auto walk = [&](int k) {
        // software-pipelined walk over a ring of three groups of kG b128 reads: the adds of
        // group i run while groups i + 1 and i + 2 are in flight.  lgkmcnt counts at most 15
        // outstanding LDS operations, so a wait for group i also waits for the head of group
        // i + 1 -- issued a whole group of adds earlier, so already in -- but never for group
        // i + 2, issued just before.  The scheduling barriers keep each group's reads ahead of
        // the adds before it (the scheduler otherwise sinks them next to their use, exposing
        // the LDS latency).  tools/ab_libs.sh: two batches of 4 / 6 / 16 reads 24.1 / 23.2 /
        // 21.0 us per k_sum_flags, the ring of 8 / 16 21.1 / 20.5 us.
        const double2 *v = reinterpret_cast<const double2 *>(s_v[k % 3][tid]);
        constexpr int kG = PCP_SUM_BATCH, kN = kSumCh / 2;
        static_assert(kN % (3 * kG) == 0, "whole group triples per chunk");
        double2 g0[kG], g1[kG], g2[kG];
        auto rd = [&](double2 *g, int j) {
#pragma unroll
            for (int i = 0; i < kG; ++i) g[i] = v[j + i];
        };
        auto add = [&](const double2 *g) {
#pragma unroll
            for (int i = 0; i < kG; ++i) {
                acc += g[i].x;
                acc += g[i].y;
            }
        };
        rd(g0, 0);
        rd(g1, kG);
#pragma unroll
        for (int j = 0; j < kN; j += 3 * kG) {
            if (j + 2 * kG < kN) rd(g2, j + 2 * kG);
            __builtin_amdgcn_sched_barrier(0);
            add(g0);
            __builtin_amdgcn_sched_barrier(0);
            if (j + 3 * kG < kN) rd(g0, j + 3 * kG);
            __builtin_amdgcn_sched_barrier(0);
            add(g1);
            __builtin_amdgcn_sched_barrier(0);
            if (j + 4 * kG < kN) rd(g1, j + 4 * kG);
            __builtin_amdgcn_sched_barrier(0);
            add(g2);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // one chunk: the loaders form chunk k + 2 (and load k + 4) while the chain walks chunk k
    auto step = [&](int k, double (&m)[kSumLpt][kSumRows], double (&sz)[kSumLpt]) {
        if (tid >= 64) {
            if (k + 2 < nch) {
                form(k + 2, m, sz);
                if (k + 4 < nch) load(k + 4, m, sz);
            }
        } else if (tid < kSumRows) {
            walk(k);
        }
        __syncthreads();
    };
    if (tid >= 64) {
        load(0, mA, szA);
        if (nch > 1) load(1, mB, szB);
        form(0, mA, szA);
        if (nch > 2) load(2, mA, szA);
        if (nch > 1) form(1, mB, szB);
        if (nch > 3) load(3, mB, szB);
    }
    __syncthreads();
    for (int k = 0; k < nch; k += 2) {
        step(k, mA, szA);
        if (k + 1 < nch) step(k + 1, mB, szB);
    }
    if (tid >= 64) {
#pragma unroll
        for (int q = 0; q < kSumRows; ++q) {
            int32_t x = cov[q];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
            if ((tid & 63) == 0) atomicAdd(&s_cov[q], x);
        }
    }
    __syncthreads();
    if (tid < kSumRows && r0 + tid <= P) {
        total[r0 + tid] = acc;
        covered[r0 + tid] = s_cov[tid];
    }
}
__host__ __device__ constexpr int sum_groups(int P) { return (P + 1 + kSumRows - 1) / kSumRows; }

#ifndef PCP_ROW_SUM_LANES
#define PCP_ROW_SUM_LANES 1   // 0: the readlane chain (one wave per row) above
#endif

__global__ void __launch_bounds__(64)
k_row_sum(const double *__restrict__ sm, const double *__restrict__ score_z, int C, int P,
          double *__restrict__ total, int32_t *__restrict__ covered) {
    row_sum_body(sm, score_z, C, P, total, covered, blockIdx.x);
}
__global__ void __launch_bounds__(kT)
k_row_sum_lanes(const double *__restrict__ sm, const double *__restrict__ score_z, int C, int P,
                double *__restrict__ total, int32_t *__restrict__ covered) {
    row_group_body(sm, score_z, C, C, P, total, covered, blockIdx.x);
}

// stats slots
enum {
    S_TOTAL = 0, S_ZR, S_ZF, S_ZV, S_ZG, S_ZRED, S_ZB, S_ZY, S_G, S_RED, S_B, S_Y, S_N
};

// stale-flag resolution (virtual_lidar.cpp:487-501 read flags written by the LAST
// evaluation that reached each assignment, :662-687) + colour statistics
// stats_host (nullable): the last of the nblk flag blocks to finish copies the finished
// statistics there (ticket in stats[63], zeroed with the rest by k_score_cells)
__device__ __forceinline__ void cell_flags_body(const uint8_t *__restrict__ zbits,
                                                const uint8_t *__restrict__ mbits, int C, int Ca,
                                                int P, uint8_t *__restrict__ flags,
                                                int32_t *__restrict__ stats, int blk,
                                                int32_t *__restrict__ stats_host = nullptr,
                                                int nblk = 0) {
    const int c = blk * kT + threadIdx.x;
    __shared__ int32_t bst[S_N];
    if (threadIdx.x < S_N) bst[threadIdx.x] = 0;
    __syncthreads();
    if (c < Ca) {   // (C: mbits' row stride)
        uint32_t f = flags[c];
        const uint32_t z = zbits[c];
        f = (z & 1u) ? (f | PCP_F_RANGE_Z) : (f & ~PCP_F_RANGE_Z);
        if (z & 1u) f = (z & 2u) ? (f | PCP_F_FOV_Z) : (f & ~PCP_F_FOV_Z);
        if ((z & 3u) == 3u) f = (z & 4u) ? (f | PCP_F_VIS_Z) : (f & ~PCP_F_VIS_Z);
        // evaluateZX120Only statistics use the zx120 flags right after its evaluation (:377-397)
        const bool zr = f & PCP_F_RANGE_Z, zf = f & PCP_F_FOV_Z, zv = f & PCP_F_VIS_Z;
        if (P > 0) {
            // the last pose that reached each assignment, newest first, 16 poses per round of
            // independent loads (coalesced over the cells of the block)
            const uint32_t lastb = mbits[(size_t)(P - 1) * C + c];
            f = (lastb & 1u) ? (f | PCP_F_RANGE_M) : (f & ~PCP_F_RANGE_M);
            int fov_from = -1, vis_from = -1;   // pose whose bits set the flag
            for (int p0 = P - 1; p0 >= 0 && (fov_from < 0 || vis_from < 0); p0 -= 16) {
                uint32_t b[16];
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    b[q] = (p0 - q >= 0) ? mbits[(size_t)(p0 - q) * C + c] : 0u;
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    if (fov_from < 0 && (b[q] & 1u)) fov_from = p0 - q, f = (b[q] & 2u) ? (f | PCP_F_FOV_M) : (f & ~PCP_F_FOV_M);
                    if (vis_from < 0 && (b[q] & 3u) == 3u) vis_from = p0 - q, f = (b[q] & 4u) ? (f | PCP_F_VIS_M) : (f & ~PCP_F_VIS_M);
                }
                if (p0 - 15 <= 0) break;
            }
        }
        flags[c] = (uint8_t)f;
        atomicAdd(&bst[S_TOTAL], 1);
        if (zr) atomicAdd(&bst[S_ZR], 1);
        if (zf) atomicAdd(&bst[S_ZF], 1);
        if (zv) atomicAdd(&bst[S_ZV], 1);
        if (!zr) atomicAdd(&bst[S_ZB], 1);
        else if (!zf) atomicAdd(&bst[S_ZY], 1);
        else if (!zv) atomicAdd(&bst[S_ZRED], 1);
        else atomicAdd(&bst[S_ZG], 1);
        const bool mr = f & PCP_F_RANGE_M, mf = f & PCP_F_FOV_M, mv = f & PCP_F_VIS_M;
        const bool zr2 = f & PCP_F_RANGE_Z, zf2 = f & PCP_F_FOV_Z, zv2 = f & PCP_F_VIS_Z;
        if (!zr2 && !mr) atomicAdd(&bst[S_B], 1);
        else if (!zf2 && !mf) atomicAdd(&bst[S_Y], 1);
        else if (!zv2 && !mv) atomicAdd(&bst[S_RED], 1);
        else atomicAdd(&bst[S_G], 1);
    }
    __syncthreads();
    if (threadIdx.x < S_N && bst[threadIdx.x]) atomicAdd(&stats[threadIdx.x], bst[threadIdx.x]);
    if (!stats_host) return;
    __threadfence();   // this block's statistics adds before its ticket
    __syncthreads();
    __shared__ int last;
    if (threadIdx.x == 0) last = atomicAdd(&stats[63], 1) == nblk - 1;
    __syncthreads();
    if (last && threadIdx.x < S_N) stats_host[threadIdx.x] = atomicAdd(&stats[threadIdx.x], 0);
}

__global__ void __launch_bounds__(kT)
k_cell_flags(const uint8_t *__restrict__ zbits, const uint8_t *__restrict__ mbits, int C, int P,
             uint8_t *__restrict__ flags, int32_t *__restrict__ stats) {
    cell_flags_body(zbits, mbits, C, C, P, flags, stats, blockIdx.x);
}

// the two independent tails of a score query in ONE launch: the first blocks are the ordered
// row sums (row_group_body, kSumRows rows per block; a 3,704-add chain per row, ~20 us), the
// blocks after them the stale-flag resolution (~7 us), which so runs beside the chains
// instead of after them
__global__ void __launch_bounds__(kT)
k_sum_flags(const double *__restrict__ sm, const double *__restrict__ score_z, int C, int P,
            double *__restrict__ total, int32_t *__restrict__ covered,
            const uint8_t *__restrict__ zbits, const uint8_t *__restrict__ mbits,
            uint8_t *__restrict__ flags, int32_t *__restrict__ stats,
            int32_t *__restrict__ stats_host, const uint32_t *__restrict__ P_dev,
            const uint32_t *__restrict__ C_dev) {
    // P: the rows the grid was sized for; Pa: the poses (the device's count with P_dev, the
    // row blocks past it idle); C: the rows' stride and the cells the grid was sized for, Ca
    // the cells (the device's count with C_dev)
    const int Pa = P_dev ? (int)*P_dev : P;
    const int Ca = C_dev ? (int)*C_dev : C;
#if PCP_ROW_SUM_LANES
    const int nr = sum_groups(P);
    if ((int)blockIdx.x < nr) {
        if ((int)blockIdx.x < sum_groups(Pa))
            row_group_body(sm, score_z, C, Ca, Pa, total, covered, blockIdx.x);
        return;
    }
#else
    const int nr = P + 1;
    if ((int)blockIdx.x < nr) {
        if (threadIdx.x < 64 && (int)blockIdx.x <= Pa)
            row_sum_body(sm, score_z, C, Pa, total, covered, blockIdx.x);   // (C_dev: lanes path only)
        return;
    }
#endif
    cell_flags_body(zbits, mbits, C, Ca, Pa, flags, stats, (int)blockIdx.x - nr, stats_host,
                    (int)gridDim.x - nr);
}
__host__ __device__ constexpr int sum_flag_row_blocks(int P) {
    return PCP_ROW_SUM_LANES ? sum_groups(P) : P + 1;
}

// ---------------------------------------------------------------------------------------
// pose-sharded search across GPUs (pcp_multi.hip): per-rank key vectors, reduced by ONE
// collective, then finalized on one rank
// ---------------------------------------------------------------------------------------
// fan: keys[i] = (blocked << 32) | i for this rank's poses [lo, lo + cnt), UINT64_MAX elsewhere;
// all-reduce(MIN) leaves every pose's key on every rank and the minimum key is the reference
// argmin with ties to the lowest index
__global__ void __launch_bounds__(kT)
k_fan_keys(const uint32_t *__restrict__ blocked, uint32_t lo, uint32_t cnt, uint32_t P,
           unsigned long long *__restrict__ keys, unsigned long long identity) {
    const uint32_t i = blockIdx.x * kT + threadIdx.x;
    if (i >= P) return;
    keys[i] = (i >= lo && i - lo < cnt)
                  ? (((unsigned long long)blocked[i - lo] << 32) | (unsigned long long)i)
                  : identity;
}

// reference mode: v = [P totals | P covered | C range | C fov | C vis], all-reduce(MAX).
// Totals are >= +0.0 (sums of positive scores from +0.0), so their IEEE bits order like the
// values; 0 = +0.0 marks other ranks' poses.  A covered key carries kScoreWritten beside the
// count, so a pose no rank scored reduces to 0 and is reported, not read as a zero total (as the
// fan's UINT64_MAX key).  Per cell, the newest pose of this rank that
// reached each stale-flag assignment (:662-687) as ((global index + 1) << 1) | bit, 0 = none:
// the maximum over the ranks is the newest pose overall, which is what k_cell_flags resolves.
__global__ void __launch_bounds__(kT)
k_score_keys(const double *__restrict__ tot, const int32_t *__restrict__ cov,
             const uint8_t *__restrict__ mbits, int C, int Pl, int lo, int P,
             unsigned long long *__restrict__ v) {
    const int i = blockIdx.x * kT + threadIdx.x;
    if (i < P) {
        const bool mine = i >= lo && i - lo < Pl;
        v[i] = mine ? (unsigned long long)__double_as_longlong(tot[i - lo]) : 0ull;
        v[P + i] = mine ? (kScoreWritten | (unsigned long long)(uint32_t)cov[i - lo]) : 0ull;
    }
    if (i < C) {
        unsigned long long kr = 0, kf = 0, kv = 0;
        if (Pl > 0) {
            const uint32_t lb = mbits[(size_t)(Pl - 1) * C + i];
            kr = ((unsigned long long)(lo + Pl) << 1) | (lb & 1u);
            for (int q = Pl - 1; q >= 0 && (!kf || !kv); --q) {
                const uint32_t b = mbits[(size_t)q * C + i];
                const unsigned long long g1 = (unsigned long long)(lo + q + 1) << 1;
                if (!kf && (b & 1u)) kf = g1 | ((b >> 1) & 1u);
                if (!kv && (b & 3u) == 3u) kv = g1 | ((b >> 2) & 1u);
            }
        }
        v[2 * (size_t)P + i] = kr;
        v[2 * (size_t)P + C + i] = kf;
        v[2 * (size_t)P + 2 * (size_t)C + i] = kv;
    }
}

// colour statistics of one cell's final flags (evaluateZX120Only :377-397 and :487-501)
__device__ __forceinline__ void count_flags(uint32_t f, int32_t *bst) {
    const bool zr = f & PCP_F_RANGE_Z, zf = f & PCP_F_FOV_Z, zv = f & PCP_F_VIS_Z;
    atomicAdd(&bst[S_TOTAL], 1);
    if (zr) atomicAdd(&bst[S_ZR], 1);
    if (zf) atomicAdd(&bst[S_ZF], 1);
    if (zv) atomicAdd(&bst[S_ZV], 1);
    if (!zr) atomicAdd(&bst[S_ZB], 1);
    else if (!zf) atomicAdd(&bst[S_ZY], 1);
    else if (!zv) atomicAdd(&bst[S_ZRED], 1);
    else atomicAdd(&bst[S_ZG], 1);
    const bool mr = f & PCP_F_RANGE_M, mf = f & PCP_F_FOV_M, mv = f & PCP_F_VIS_M;
    if (!zr && !mr) atomicAdd(&bst[S_B], 1);
    else if (!zf && !mf) atomicAdd(&bst[S_Y], 1);
    else if (!zv && !mv) atomicAdd(&bst[S_RED], 1);
    else atomicAdd(&bst[S_G], 1);
}

// the reduced keys -> cell flags + colour statistics (the k_cell_flags result)
__global__ void __launch_bounds__(kT)
k_flags_from_keys(const unsigned long long *__restrict__ v, const uint8_t *__restrict__ zbits,
                  int C, int P, uint8_t *__restrict__ flags, int32_t *__restrict__ stats) {
    const int c = blockIdx.x * kT + threadIdx.x;
    __shared__ int32_t bst[S_N];
    if (threadIdx.x < S_N) bst[threadIdx.x] = 0;
    __syncthreads();
    if (c < C) {
        uint32_t f = flags[c];
        const uint32_t z = zbits[c];
        f = (z & 1u) ? (f | PCP_F_RANGE_Z) : (f & ~PCP_F_RANGE_Z);
        if (z & 1u) f = (z & 2u) ? (f | PCP_F_FOV_Z) : (f & ~PCP_F_FOV_Z);
        if ((z & 3u) == 3u) f = (z & 4u) ? (f | PCP_F_VIS_Z) : (f & ~PCP_F_VIS_Z);
        const unsigned long long kr = v[2 * (size_t)P + c], kf = v[2 * (size_t)P + C + c],
                                 kv = v[2 * (size_t)P + 2 * (size_t)C + c];
        if (kr) f = (kr & 1ull) ? (f | PCP_F_RANGE_M) : (f & ~PCP_F_RANGE_M);
        if (kf) f = (kf & 1ull) ? (f | PCP_F_FOV_M) : (f & ~PCP_F_FOV_M);
        if (kv) f = (kv & 1ull) ? (f | PCP_F_VIS_M) : (f & ~PCP_F_VIS_M);
        flags[c] = (uint8_t)f;
        count_flags(f, bst);
    }
    __syncthreads();
    if (threadIdx.x < S_N && bst[threadIdx.x]) atomicAdd(&stats[threadIdx.x], bst[threadIdx.x]);
}

// element-wise min / max of two key vectors (ranks sharing one device, no RCCL)
__global__ void __launch_bounds__(kT)
k_keys_combine(unsigned long long *__restrict__ a, const unsigned long long *__restrict__ b,
               size_t n, int is_max) {
    const size_t i = (size_t)blockIdx.x * kT + threadIdx.x;
    if (i >= n) return;
    a[i] = is_max ? (a[i] > b[i] ? a[i] : b[i]) : (a[i] < b[i] ? a[i] : b[i]);
}

void launch_fan_keys(hipStream_t st, const uint32_t *blocked_d, uint32_t lo, uint32_t cnt,
                     uint32_t P, unsigned long long *keys, unsigned long long identity) {
    hipLaunchKernelGGL(k_fan_keys, dim3((P + kT - 1) / kT), dim3(kT), 0, st, blocked_d, lo, cnt,
                       P, keys, identity);
}
void launch_score_keys(hipStream_t st, const ScoreEnq &o, int lo, int P,
                       unsigned long long *v) {
    const int n = std::max(P, o.C);
    hipLaunchKernelGGL(k_score_keys, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, st,
                       (const double *)o.tot_d, (const int32_t *)o.cov_d,
                       (const uint8_t *)o.mbits, o.C, o.P, lo, P, v);
}
void launch_flags_from_keys(hipStream_t st, const unsigned long long *v, const uint8_t *zbits,
                            int C, int P, uint8_t *flags, int32_t *stats) {
    if (C)
        hipLaunchKernelGGL(k_flags_from_keys, dim3((unsigned)((C + kT - 1) / kT)), dim3(kT), 0, st,
                           v, zbits, C, P, flags, stats);
}
// the one-collective scoring's results into the caller's pinned block in one launch (instead of
// five D2H copies): [2P reduced keys | the zx120 total | the health word | C flags | 64 stats]
__global__ void __launch_bounds__(kT)
k_score_land(const unsigned long long *__restrict__ v, int P, size_t hw,
             const double *__restrict__ zx_total, const uint8_t *__restrict__ flags, int C,
             const int32_t *__restrict__ stats, unsigned char *__restrict__ pin, size_t fl_off,
             size_t st_off) {
    const size_t t = (size_t)blockIdx.x * kT + threadIdx.x, nt = (size_t)gridDim.x * kT;
    unsigned long long *ph = reinterpret_cast<unsigned long long *>(pin);
    for (size_t i = t; i < 2 * (size_t)P; i += nt) ph[i] = v[i];
    if (t == 0) {
        ph[2 * (size_t)P] = (unsigned long long)__double_as_longlong(*zx_total);
        ph[2 * (size_t)P + 1] = v[hw];
    }
    for (size_t i = t; i < (size_t)C; i += nt) pin[fl_off + i] = flags[i];
    if (t < 64) reinterpret_cast<int32_t *>(pin + st_off)[t] = stats[t];
}
void launch_score_land(hipStream_t st, const unsigned long long *v, int P, size_t hw,
                       const double *zx_total, const uint8_t *flags, int C, const int32_t *stats,
                       void *pin, size_t fl_off, size_t st_off) {
    const size_t work = std::max<size_t>(std::max<size_t>(2 * (size_t)P, (size_t)C), 64);
    const unsigned g = (unsigned)std::min<size_t>((work + kT - 1) / kT, 64);
    hipLaunchKernelGGL(k_score_land, dim3(g), dim3(kT), 0, st, v, P, hw, zx_total, flags, C,
                       stats, static_cast<unsigned char *>(pin), fl_off, st_off);
}
void launch_keys_combine(hipStream_t st, unsigned long long *a, const unsigned long long *b,
                         size_t n, bool is_max) {
    if (n)
        hipLaunchKernelGGL(k_keys_combine, dim3((unsigned)((n + kT - 1) / kT)), dim3(kT), 0, st,
                           a, b, n, is_max ? 1 : 0);
}

// ---------------------------------------------------------------------------------------
// candidates (generateCandidatePositions :550-598, getGroundHeight :600-625)
// ---------------------------------------------------------------------------------------
struct CandArgs {
    GridView g;
    int ground_enabled;    // terrain cloud non-empty (:601)
    int gs;
    double exminx, exminy, xs, ys;
    double gminx, gmaxx, gminy, gmaxy;
    double cx, cy, cz;
    double zxx, zxy;
    double sensor_height;
    double *lat;           // gs*gs x 6: valid, x, y, z, pitch, yaw
};

// 1,024 threads per lattice point: the ground query's rows of cells (~600 for a 0.12 m terrain
// grid) one per thread, so a block's latency is one row walk, not three
constexpr int kCandT = 1024;
__global__ void __launch_bounds__(kCandT) k_candidates(CandArgs a) {
    const int l = blockIdx.x;
    const int i = l / a.gs, j = l - i * a.gs;
    const double x = a.exminx + i * a.xs;
    const double y = a.exminy + j * a.ys;
    double *out = a.lat + 6 * (size_t)l;
    const double ddx = x - a.zxx, ddy = y - a.zxy;
    if (sqrt(ddx * ddx + ddy * ddy) < 0.5 ||
        (x >= a.gminx && x <= a.gmaxx && y >= a.gminy && y <= a.gmaxy)) {
        if (threadIdx.x == 0) out[0] = 0.0;
        return;
    }
    // getGroundHeight: radiusSearch((float)x,(float)y,0; r=2) then 2-D distance < 1.0
    double mz = -DBL_MAX;
    if (a.ground_enabled && a.g.n_pts > 0) {
        const GridView &g = a.g;
        const float qx = (float)x, qy = (float)y, qz = 0.0f;
        const float r2 = (float)(2.0 * 2.0);
        const double m = kQueryMargin;
        auto rng = [&](double lo, double hi, double o, int n, int &i0, int &i1) {
            i0 = (int)fmax(floor((lo - o) * g.inv_c), 0.0);
            i1 = (int)fmin(floor((hi - o) * g.inv_c), (double)(n - 1));
        };
        int x0, x1, y0, y1, z0, z1;
        rng(x - 1.0 - m, x + 1.0 + m, g.ox, g.nx, x0, x1);
        rng(y - 1.0 - m, y + 1.0 + m, g.oy, g.ny, y0, y1);
        rng(-2.0 - m, 2.0 + m, g.oz, g.nz, z0, z1);
        if (x0 <= x1 && y0 <= y1 && z0 <= z1) {
            const int ny_r = y1 - y0 + 1, rows = ny_r * (z1 - z0 + 1);
            for (int r = threadIdx.x; r < rows; r += kCandT) {
                const int iy = y0 + r % ny_r, iz = z0 + r / ny_r;
                const size_t row = (size_t)g.nx * ((size_t)iy + (size_t)g.ny * iz);
                const uint32_t s = g.start[row + x0], e = g.start[row + x1 + 1];
                // four independent loads per step: a row's walk is a chain of load latencies,
                // and the maximum does not depend on the order the points come in
                for (uint32_t k0 = s; k0 < e; k0 += 4) {
                    float4 p4[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) p4[u] = g.pts[min(k0 + (uint32_t)u, e - 1)];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float4 p = p4[u];
                        if (k0 + (uint32_t)u >= e || !flann_within(qx, qy, qz, p, r2)) continue;
                        const double dx = (double)p.x - x, dy = (double)p.y - y;
                        if (sqrt(dx * dx + dy * dy) < 1.0) mz = fmax(mz, (double)p.z);
                    }
                }
            }
        }
    }
    // block max
    __shared__ double red[kCandT / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mz = fmax(mz, __shfl_xor(mz, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mz;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < kCandT / 64; ++w) mz = fmax(mz, red[w]);
    const double ground = (mz != -DBL_MAX) ? mz : 0.0;
    const double z = ground + a.sensor_height;
    const double dx = a.cx - x, dy = a.cy - y, dz = a.cz - z;
    const double hd = sqrt(dx * dx + dy * dy);
    if (hd < 0.1) {
        out[0] = 0.0;
        return;
    }
    // glibc's atan2 (the reference's) rounds correctly but for rare near-ties; ocml's is within
    // an ulp: pcp_cr_atan2_fix rounds it correctly (pcp_crmath.h, tests/test_crmath.py)
    const double elev = pcp_cr_atan2_fix(-dz, hd, atan2(-dz, hd));
    if (elev >= kMinElevation && elev <= kMaxElevation) {
        out[0] = 1.0;
        out[1] = x;
        out[2] = y;
        out[3] = z;
        out[4] = -kPi / 2 + elev;
        out[5] = pcp_cr_atan2_fix(dy, dx, atan2(dy, dx));
    } else {
        out[0] = 0.0;
    }
}

// order-preserving compaction of the lattice (single block)
__global__ void __launch_bounds__(1024)
k_cand_compact(const double *__restrict__ lat, int L, double *__restrict__ out, uint32_t *n_out,
               double *__restrict__ out_h = nullptr, uint32_t *__restrict__ n_h = nullptr) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t base_s;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int chunk = 0; chunk < L; chunk += 1024) {
        const int l = chunk + threadIdx.x;
        const bool v = l < L && lat[6 * (size_t)l] != 0.0;
        const uint64_t bal = __ballot(v);
        const uint32_t pre = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        uint32_t off = base_s;
        uint32_t tot = 0;
        for (int k = 0; k < 16; ++k) {
            if (k < w) off += wsum[k];
            tot += wsum[k];
        }
        if (v) {
            const uint32_t d = off + pre;
            for (int q = 0; q < 5; ++q) {
                const double x = lat[6 * (size_t)l + 1 + q];
                out[5 * (size_t)d + q] = x;
                if (out_h) out_h[5 * (size_t)d + q] = x;   // the host's copy (pinned)
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) base_s += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        *n_out = base_s;
        if (n_h) *n_h = base_s;
    }
}

// ---------------------------------------------------------------------------------------
// dense ray fan (BASELINE configs[1])
// ---------------------------------------------------------------------------------------
struct FanArgs {
    GridView g;
    const double *ca, *sa, *ce, *se;
    const double *pose;    // P x 8: x, y, z, pitch, yaw, cos(yaw), sin(yaw), pad
    const double *steps;
    int K;
    int n_az;
    int uniform_el;        // every wave lies in one elevation ring
    uint32_t rays;
    uint32_t waves;        // waves per pose = ceil(rays / 64)
    float r2, rexit;
    int present;
    int16_t *first_hit;
    // per-wave partials {blocked, units}, one 8-byte store per wave (no atomics), pose-major:
    // slot = p * waves + w.  Every wave of a pose runs on one XCD (the XCD-chunk kernels: XCD
    // p / (P / 8); the interleaved ones: XCD p % 8), so that XCD's L2 fills the pose's lines,
    // and k_fan_reduce reads each pose's partials as one contiguous run
    uint2 *wave_part;
    uint32_t P;
    unsigned long long *stats;     // MODE 1: probes, scanned stencils, point tests
                                   // MODE 2: per-wave s_memtime stamps [P*waves][4]
};

enum { FAN_PLAIN = 0, FAN_STATS = 1, FAN_STAMPS = 2 };

// sum over the 64 lanes (all active): rotate-adds inside each 16-lane row (DPP row_ror 8, 4,
// 2, 1), then the four row sums by readlane -- no LDS crossbar round trips
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x122, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x121, 0xF, 0xF, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// one lane = one ray; 64 consecutive azimuths of one elevation ring per wave (coherent
// termination on near-flat terrain).  Each wave writes its blocked-ray count and its
// sample-query count to its own slot: the per-pose sums are formed by k_fan_reduce in a fixed
// order (deterministic, no same-address atomics).
template <int MODE, int BS, bool ZB = true, int FN = 0, bool UE = false, int NPW = 1,
          bool SL = false>
__device__ __forceinline__ void fan_body(const FanArgs &a, uint32_t p0, uint32_t rblock) {
    const uint32_t ray = rblock * BS + threadIdx.x;
    const uint32_t wid = ray >> 6;
    const bool active = ray < a.rays;
    // the ray's direction in the pose frame, loaded once for the wave's NPW poses (poses
    // p0 .. p0 + NPW - 1 share the fan: the table loads are a quarter of the launch's
    // vector-memory bytes at NPW 1)
    double lx = 0.0, ly = 0.0, lz = 0.0;
    // SL: the step table in LDS (the launcher guarantees K <= kStepLds): one load per 64
    // entries per workgroup, then a candidate's step is an LDS read instead of a gather through
    // the texture path
    __shared__ double s_steps[SL ? kStepLds : 1];
    if (SL) {
        for (int q = threadIdx.x; q < a.K; q += BS) s_steps[q] = a.steps[q];
        __syncthreads();
    }
    const double *steps = SL ? s_steps : a.steps;
    if (active && a.present) {
        // UE (n_az % 64 == 0): the wave's ring is uniform, a scalar division of its first ray
        const uint32_t j = UE ? (rblock * BS + (threadIdx.x & ~63u)) / (uint32_t)a.n_az
                              : ray / (uint32_t)a.n_az;
        const uint32_t i = ray - j * (uint32_t)a.n_az;
        const double cej = a.ce[j];
        lx = cej * a.ca[i];
        ly = cej * a.sa[i];
        lz = a.se[j];
    }
#pragma unroll 1
    for (int q = 0; q < NPW; ++q) {
    const uint32_t p = p0 + (uint32_t)q;
    const uint32_t wslot = p * a.waves + wid;
    unsigned long long t0 = 0, t1 = 0, t2 = 0;
    if (MODE == FAN_STAMPS) t0 = __builtin_amdgcn_s_memtime();
    int hit = -1;
    uint32_t cnt[4] = {0, 0, 0, 0};   // [3]: PCP_WALK_CENSUS builds only
    if (active && a.present) {
        const double *P = a.pose + 8 * (size_t)p;
        const double cy = P[5], sy = P[6];
        const double dx = cy * lx - sy * ly;
        const double dy = sy * lx + cy * ly;
        const double dz = lz;
        if (MODE == FAN_STAMPS) {
            asm volatile("" ::"v"(dx), "v"(dy));
            t1 = __builtin_amdgcn_s_memtime();
        }
        hit = march<MODE == FAN_STATS, ZB, 1, FN>(a.g, P[0], P[1], P[2], dx, dy, dz, steps,
                                                  a.K, 1e300, a.r2, a.rexit, cnt);
    }
    if (MODE == FAN_STAMPS) {
        asm volatile("" ::"v"(hit));
        t2 = __builtin_amdgcn_s_memtime();
    }
    if (active && a.first_hit) a.first_hit[(size_t)p * a.rays + ray] = (int16_t)hit;
    const uint64_t bal = __ballot(active && hit >= 0);
    uint32_t u = active ? (hit >= 0 ? (uint32_t)hit + 1u : (uint32_t)a.K) : 0u;
    u = wave_sum_u32(u);
    if ((threadIdx.x & 63) == 0 && wid < a.waves) {
        a.wave_part[(size_t)p * a.waves + wid] = make_uint2((uint32_t)__popcll(bal), u);
    }
    if (MODE == FAN_STATS) {   // per-wave slots [4][P * waves], summed by k_sum_u64
        const size_t nw = (size_t)a.P * a.waves;
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // [3] directory loads: one per scan (none: FN, the
                                        // probe's record is the directory)
            // (a PCP_WALK_CENSUS build: FN's [3] = the walks' tests of entries r above q)
            unsigned long long v = c < 3 ? cnt[c] : (FN ? cnt[3] : cnt[1]);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
            if ((threadIdx.x & 63) == 0 && wid < a.waves) a.stats[c * nw + wslot] = v;
        }
    }
    if (MODE == FAN_STAMPS && (threadIdx.x & 63) == 0 && wid < a.waves) {
        const unsigned long long t3 = __builtin_amdgcn_s_memtime();
        unsigned long long *o = a.stats + 4 * (size_t)wslot;
        o[0] = t0;
        o[1] = t1;
        o[2] = t2;
        o[3] = t3;
    }
    }   // poses of the wave
}

// The fan kernel: one wave per workgroup (a finished wave's slot refills without waiting for
// the rest of a workgroup), 1-D grid interleaving the poses (block b = ray block b / P of pose
// b % P: the waves in flight at any time march the same ring of many poses), capped at 7 waves
// per SIMD (94 SGPRs; the compiler's own choice, 106, admits only 6).
template <int MODE, int BS = 64, bool ZB = true, int W = 7, int FN = 0, bool UE = false>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(W, W)))
k_raycast_fan(FanArgs a, uint32_t P) {
    fan_body<MODE, BS, ZB, FN, UE>(a, blockIdx.x % P, blockIdx.x / P);
}

// A/B: XCD-chunked placement (P % 8 == 0): workgroup b runs on XCD b % 8, which takes the
// contiguous pose chunk [x P/8, (x + 1) P/8) -- neighbouring candidate poses, overlapping fans
// -- interleaved inside the XCD as above
// NPW > 1: each wave marches its rays for NPW consecutive poses of the chunk (one direction-
// table load for all of them); P % (8 NPW) == 0, grid = waves * P / NPW
template <int MODE, int BS = 64, bool ZB = true, int W = 8, int FN = 1, bool UE = true, int NPW = 1>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(W, W)))
k_raycast_fan_xcd(FanArgs a, uint32_t P) {
    const uint32_t pc = P >> 3, gpc = pc / NPW, j = blockIdx.x >> 3;
    fan_body<MODE, BS, ZB, FN, UE, NPW, true>(a, (blockIdx.x & 7u) * pc + (j % gpc) * NPW,
                                             j / gpc);
}

// A/B: pose-major 2-D grid (blockIdx.y = pose), BS-thread workgroups
template <int BS, bool ZB>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(7, 7)))
k_raycast_fan_pm(FanArgs a) {
    fan_body<FAN_PLAIN, BS, ZB>(a, blockIdx.y, blockIdx.x);
}

// out[q] = sum of in[q * n .. (q + 1) * n) (one block per q)
__global__ void __launch_bounds__(1024)
k_sum_u64(const unsigned long long *__restrict__ in, size_t n, unsigned long long *__restrict__ out) {
    const unsigned long long *row = in + (size_t)blockIdx.x * n;
    unsigned long long v = 0;
    for (size_t k = threadIdx.x; k < n; k += 1024) v += row[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    __shared__ unsigned long long sw[16];
    if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < 16; ++w) t += sw[w];
        out[blockIdx.x] = t;
    }
}

// per-pose sums of the per-wave partials: one block per pose, fixed order (integer sums:
// exact and deterministic)
__global__ void __launch_bounds__(kT)
k_fan_reduce(const uint2 *__restrict__ part, uint32_t waves,
             uint32_t *__restrict__ blocked, unsigned long long *__restrict__ units,
             unsigned long long *__restrict__ keys, uint32_t lo, uint32_t Pall) {
    const uint32_t p = blockIdx.x;
    if (keys)   // (FanEnq.keys) the other ranks' slots and the health word: the MIN identity
        for (uint32_t i = p * kT + threadIdx.x; i <= Pall; i += gridDim.x * kT)
            if (i < lo || i - lo >= gridDim.x) keys[i] = ~0ull;
    const uint2 *row = part + (size_t)p * waves;   // the pose's partials, contiguous
    uint32_t b = 0;
    unsigned long long u = 0;
    for (uint32_t w = threadIdx.x; w < waves; w += kT) {
        const uint2 v = row[w];
        b += v.x;
        u += v.y;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        b += __shfl_xor(b, o, 64);
        u += __shfl_xor(u, o, 64);
    }
    __shared__ uint32_t sb[kT / 64];
    __shared__ unsigned long long su[kT / 64];
    if ((threadIdx.x & 63) == 0) {
        sb[threadIdx.x >> 6] = b;
        su[threadIdx.x >> 6] = u;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t bs = sb[0] + sb[1] + sb[2] + sb[3];
        const unsigned long long us = su[0] + su[1] + su[2] + su[3];
        blocked[p] = bs;
        units[p] = us;
        if (keys) {
            keys[lo + p] = ((unsigned long long)bs << 32) | (unsigned long long)(lo + p);
            keys[(size_t)Pall + 1 + p] = us;
        }
        // the outputs may be pinned host memory (fan_host_out): the caller reads them after
        // hipStreamSynchronize, whose completion signal carries the kernel's system-scope
        // release.  A __threadfence_system() per block here measured 11.7 vs 5.8 us per launch
        // (profiles/r02_fan_ab_fence.log) for nothing the synchronisation does not give.
    }
}

// the production fan kernel (fine tiled windows, uniform rings, XCD pose chunks) with NPW poses
// per wave; ev0/ev1 non-null: hipExtLaunchKernelGGL's start/stop events
static void launch_xcd(int npw, const FanArgs &a, uint32_t P, uint32_t waves, hipStream_t st,
                       hipEvent_t ev0, hipEvent_t ev1) {
    const dim3 g(waves * P / (uint32_t)npw);
#define PCP_XCD(N)                                                                             \
    do {                                                                                       \
        if (a.g.ftile == 2)                                                                    \
            hipExtLaunchKernelGGL((k_raycast_fan_xcd<FAN_PLAIN, 64, true, 8, 8, true, N>), g,   \
                                  dim3(64), 0, st, ev0, ev1, 0, a, P);                         \
        else                                                                                   \
            hipExtLaunchKernelGGL((k_raycast_fan_xcd<FAN_PLAIN, 64, true, 8, 4, true, N>), g,   \
                                  dim3(64), 0, st, ev0, ev1, 0, a, P);                         \
    } while (0)
    switch (npw) {
    case 2: PCP_XCD(2); break;
    case 4: PCP_XCD(4); break;
    case 8: PCP_XCD(8); break;
    case 16: PCP_XCD(16); break;
    case 32: PCP_XCD(32); break;
    default: PCP_XCD(1); break;
    }
#undef PCP_XCD
}

static VisEnv make_env(pcp_ctx *ctx, const pcp_vl_params *p, const double *steps_d, int K) {
    VisEnv E{};
    E.terrain_present = ctx->terrain.present ? 1 : 0;
    if (E.terrain_present) E.terrain = ctx->terrain.view();
    E.aux_present = (ctx->aux.present && ctx->aux_cloud_n > 0) ? 1 : 0;
    if (E.aux_present) E.aux = ctx->aux.view();
    E.max_distance = p->max_distance;
    E.steps = steps_d;
    E.K = K;
    E.r2_ray = (float)(kRayRadius * kRayRadius);
    E.r2_relaxed = (float)(kRelaxedRadius * kRelaxedRadius);
    E.rexit_ray = exit_dist(E.r2_ray);
    return E;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_set_cells(pcp_ctx *ctx, const double *xyz, const float *normals, uint64_t n) {
    if (!ctx) return PCP_E_INVALID;
    if (n && (!xyz || !normals)) return set_err(ctx, PCP_E_INVALID, "pcp_set_cells: null input");
    if (n > (1u << 30)) return set_err(ctx, PCP_E_INVALID, "pcp_set_cells: too many cells");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    if (int rc = area_finish(ctx)) return rc;   // (a setup in flight writes the same buffers)
    PCP_HIP(ctx, ctx->cells_xyz.ensure(n * 3 * sizeof(double) + 16));
    PCP_HIP(ctx, ctx->cells_nrm.ensure(n * 3 * sizeof(float) + 16));
    if (n) {   // through the pinned ring: no wait on the stream, the caller may reuse its arrays
        if (int rc = upload_async(ctx, ctx->cells_xyz.p, xyz, n * 3 * sizeof(double), ctx->stream))
            return rc;
        if (int rc = upload_async(ctx, ctx->cells_nrm.p, normals, n * 3 * sizeof(float), ctx->stream))
            return rc;
    }
    ctx->n_cells = n;
    return PCP_OK;
}

}  // extern "C"

namespace pcp {
// generateCandidatePositions' kernel arguments (:357-415)
static CandArgs cand_args(pcp_ctx *ctx, const double bb[6], const pcp_vl_params *p,
                          const double zx[5], int gs) {
    CandArgs a{};
    a.ground_enabled = (ctx->terrain_cloud_n > 0 && ctx->terrain.present) ? 1 : 0;
    if (a.ground_enabled) a.g = ctx->terrain.view();
    a.gs = gs;
    const double exminx = bb[0] - p->search_radius, exmaxx = bb[1] + p->search_radius;
    const double exminy = bb[2] - p->search_radius, exmaxy = bb[3] + p->search_radius;
    a.exminx = exminx;
    a.exminy = exminy;
    a.xs = (exmaxx - exminx) / (gs - 1);
    a.ys = (exmaxy - exminy) / (gs - 1);
    a.gminx = bb[0];
    a.gmaxx = bb[1];
    a.gminy = bb[2];
    a.gmaxy = bb[3];
    a.cx = (bb[0] + bb[1]) / 2.0;
    a.cy = (bb[2] + bb[3]) / 2.0;
    a.cz = (bb[4] + bb[5]) / 2.0;
    a.zxx = zx[0];
    a.zxy = zx[1];
    a.sensor_height = p->sensor_height;
    return a;
}

}  // namespace pcp

extern "C" {

int pcp_generate_candidates(pcp_ctx *ctx, const double bb[6], const pcp_vl_params *p,
                            const double zx[5], double *poses5, uint64_t cap, uint64_t *n_out) {
    if (!ctx) return PCP_E_INVALID;
    if (!bb || !p || !zx || !n_out || (cap && !poses5))
        return set_err(ctx, PCP_E_INVALID, "pcp_generate_candidates: null argument");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *n_out = 0;
    const int gs = (int)std::ceil(std::sqrt((double)p->num_candidates));
    if (gs <= 0) return PCP_OK;
    if ((int64_t)gs * gs > (1 << 24))
        return set_err(ctx, PCP_E_INVALID, "pcp_generate_candidates: num_candidates too large");
    CandArgs a = cand_args(ctx, bb, p, zx, gs);
    const int L = gs * gs;
    PCP_HIP(ctx, ctx->out_a.ensure((size_t)L * 6 * sizeof(double)));
    a.lat = ctx->out_a.as<double>();
    // the poses and their count are adjacent: k_cand_compact stores them straight into pinned
    // memory (one synchronisation, no copy); huge lattices go through a device buffer, the
    // count first, then the poses
    const size_t span = (size_t)L * 5 * sizeof(double) + sizeof(uint32_t);
    const bool land = span <= (4u << 20);
    double *outp;
    if (land) {
        PCP_HIP(ctx, ctx->cand_host.ensure(span));
        outp = ctx->cand_host.as<double>();
    } else {
        PCP_HIP(ctx, ctx->out_b.ensure((size_t)L * 5 * sizeof(double) + 64));
        outp = ctx->out_b.as<double>();
    }
    uint32_t *n_d = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(outp) +
                                                 (size_t)L * 5 * sizeof(double));
    {
        ProfScope ps(ctx, PCP_K_CANDIDATES);
        hipLaunchKernelGGL(k_candidates, dim3(L), dim3(kCandT), 0, ctx->stream, a);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_cand_compact, dim3(1), dim3(1024), 0, ctx->stream,
                           ctx->out_a.as<const double>(), L, outp, n_d);
        PCP_CHECK_LAUNCH(ctx);
    }
    if (!land) {
        uint32_t nh = 0;
        if (int rc0 = read_small(ctx, &nh, n_d, 4, ctx->stream)) return rc0;
        *n_out = nh;
        prof_resolve(ctx);
        if (nh > cap)
            return set_err(ctx, PCP_E_CAPACITY, "pcp_generate_candidates: need %u poses, cap %llu",
                           nh, (unsigned long long)cap);
        if (nh)
            PCP_HIP(ctx, hipMemcpyAsync(poses5, outp, (size_t)nh * 5 * sizeof(double),
                                        hipMemcpyDeviceToHost, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        return PCP_OK;
    }
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    uint32_t nh = 0;
    std::memcpy(&nh, n_d, sizeof(nh));
    *n_out = nh;
    prof_resolve(ctx);
    if (nh > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_generate_candidates: need %u poses, cap %llu", nh,
                       (unsigned long long)cap);
    if (nh) std::memcpy(poses5, outp, (size_t)nh * 5 * sizeof(double));
    return PCP_OK;
}

static int ensure_steps(pcp_ctx *ctx, double end, int *K) {
    if (ctx->steps_end == end) {
        *K = ctx->steps_K;
        return PCP_OK;
    }
    std::vector<double> s = step_table(end);
    PCP_HIP(ctx, ctx->steps_d.ensure((s.size() + 1) * sizeof(double)));
    if (!s.empty()) {
        PCP_HIP(ctx, hipMemcpyAsync(ctx->steps_d.p, s.data(), s.size() * sizeof(double),
                                    hipMemcpyHostToDevice, ctx->stream));
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->steps_end = end;
    ctx->steps_K = (int)s.size();
    *K = ctx->steps_K;
    return PCP_OK;
}

}  // extern "C"

namespace pcp {
// the production k_score_cells launch of a query (one lane per ray, or kWideG lanes per ray for
// the few-ray queries of C1 / C5); score_enqueue and pcp_score_poses_burst
static void launch_score_cells(hipStream_t st, pcp_ctx *ctx, const VisEnv &E, int C, int P,
                               const double *poses_k, const double *zx_k, const ScoreEnq &o,
                               double *score_z, const uint32_t *P_dev, const uint32_t *C_dev) {
    const unsigned cb = (unsigned)((C + kT - 1) / kT);
    const dim3 g(cb, (unsigned)(P + 1));
    const uint64_t wide_rays = ctx->score_wide_rays >= 0 ? (uint64_t)ctx->score_wide_rays
                                                         : (uint64_t)kWideMaxRays;
    const bool wide = (uint64_t)(P + 1) * (uint64_t)C <= wide_rays && ctx->score_wide;
    const int G = ctx->score_wide_g ? ctx->score_wide_g : kWideG;
    const dim3 gw((unsigned)(((uint64_t)C * G + kT - 1) / kT), (unsigned)(P + 1));
    const double *cx = ctx->cells_xyz.as<const double>();
    const float *cn = ctx->cells_nrm.as<const float>();
#define PCP_WIDE_LAUNCH(SL, GG)                                                                  \
    hipLaunchKernelGGL((k_score_cells_wide<SL, GG>), gw, dim3(kT), 0, st, E, cx, cn, C, poses_k, \
                       P, zx_k, o.comb, o.mbits, score_z, o.zbits, o.stats, P_dev, C_dev)
    if (wide && E.K <= kStepLds) {
        if (G == 2) PCP_WIDE_LAUNCH(true, 2);
        else if (G == 4) PCP_WIDE_LAUNCH(true, 4);
        else if (G == 8) PCP_WIDE_LAUNCH(true, 8);
        else PCP_WIDE_LAUNCH(true, kWideG);
    } else if (wide) {
        PCP_WIDE_LAUNCH(false, kWideG);   // (a step table past LDS: the default width only)
    } else if (E.K <= kStepLds) {
        hipLaunchKernelGGL(k_score_cells<true>, g, dim3(kT), 0, st, E, cx, cn, C, poses_k, P, zx_k,
                           o.comb, o.mbits, score_z, o.zbits, o.stats, P_dev, C_dev);
    } else {
        hipLaunchKernelGGL(k_score_cells<false>, g, dim3(kT), 0, st, E, cx, cn, C, poses_k, P,
                           zx_k, o.comb, o.mbits, score_z, o.zbits, o.stats, P_dev, C_dev);
    }
#undef PCP_WIDE_LAUNCH
}

// runOptimization's scoring up to the per-pose sums, enqueued on ctx->stream: poses + the
// zx120 pose uploaded through the pinned block, k_score_cells (rows 0..P-1 = poses, row P =
// zx120), k_row_sum.  On return the device holds comb/mbits [P][C], zbits [C], tot_d/cov_d
// [P+1] (row P = zx120); the caller synchronizes.  Validation is the caller's.
int score_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                  const pcp_vl_params *p, ScoreEnq &o, const uint8_t *cell_flags,
                  bool fuse_tail, bool zc, const uint32_t *P_dev, const double *poses_dev) {
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // a setup in flight (pcp_set_excavation_area_async): its lattice capacity is the rows'
    // stride and the grids' size, the device's count the cells (only pcp_generate_and_score
    // queries it that way: every other caller settled it first)
    const bool pend = ctx->area_pending;
    area_join(ctx);   // (a setup's side stream: the cells, their normals and count)
    const int C = pend ? (int)ctx->cells_cap : (int)ctx->n_cells, P = (int)n;
    const uint32_t *C_dev = pend ? ctx->cells_n_d.as<const uint32_t>() : nullptr;
    o.C_dev = C_dev;
    int K = 0;
    int rc = ensure_steps(ctx, p->max_distance - kVisRadius, &K);
    if (rc) return rc;
    if ((rc = terrain_blocks_before_query(ctx))) return rc;
    VisEnv E = make_env(ctx, p, ctx->steps_d.as<const double>(), K);
    // buffers.  One device block mirrors the pinned one, so a query is ONE upload and ONE
    // download: [poses + zx120 (P + 1) x 5 f64 | cell flags C | totals f64 (P + 1) | covered
    // i32 (P + 1) | stats 64 i32] -- upload [poses .. flags], download [flags .. stats]
    const size_t pc = (size_t)P * (size_t)C;
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    o.fl_off = a16((size_t)(P + 1) * 5 * sizeof(double));
    const size_t to_off = a16(o.fl_off + (size_t)C);
    o.tc_bytes = (size_t)(P + 1) * (sizeof(double) + sizeof(int32_t));
    o.st_off = a16(to_off + o.tc_bytes);
    o.blk_bytes = o.st_off + 64 * sizeof(int32_t);
    PCP_HIP(ctx, ctx->poses_d.ensure(o.blk_bytes + 64));
    PCP_HIP(ctx, ctx->out_a.ensure(pc * sizeof(double) + (size_t)C * sizeof(double) + 64));
    PCP_HIP(ctx, ctx->out_b.ensure(pc + (size_t)C * 2 + 64));
    char *blk = ctx->poses_d.as<char>();
    o.P = P;
    o.C = C;
    o.comb = ctx->out_a.as<double>();
    double *score_z = o.comb + pc;
    o.mbits = ctx->out_b.as<uint8_t>();
    o.zbits = o.mbits + pc;
    o.flags_d = reinterpret_cast<uint8_t *>(blk + o.fl_off);
    o.tot_d = reinterpret_cast<double *>(blk + to_off);
    o.cov_d = reinterpret_cast<int32_t *>(o.tot_d + (P + 1));
    o.stats = reinterpret_cast<int32_t *>(blk + o.st_off);
    PCP_HIP(ctx, ctx->res_host.ensure(o.blk_bytes + 64));
    char *pin = ctx->res_host.as<char>();
    // the candidates, then the zx120 pose behind them (row P of k_score_cells), then the
    // caller's cell flags: one upload -- or none (zc: the kernels read the pinned block)
    if (P && poses5) std::memcpy(pin, poses5, (size_t)P * 5 * sizeof(double));
    o.P_dev = P_dev;
    std::memcpy(pin + (size_t)P * 5 * sizeof(double), zx, 5 * sizeof(double));
    size_t up = (size_t)(P + 1) * 5 * sizeof(double);
    if (pend && C) {   // fresh GridCells (:259): the setup's cells start with every flag clear
        std::memset(pin + o.fl_off, 0, C);
        up = o.fl_off + C;
    } else if (cell_flags && C) {
        std::memcpy(pin + o.fl_off, cell_flags, C);
        up = o.fl_off + C;
    }
    o.zc = zc && fuse_tail && C > 0;
    const char *pose_blk = blk;
    if (o.zc) {
        pose_blk = pin;
        o.flags_d = reinterpret_cast<uint8_t *>(pin + o.fl_off);
        o.tot_d = reinterpret_cast<double *>(pin + to_off);
        o.cov_d = reinterpret_cast<int32_t *>(o.tot_d + (P + 1));
        o.stats_host = reinterpret_cast<int32_t *>(pin + o.st_off);
    } else {
        PCP_HIP(ctx, hipMemcpyAsync(blk, pin, up, hipMemcpyHostToDevice, st));
    }
    const double *poses_k = reinterpret_cast<const double *>(pose_blk);
    const double *zx_k = poses_k + 5 * (size_t)P;
    if (poses_dev) poses_k = poses_dev;   // (the zx120 pose stays in the block)
    o.poses_k = poses_k;
    o.zx_k = zx_k;
    if (C) {
        {
            ProfScope ps(ctx, PCP_K_SCORE_CELLS);
            launch_score_cells(st, ctx, E, C, P, poses_k, zx_k, o, score_z, P_dev, C_dev);
            PCP_CHECK_LAUNCH(ctx);
        }
        o.score_z = score_z;
        if (!fuse_tail) {   // (fused: k_sum_flags, launched by the caller)
            ProfScope ps(ctx, PCP_K_POSE_SUM);
            if (PCP_ROW_SUM_LANES)
                hipLaunchKernelGGL(k_row_sum_lanes, dim3((unsigned)sum_groups(P)), dim3(kT), 0, st,
                                   (const double *)o.comb, (const double *)score_z, C, P, o.tot_d,
                                   o.cov_d);
            else
                hipLaunchKernelGGL(k_row_sum, dim3(P + 1), dim3(64), 0, st, (const double *)o.comb,
                                   (const double *)score_z, C, P, o.tot_d, o.cov_d);
            PCP_CHECK_LAUNCH(ctx);
        }
    } else {
        PCP_HIP(ctx, hipMemsetAsync(o.tot_d, 0, (size_t)(P + 1) * sizeof(double), st));
        PCP_HIP(ctx, hipMemsetAsync(o.cov_d, 0, (size_t)(P + 1) * sizeof(int32_t), st));
        PCP_HIP(ctx, hipMemsetAsync(o.stats, 0, 64 * sizeof(int32_t), st));
    }
    return PCP_OK;
}

void fill_report(const int32_t *st_h, double zx_total, int64_t best_idx, double best,
                 pcp_vl_report *rep) {
    std::memset(rep, 0, sizeof(*rep));
    rep->best_idx = best_idx;
    rep->best_score = best;
    rep->zx120_total_score = zx_total;
    rep->total_cells = st_h[S_TOTAL];
    rep->zx120_range_ok = st_h[S_ZR];
    rep->zx120_fov_ok = st_h[S_ZF];
    rep->zx120_visible_ok = st_h[S_ZV];
    rep->zx120_green = st_h[S_ZG];
    rep->zx120_red = st_h[S_ZRED];
    rep->zx120_blue = st_h[S_ZB];
    rep->zx120_yellow = st_h[S_ZY];
    rep->green = st_h[S_G];
    rep->red = st_h[S_RED];
    rep->blue = st_h[S_B];
    rep->yellow = st_h[S_Y];
}
}  // namespace pcp

extern "C" {

int pcp_score_poses(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                    const pcp_vl_params *p, uint8_t *cell_flags, double *total_score,
                    int32_t *covered, pcp_vl_report *rep) {
    if (!ctx) return PCP_E_INVALID;
    if (int rc = area_finish(ctx)) return rc;   // (the host's flags need the settled count)
    if (!zx || !p || !rep || (n && !poses5) || (ctx->n_cells && !cell_flags))
        return set_err(ctx, PCP_E_INVALID, "pcp_score_poses: null argument");
    if (n > 65535) return set_err(ctx, PCP_E_INVALID, "pcp_score_poses: at most 65535 poses per call");
    ScoreEnq o;
    if (int rc = score_enqueue(ctx, poses5, n, zx, p, o, cell_flags, true, ctx->zc_in)) return rc;
    hipStream_t st = ctx->stream;
    const int C = o.C, P = o.P;
    char *pin = ctx->res_host.as<char>();
    if (C) {   // the ordered row sums and the stale-flag resolution side by side
        ProfScope ps(ctx, PCP_K_POSE_SUM);
        hipLaunchKernelGGL(k_sum_flags,
                           dim3((unsigned)(sum_flag_row_blocks(P) + (C + kT - 1) / kT)), dim3(kT),
                           0,
                           st, (const double *)o.comb, (const double *)o.score_z, C, P, o.tot_d,
                           o.cov_d, (const uint8_t *)o.zbits, (const uint8_t *)o.mbits, o.flags_d,
                           o.stats, o.stats_host, o.P_dev, o.C_dev);
        PCP_CHECK_LAUNCH(ctx);
    }
    // flags, totals, covered counts and statistics are one span of the block: one download
    // (zc: the kernels stored them in the pinned block)
    if (!o.zc)
        PCP_HIP(ctx, hipMemcpyAsync(pin + o.fl_off, reinterpret_cast<const char *>(o.flags_d),
                                    o.blk_bytes - o.fl_off, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    const double *tot_h = o.zc ? o.tot_d
                               : reinterpret_cast<const double *>(
                                     pin + (reinterpret_cast<const char *>(o.tot_d) -
                                            ctx->poses_d.as<const char>()));
    const int32_t *cov_h = reinterpret_cast<const int32_t *>(tot_h + (P + 1));
    const int32_t *st_h = reinterpret_cast<const int32_t *>(pin + o.st_off);
    if (C) std::memcpy(cell_flags, pin + o.fl_off, C);
    prof_resolve(ctx);
    // runOptimization candidate loop (:464-475): strict '>' keeps the first maximum
    double best = -INFINITY;
    int64_t best_idx = -1;
    for (int k = 0; k < P; ++k) {
        if (total_score) total_score[k] = tot_h[k];
        if (covered) covered[k] = cov_h[k];
        if (tot_h[k] > best) {
            best = tot_h[k];
            best_idx = k;
        }
    }
    fill_report(st_h, tot_h[P], best_idx, best, rep);
    return PCP_OK;
}

// the roofline's inputs for the reference's own ray march (k_score_cells): the query's
// production launch set up by score_enqueue, then either its lane-loads counted by the STATS
// twin or the production launch `reps` times back-to-back between two events
static int score_diag(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                      const pcp_vl_params *p, uint64_t *stats, int reps, double *ms) {
    if (!ctx) return PCP_E_INVALID;
    if (int rc = area_finish(ctx)) return rc;
    if (!zx || !p || (n && !poses5))
        return set_err(ctx, PCP_E_INVALID, "pcp_score_poses_stats/burst: null argument");
    if (n > 65535) return set_err(ctx, PCP_E_INVALID, "pcp_score_poses_stats/burst: too many poses");
    ScoreEnq o;
    if (int rc = score_enqueue(ctx, poses5, n, zx, p, o)) return rc;
    hipStream_t st = ctx->stream;
    const int C = o.C, P = o.P;
    int K = 0;
    if (int rc = ensure_steps(ctx, p->max_distance - kVisRadius, &K)) return rc;
    const VisEnv E = make_env(ctx, p, ctx->steps_d.as<const double>(), K);
    if (stats) {
        PCP_HIP(ctx, ctx->stats_d.ensure(4 * sizeof(unsigned long long) + 64));
        unsigned long long *sd = ctx->stats_d.as<unsigned long long>();
        PCP_HIP(ctx, hipMemsetAsync(sd, 0, 4 * sizeof(unsigned long long), st));
        if (C) {
            const dim3 g((unsigned)((C + kT - 1) / kT), (unsigned)(P + 1));
            if (E.K <= kStepLds)
                hipLaunchKernelGGL(k_score_cells_stats<true>, g, dim3(kT), 0, st, E,
                                   ctx->cells_xyz.as<const double>(),
                                   ctx->cells_nrm.as<const float>(), C, o.poses_k, P, o.zx_k, sd);
            else
                hipLaunchKernelGGL(k_score_cells_stats<false>, g, dim3(kT), 0, st, E,
                                   ctx->cells_xyz.as<const double>(),
                                   ctx->cells_nrm.as<const float>(), C, o.poses_k, P, o.zx_k, sd);
            PCP_CHECK_LAUNCH(ctx);
        }
        unsigned long long h[4] = {0, 0, 0, 0};
        PCP_HIP(ctx, hipMemcpyAsync(h, sd, sizeof(h), hipMemcpyDeviceToHost, st));
        PCP_HIP(ctx, hipStreamSynchronize(st));
        for (int i = 0; i < 4; ++i) stats[i] = h[i];
    }
    if (ms) {
        *ms = 0.0;
        hipEvent_t a = nullptr, b = nullptr;
        PCP_HIP(ctx, hipEventCreate(&a));
        PCP_HIP(ctx, hipEventCreate(&b));
        hipError_t e = hipEventRecord(a, st);
        for (int r = 0; r < reps && e == hipSuccess && C; ++r) {
            launch_score_cells(st, ctx, E, C, P, o.poses_k, o.zx_k, o, o.score_z, nullptr, nullptr);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(b, st);
        if (e == hipSuccess) e = hipEventSynchronize(b);
        float t = 0.0f;
        if (e == hipSuccess) e = hipEventElapsedTime(&t, a, b);
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        if (e != hipSuccess) return hip_fail(ctx, e, "pcp_score_poses_burst", __FILE__, __LINE__);
        *ms = (double)t / reps;
    }
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
    return PCP_OK;
}

int pcp_score_matrix(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                     const pcp_vl_params *p, double *score_mobile, double *score_zx120) {
    if (!ctx) return PCP_E_INVALID;
    if (int rc = area_finish(ctx)) return rc;
    if (!zx || !p || (n && !poses5) || (ctx->n_cells && (!score_zx120 || (n && !score_mobile))))
        return set_err(ctx, PCP_E_INVALID, "pcp_score_matrix: null argument");
    if (n > 65535) return set_err(ctx, PCP_E_INVALID, "pcp_score_matrix: too many poses");
    ScoreEnq o;
    if (int rc = score_enqueue(ctx, poses5, n, zx, p, o)) return rc;
    hipStream_t st = ctx->stream;
    const size_t C = (size_t)o.C, P = (size_t)o.P;
    if (C) {
        if (P)
            PCP_HIP(ctx, hipMemcpyAsync(score_mobile, o.comb, P * C * sizeof(double),
                                        hipMemcpyDeviceToHost, st));
        PCP_HIP(ctx, hipMemcpyAsync(score_zx120, o.score_z, C * sizeof(double),
                                    hipMemcpyDeviceToHost, st));
    }
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
    return PCP_OK;
}

int pcp_score_poses_stats(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                          const pcp_vl_params *p, uint64_t stats[4]) {
    if (!ctx || !stats) return PCP_E_INVALID;
    stats[0] = stats[1] = stats[2] = stats[3] = 0;
    return score_diag(ctx, poses5, n, zx, p, stats, 0, nullptr);
}

int pcp_score_poses_burst(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                          const pcp_vl_params *p, int reps, double *ms_per_launch) {
    if (!ctx || !ms_per_launch || reps <= 0) return PCP_E_INVALID;
    return score_diag(ctx, poses5, n, zx, p, nullptr, reps, ms_per_launch);
}

int pcp_generate_and_score(pcp_ctx *ctx, const double bb[6], const pcp_vl_params *p,
                           const double zx[5], double *poses5, uint64_t cap, uint64_t *n_out,
                           uint8_t *cell_flags, double *total_score, int32_t *covered,
                           pcp_vl_report *rep) {
    if (!ctx) return PCP_E_INVALID;
    const bool pend = ctx->area_pending;
    if (!bb || !p || !zx || !n_out || !rep || (cap && !poses5) ||
        ((pend ? ctx->cells_cap : ctx->n_cells) && !cell_flags))
        return set_err(ctx, PCP_E_INVALID, "pcp_generate_and_score: null argument");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    *n_out = 0;
    const int gs = (int)std::ceil(std::sqrt((double)p->num_candidates));
    const int64_t L = gs > 0 ? (int64_t)gs * gs : 0;
    if (pend && (L == 0 || L > 65535 || !ctx->zc_in || !PCP_ROW_SUM_LANES)) {
        // the two-call path needs the count on the host: settle the setup (fresh flags, :259)
        if (int rc = area_finish(ctx)) return rc;
        if (ctx->n_cells) std::memset(cell_flags, 0, ctx->n_cells);
        return pcp_generate_and_score(ctx, bb, p, zx, poses5, cap, n_out, cell_flags, total_score,
                                      covered, rep);
    }
    if (L == 0 || L > 65535 || !ctx->zc_in) {   // the two calls (one synchronisation each)
        uint64_t n = 0;
        if (int rc = pcp_generate_candidates(ctx, bb, p, zx, poses5, cap, &n)) return rc;
        *n_out = n;
        return pcp_score_poses(ctx, poses5, n, zx, p, cell_flags, total_score, covered, rep);
    }
    // candidates -> device poses + their count (and the host's pinned copies), scoring sized
    // for the whole lattice with the count read on the device: one synchronisation
    CandArgs a = cand_args(ctx, bb, p, zx, gs);
    PCP_HIP(ctx, ctx->out_a.ensure((size_t)L * 6 * sizeof(double)));
    a.lat = ctx->out_a.as<double>();
    PCP_HIP(ctx, ctx->out_d.ensure((size_t)L * 5 * sizeof(double) + 64));
    double *poses_d = ctx->out_d.as<double>();
    uint32_t *n_d = reinterpret_cast<uint32_t *>(poses_d + 5 * (size_t)L);
    const size_t span = (size_t)L * 5 * sizeof(double) + sizeof(uint32_t);
    PCP_HIP(ctx, ctx->cand_host.ensure(span));
    double *poses_h = ctx->cand_host.as<double>();
    uint32_t *n_h = reinterpret_cast<uint32_t *>(poses_h + 5 * (size_t)L);
    {
        ProfScope ps(ctx, PCP_K_CANDIDATES);
        hipLaunchKernelGGL(k_candidates, dim3((unsigned)L), dim3(kCandT), 0, ctx->stream, a);
        PCP_CHECK_LAUNCH(ctx);
        hipLaunchKernelGGL(k_cand_compact, dim3(1), dim3(1024), 0, ctx->stream,
                           ctx->out_a.as<const double>(), (int)L, poses_d, n_d, poses_h, n_h);
        PCP_CHECK_LAUNCH(ctx);
    }
    ScoreEnq o;
    if (int rc = score_enqueue(ctx, nullptr, (uint64_t)L, zx, p, o, cell_flags, true, true, n_d,
                               poses_d))
        return rc;
    hipStream_t st = ctx->stream;
    const int C = o.C;
    char *pin = ctx->res_host.as<char>();
    if (C) {
        ProfScope ps(ctx, PCP_K_POSE_SUM);
        hipLaunchKernelGGL(k_sum_flags,
                           dim3((unsigned)(sum_flag_row_blocks((int)L) + (C + kT - 1) / kT)),
                           dim3(kT), 0, st, (const double *)o.comb, (const double *)o.score_z, C,
                           (int)L, o.tot_d, o.cov_d, (const uint8_t *)o.zbits,
                           (const uint8_t *)o.mbits, o.flags_d, o.stats, o.stats_host, n_d,
                           o.C_dev);
        PCP_CHECK_LAUNCH(ctx);
    }
    if (!o.zc)   // no cells: the zeroed totals and statistics
        PCP_HIP(ctx, hipMemcpyAsync(pin + o.fl_off, reinterpret_cast<const char *>(o.flags_d),
                                    o.blk_bytes - o.fl_off, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    if (pend) {
        // the setup ran in front of this tick on the stream: an overflow of its neighbour lists
        // left the cells' normals incomplete -- settle it (regrow, rerun) and tick again from
        // fresh flags; otherwise its count is final (area_finish returns at once)
        const bool over = area_overflowed(ctx);
        if (int rc = area_finish(ctx, true)) return rc;   // (joined by score_enqueue, synced)
        if (over) {
            if (ctx->n_cells) std::memset(cell_flags, 0, ctx->n_cells);
            return pcp_generate_and_score(ctx, bb, p, zx, poses5, cap, n_out, cell_flags,
                                          total_score, covered, rep);
        }
    }
    const int Cn = pend ? (int)ctx->n_cells : C;   // the cells (C: the grids' size)
    const uint32_t P = *n_h;
    *n_out = P;
    prof_resolve(ctx);
    if (P > cap)
        return set_err(ctx, PCP_E_CAPACITY, "pcp_generate_and_score: need %u poses, cap %llu", P,
                       (unsigned long long)cap);
    if (P) std::memcpy(poses5, poses_h, (size_t)P * 5 * sizeof(double));
    const double *tot_h = o.zc ? o.tot_d
                               : reinterpret_cast<const double *>(
                                     pin + (reinterpret_cast<const char *>(o.tot_d) -
                                            ctx->poses_d.as<const char>()));
    const int32_t *cov_h = reinterpret_cast<const int32_t *>(tot_h + (L + 1));
    const int32_t *st_h = reinterpret_cast<const int32_t *>(pin + o.st_off);
    if (Cn) std::memcpy(cell_flags, pin + o.fl_off, Cn);
    double best = -INFINITY;
    int64_t best_idx = -1;
    for (uint32_t k = 0; k < P; ++k) {   // :464-475, strict '>' keeps the first maximum
        if (total_score) total_score[k] = tot_h[k];
        if (covered) covered[k] = cov_h[k];
        if (tot_h[k] > best) {
            best = tot_h[k];
            best_idx = k;
        }
    }
    fill_report(st_h, tot_h[P], best_idx, best, rep);
    return PCP_OK;
}

}  // extern "C"

namespace pcp {
// Everything of a fan query up to the per-pose sums, enqueued on ctx->stream (no host sync
// unless the fan tables or the step table change): poses uploaded through the pinned block,
// the march, k_fan_reduce.  On return o.blocked_d / o.units_d (and o.fh_d when want_fh) are
// device results in flight; the caller synchronizes.  n > 0.
int fan_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n, const pcp_fan_params *fan,
                bool want_fh, bool stats, bool stamps, FanEnq &o, int burst, double *burst_ms,
                bool host_out) {
    if (fan->n_az <= 0 || fan->n_el <= 0 || (int64_t)fan->n_az * fan->n_el > (1ll << 30))
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: bad fan size %d x %d", fan->n_az,
                       fan->n_el);
    if (n > 65535) return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: at most 65535 poses per call");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int P = (int)n;
    const uint32_t rays = (uint32_t)fan->n_az * (uint32_t)fan->n_el;
    // direction tables (host libm, identical to the oracle), cached per fan shape
    const size_t tab_doubles = 2 * (size_t)fan->n_az + 2 * (size_t)fan->n_el;
    if (ctx->fan_naz != fan->n_az || ctx->fan_nel != fan->n_el || ctx->fan_elmin != fan->el_min ||
        ctx->fan_elmax != fan->el_max) {
        std::vector<double> t(tab_doubles);
        fan_tables(fan->n_az, fan->n_el, fan->el_min, fan->el_max, t.data(), t.data() + fan->n_az,
                   t.data() + 2 * fan->n_az, t.data() + 2 * fan->n_az + fan->n_el);
        PCP_HIP(ctx, ctx->fan_tab.ensure(tab_doubles * sizeof(double)));
        PCP_HIP(ctx, hipMemcpyAsync(ctx->fan_tab.p, t.data(), tab_doubles * sizeof(double),
                                    hipMemcpyHostToDevice, st));
        PCP_HIP(ctx, hipStreamSynchronize(st));
        ctx->fan_naz = fan->n_az;
        ctx->fan_nel = fan->n_el;
        ctx->fan_elmin = fan->el_min;
        ctx->fan_elmax = fan->el_max;
    }
    int K = 0;
    int rc = ensure_steps(ctx, fan->max_distance - kVisRadius, &K);
    if (rc) return rc;
    // a keys query handed to a wait_stream may not have uploaded its poses yet: its copy reads
    // the pinned staging below, so that copy must be done before the staging is rewritten (or
    // regrown) by this query, whichever entry point enqueues it
    if (ctx->keys_pending) PCP_HIP(ctx, hipEventSynchronize(ctx->keys_ev));
    ctx->keys_pending = false;
    // pinned staging: poses in (P x 8 doubles), then {units u64[P], blocked u32[P]} out
    PCP_HIP(ctx, ctx->fan_host.ensure((size_t)P * (8 * sizeof(double) + 12) + 64));
    double *pose8 = ctx->fan_host.as<double>();
    for (int k = 0; k < P; ++k) {
        const double *s = poses5 + 5 * (size_t)k;
        double *d = pose8 + 8 * (size_t)k;
        for (int q = 0; q < 5; ++q) d[q] = s[q];
        d[5] = std::cos(s[4]);
        d[6] = std::sin(s[4]);
        d[7] = 0.0;
    }
    PCP_HIP(ctx, ctx->poses_d.ensure((size_t)P * 8 * sizeof(double)));
    const uint32_t waves = (rays + 63) / 64;
    if ((uint64_t)waves * (uint64_t)P >= (1ull << 31))
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: %d poses x %u rays exceed one launch",
                       P, rays);
    PCP_HIP(ctx, ctx->out_c.ensure((size_t)P * (sizeof(uint32_t) + sizeof(uint64_t)) + 64));
    PCP_HIP(ctx, ctx->out_b.ensure(((size_t)P * waves + 8) * sizeof(uint2)));
    // stamps: 4 per wave; stats: 3 per wave + the 3 sums
    const size_t stats_bytes = stamps  ? (size_t)P * waves * 4 * sizeof(uint64_t)
                               : stats ? ((size_t)P * waves * 4 + 4) * sizeof(uint64_t)
                                       : 64 * sizeof(uint64_t);
    PCP_HIP(ctx, ctx->stats_d.ensure(stats_bytes));
    if (int rc0 = copy_pinned_async(ctx, ctx->poses_d.p, pose8, (size_t)P * 8 * sizeof(double), st))
        return rc0;
    // results land in device memory, or (host_out) straight in the pinned block behind the
    // staged poses: one copy and its dispatch fewer per query
    unsigned long long *units_d =
        host_out ? reinterpret_cast<unsigned long long *>(pose8 + 8 * (size_t)P)
                 : ctx->out_c.as<unsigned long long>();
    uint32_t *blocked_d = reinterpret_cast<uint32_t *>(units_d + P);
    int16_t *fh_d = nullptr;
    if (want_fh) {
        PCP_HIP(ctx, ctx->out_d.ensure((size_t)P * rays * sizeof(int16_t)));
        fh_d = ctx->out_d.as<int16_t>();
    }
    if (int rcb = terrain_blocks_before_query(ctx)) return rcb;
    FanArgs a{};
    a.present = ctx->terrain.present ? 1 : 0;
    if (a.present) {
        a.g = ctx->terrain.view();
        if (!a.g.occz) return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: terrain index has no z bands");
        if (ctx->fan_batch == 2 && !a.g.occ2)
            return set_err(ctx, PCP_E_STATE, "pcp_raycast_fan: variant 2 needs a terrain set with PCP_FAN_BATCH=2");
    }
    const double *tab = ctx->fan_tab.as<const double>();
    a.ca = tab;
    a.sa = tab + fan->n_az;
    a.ce = tab + 2 * fan->n_az;
    a.se = tab + 2 * fan->n_az + fan->n_el;
    a.pose = ctx->poses_d.as<const double>();
    a.steps = ctx->steps_d.as<const double>();
    a.K = K;
    a.n_az = fan->n_az;
    a.uniform_el = (fan->n_az % 64 == 0) ? 1 : 0;
    a.rays = rays;
    a.waves = waves;
    a.P = (uint32_t)P;
    a.r2 = (float)(kRayRadius * kRayRadius);
    a.rexit = exit_dist(a.r2);
    a.first_hit = fh_d;
    a.wave_part = ctx->out_b.as<uint2>();
    a.stats = ctx->stats_d.as<unsigned long long>();
    const dim3 grid1(waves * (uint32_t)P);           // 64-thread blocks, pose-interleaved
    // the fine-window kernels (28 VGPRs, 8 waves per SIMD), the ring index a
    // scalar when n_az % 64 == 0 (UE); the coarse layouts' kernel otherwise
    const bool fine = a.g.frec != nullptr, ue = a.uniform_el != 0, tile = a.g.ftile != 0;
    const bool split = a.g.ftile == 2;
    // poses per wave: the largest of ctx->fan_npw, ..., 2, 1 that divides the XCD pose chunk
    int npw = ctx->fan_npw;
    while (npw > 1 && P % (8 * npw) != 0) npw >>= 1;
#define PCP_FAN_LAUNCH(MODE)                                                                   \
    do {                                                                                       \
        if (fine && split && ue)                                                               \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 8, true>), grid1, dim3(64), 0, \
                               st, a, (uint32_t)P);                                            \
        else if (fine && split)                                                                \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 8, false>), grid1, dim3(64), 0,\
                               st, a, (uint32_t)P);                                            \
        else if (fine && tile && ue)                                                           \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 4, true>), grid1, dim3(64), 0, \
                               st, a, (uint32_t)P);                                            \
        else if (fine && tile)                                                                 \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 4, false>), grid1, dim3(64), 0,\
                               st, a, (uint32_t)P);                                            \
        else if (fine && ue)                                                                   \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 1, true>), grid1, dim3(64), 0, \
                               st, a, (uint32_t)P);                                            \
        else if (fine)                                                                         \
            hipLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 1, false>), grid1, dim3(64), 0,\
                               st, a, (uint32_t)P);                                            \
        else                                                                                   \
            hipLaunchKernelGGL((k_raycast_fan<MODE>), grid1, dim3(64), 0, st, a, (uint32_t)P); \
    } while (0)
#define PCP_FAN_LAUNCH_T(MODE)                                                                 \
    do {                                                                                       \
        if (fine && split && ue)                                                               \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 8, true>), grid1, dim3(64), \
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else if (fine && split)                                                                \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 8, false>), grid1, dim3(64),\
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else if (fine && tile && ue)                                                           \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 4, true>), grid1, dim3(64), \
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else if (fine && tile)                                                                 \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 4, false>), grid1, dim3(64),\
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else if (fine && ue)                                                                   \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 1, true>), grid1, dim3(64), \
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else if (fine)                                                                         \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE, 64, true, 8, 1, false>), grid1, dim3(64),\
                                  0, st, kt.a, kt.b, 0, a, (uint32_t)P);                       \
        else                                                                                   \
            hipExtLaunchKernelGGL((k_raycast_fan<MODE>), grid1, dim3(64), 0, st, kt.a, kt.b, 0, \
                                  a, (uint32_t)P);                                             \
    } while (0)
    if (stats) {
        PCP_FAN_LAUNCH(FAN_STATS);
        PCP_CHECK_LAUNCH(ctx);
        const size_t nw = (size_t)P * waves;
        hipLaunchKernelGGL(k_sum_u64, dim3(4), dim3(1024), 0, st,
                           (const unsigned long long *)a.stats, nw, a.stats + 4 * nw);
        PCP_CHECK_LAUNCH(ctx);
        o.stats_d = a.stats + 4 * nw;
    } else if (stamps) {
        PCP_FAN_LAUNCH(FAN_STAMPS);
        PCP_CHECK_LAUNCH(ctx);
        o.stats_d = a.stats;
    } else if (burst > 0) {
        // the production kernel `burst` times back-to-back between two events: the queue never
        // idles between the events, so the interval is the launches themselves (the per-call
        // events of a synchronous query also hold the queue's wake-up before the kernel)
        hipEvent_t e0 = nullptr, e1 = nullptr;
        PCP_HIP(ctx, hipEventCreate(&e0));
        PCP_HIP(ctx, hipEventCreate(&e1));
        PCP_HIP(ctx, hipEventRecord(e0, st));
        for (int r = 0; r < burst; ++r) {
            if (fine && tile && ue && P % (8 * npw) == 0 && K <= kStepLds)
                launch_xcd(npw, a, (uint32_t)P, waves, st, nullptr, nullptr);
            else if (fine && ue && P % 8 == 0 && K <= kStepLds)
                hipLaunchKernelGGL((k_raycast_fan_xcd<FAN_PLAIN>), grid1, dim3(64), 0, st, a,
                                   (uint32_t)P);
            else
                PCP_FAN_LAUNCH(FAN_PLAIN);
        }
        PCP_CHECK_LAUNCH(ctx);
        PCP_HIP(ctx, hipEventRecord(e1, st));
        PCP_HIP(ctx, hipEventSynchronize(e1));
        float ms = 0.0f;
        PCP_HIP(ctx, hipEventElapsedTime(&ms, e0, e1));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (burst_ms) *burst_ms = (double)ms / burst;
    } else {
        KernelTimer kt(ctx, PCP_K_RAYCAST_FAN);   // events around the kernel itself
        // PCP_FAN_BATCH selects the A/B variants of DESIGN.md §6b
        const dim3 grid128((rays + 127) / 128, P);
        switch (ctx->fan_batch) {
        case 1: hipExtLaunchKernelGGL((k_raycast_fan_pm<128, true>), grid128, dim3(128), 0, st, kt.a, kt.b, 0, a); break;
        case 2: hipExtLaunchKernelGGL((k_raycast_fan<FAN_PLAIN, 64, false>), grid1, dim3(64), 0, st, kt.a, kt.b, 0, a, (uint32_t)P); break;
        case 4: PCP_FAN_LAUNCH_T(FAN_PLAIN); break;   // A/B: plain pose interleaving
        default:
            // XCD-chunked placement (each XCD's L2 serves neighbouring poses' overlapping fans):
            // 0.61 vs 0.63 ms on C2
            if (fine && tile && ue && P % (8 * npw) == 0 && K <= kStepLds)
                launch_xcd(npw, a, (uint32_t)P, waves, st, kt.a, kt.b);
            else if (fine && ue && P % 8 == 0 && K <= kStepLds)
                hipExtLaunchKernelGGL((k_raycast_fan_xcd<FAN_PLAIN>), grid1, dim3(64), 0, st, kt.a,
                                      kt.b, 0, a, (uint32_t)P);
            else
                PCP_FAN_LAUNCH_T(FAN_PLAIN);
            break;
        }
        PCP_CHECK_LAUNCH(ctx);
    }
#undef PCP_FAN_LAUNCH
#undef PCP_FAN_LAUNCH_T
    hipLaunchKernelGGL(k_fan_reduce, dim3(P), dim3(kT), 0, st,
                       (const uint2 *)a.wave_part, waves, blocked_d,
                       units_d, o.keys, o.keys_lo, o.keys_P);
    PCP_CHECK_LAUNCH(ctx);
    o.blocked_d = host_out ? nullptr : blocked_d;
    o.units_d = host_out ? nullptr : units_d;
    o.fh_d = fh_d;
    o.rays = rays;
    o.stats_bytes = stats_bytes;
    return PCP_OK;
}
}  // namespace pcp

extern "C" {

static int raycast_fan_impl(pcp_ctx *ctx, const double *poses5, uint64_t n,
                            const pcp_fan_params *fan, uint32_t *blocked, uint64_t *units,
                            int16_t *first_hit, int64_t *best_idx, uint64_t *stats,
                            uint64_t *stamps, int burst = 0, double *burst_ms = nullptr) {
    if (!ctx) return PCP_E_INVALID;
    if (!fan || (n && (!poses5 || !blocked)))
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: null argument");
    if (best_idx) *best_idx = -1;
    if (n == 0) {
        if (fan->n_az <= 0 || fan->n_el <= 0 || (int64_t)fan->n_az * fan->n_el > (1ll << 30))
            return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan: bad fan size %d x %d",
                           fan->n_az, fan->n_el);
        return PCP_OK;
    }
    FanEnq o;
    const bool host_out = ctx->fan_host_out;
    if (int rc = fan_enqueue(ctx, poses5, n, fan, first_hit != nullptr, stats != nullptr,
                             stamps != nullptr, o, burst, burst_ms, host_out))
        return rc;
    hipStream_t st = ctx->stream;
    const int P = (int)n;
    const uint32_t rays = o.rays;
    if (stats)
        PCP_HIP(ctx, hipMemcpyAsync(stats, o.stats_d, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                    st));
    if (stamps)
        PCP_HIP(ctx, hipMemcpyAsync(stamps, o.stats_d, o.stats_bytes, hipMemcpyDeviceToHost, st));
    // units and blocked are adjacent on the device: one copy into the pinned block
    double *pose8 = ctx->fan_host.as<double>();
    uint64_t *u_h = reinterpret_cast<uint64_t *>(pose8 + 8 * (size_t)P);
    const uint32_t *b_h = reinterpret_cast<const uint32_t *>(u_h + P);
    if (!host_out)   // else k_fan_reduce stored them into u_h / b_h itself
        PCP_HIP(ctx, hipMemcpyAsync(u_h, o.units_d, (size_t)P * 12, hipMemcpyDeviceToHost, st));
    if (first_hit)
        PCP_HIP(ctx, hipMemcpyAsync(first_hit, o.fh_d, (size_t)P * rays * sizeof(int16_t),
                                    hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
    std::memcpy(blocked, b_h, (size_t)P * sizeof(uint32_t));
    if (units)
        for (int k = 0; k < P; ++k) units[k] = u_h[k];
    if (best_idx) {
        int64_t b = 0;
        for (int k = 1; k < P; ++k)
            if (blocked[k] < blocked[b]) b = k;
        *best_idx = b;
    }
    return PCP_OK;
}

int pcp_raycast_fan(pcp_ctx *ctx, const double *poses5, uint64_t n, const pcp_fan_params *fan,
                    uint32_t *blocked, uint64_t *units, int16_t *first_hit, int64_t *best_idx) {
    return raycast_fan_impl(ctx, poses5, n, fan, blocked, units, first_hit, best_idx, nullptr,
                            nullptr);
}

int pcp_raycast_fan_stats(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, uint64_t stats[4]) {
    if (!ctx || !stats) return PCP_E_INVALID;
    std::vector<uint32_t> blocked(n ? n : 1);
    stats[0] = stats[1] = stats[2] = stats[3] = 0;
    return raycast_fan_impl(ctx, poses5, n, fan, blocked.data(), nullptr, nullptr, nullptr, stats,
                            nullptr);
}

int pcp_raycast_fan_burst(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, int reps, double *ms_per_launch) {
    if (!ctx || !ms_per_launch || reps <= 0) return PCP_E_INVALID;
    std::vector<uint32_t> blocked(n ? n : 1);
    *ms_per_launch = 0.0;
    return raycast_fan_impl(ctx, poses5, n, fan, blocked.data(), nullptr, nullptr, nullptr,
                            nullptr, nullptr, reps, ms_per_launch);
}

int pcp_raycast_fan_stamps(pcp_ctx *ctx, const double *poses5, uint64_t n,
                           const pcp_fan_params *fan, uint64_t *stamps) {
    if (!ctx || !stamps) return PCP_E_INVALID;
    std::vector<uint32_t> blocked(n ? n : 1);
    return raycast_fan_impl(ctx, poses5, n, fan, blocked.data(), nullptr, nullptr, nullptr,
                            nullptr, stamps);
}

// one rank's shard of a pose-sharded fan query whose collective the caller runs (one process
// per GPU, torch.distributed over RCCL): keys stay on the device, in the caller's buffer
int pcp_raycast_fan_keys(pcp_ctx *ctx, const double *poses5, uint64_t n,
                         const pcp_fan_params *fan, uint64_t lo, uint64_t p_total,
                         int64_t *keys_dev, uint64_t *units_dev, void *wait_stream) {
    if (!ctx) return PCP_E_INVALID;
    if (!fan || !keys_dev || (n && !poses5))
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan_keys: null argument");
    if (lo + n > p_total || p_total > 65535u * 64u)
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan_keys: shard [%llu, %llu) of %llu poses",
                       (unsigned long long)lo, (unsigned long long)(lo + n),
                       (unsigned long long)p_total);
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // (fan_enqueue waits for a previous keys query's pose upload before it rewrites the
    // pinned staging; an n == 0 shard touches no staging)
    const uint32_t *blocked_d = nullptr;
    if (n) {
        FanEnq o;
        if (int rc = fan_enqueue(ctx, poses5, n, fan, false, false, false, o)) return rc;
        blocked_d = o.blocked_d;
        if (units_dev)
            PCP_HIP(ctx, hipMemcpyAsync(units_dev, o.units_d, n * sizeof(uint64_t),
                                        hipMemcpyDeviceToDevice, st));
    }
    launch_fan_keys(st, blocked_d, (uint32_t)lo, (uint32_t)n, (uint32_t)p_total,
                    reinterpret_cast<unsigned long long *>(keys_dev), 0x7fffffffffffffffull);
    PCP_CHECK_LAUNCH(ctx);
    if (!ctx->keys_ev) PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->keys_ev, hipEventDisableTiming));
    PCP_HIP(ctx, hipEventRecord(ctx->keys_ev, st));
    if (wait_stream) {
        PCP_HIP(ctx, hipStreamWaitEvent(static_cast<hipStream_t>(wait_stream), ctx->keys_ev, 0));
        ctx->keys_pending = true;
    } else {
        PCP_HIP(ctx, hipEventSynchronize(ctx->keys_ev));
    }
    return PCP_OK;
}

}  // extern "C"
