// pcp_fine.hip -- the fine-window copy of the terrain index, the layout the
// ray march walks once a terrain is queried repeatedly.
//
// The xy plane is cut into fine cells of c_f = c / F (F = PCP_TERRAIN_FINE, default 2: 0.06 m
// for the ray radius).  The WINDOW of fine cell W holds every point whose xy distance to W's
// rectangle is at most R = r + m: a rounded square that contains the radius-r disk around any
// query whose xy lies in W (or within float rounding of it) -- 0.027 m^2 at F = 2 against the
// 0.058 m^2 of the 2x2x2 block's square (F = 3: 0.021 m^2, fewer point tests but 2.25x the
// records for the probes to gather: measured slower).  Each window's points are
// one run in descending z (ties by original index, as k_cell_rank_z), ended by a sentinel
// (x, y NaN: never within r; z -inf: always r below).  One 8-byte record per (fine cell x, y,
// coarse z corner iz), in 4 x 4 xy tiles of one 128-byte line (PCP_FINE_TILE; 0: x-fastest):
// {first point of the window in coarse z cells <= iz + 1, probe thresholds}; the walk stops at
// the first point r below q, at the latest the first point below cell iz, or at the sentinel.
//
// Build (all on the device, O(pairs log)): global z order of the points (radix sort of
// (descending z, index) keys) -> per point, the windows that hold it, emitted in z order ->
// stable radix sort of the (window, z rank) pairs by window -> runs + sentinels -> records.
#pragma clang fp contract(off)

#include <cfloat>
#include <cmath>

#include <rocprim/device/device_radix_sort.hpp>

#include "pcp_grid.hpp"
#include "pcp_internal.hpp"

namespace pcp {

namespace {

constexpr int kThreads = 256;

struct FineGeo {
    double ox, oy;        // grid origin (x, y)
    double cf, inv_cf;    // fine cell edge and its inverse
    double R2;            // (r + m)^2
    int32_t fnx, fny;     // fine cells per axis (= windows per axis)
    int32_t reach;        // ceil(R / c_f): windows within this many cells can hold a point
};

// p's xy distance to window (wx, wy)'s rectangle is <= R (double arithmetic, the same in every
// kernel, so counts and emissions agree)
__device__ __forceinline__ bool in_window(const FineGeo &f, double px, double py, int wx, int wy) {
    const double x0 = f.ox + (double)wx * f.cf, y0 = f.oy + (double)wy * f.cf;
    const double dx = fmax(fmax(x0 - px, px - (x0 + f.cf)), 0.0);
    const double dy = fmax(fmax(y0 - py, py - (y0 + f.cf)), 0.0);
    return dx * dx + dy * dy <= f.R2;
}

__device__ __forceinline__ void fine_cell(const FineGeo &f, float x, float y, int &cx, int &cy) {
    cx = min(max((int)floor(((double)x - f.ox) * f.inv_cf), 0), f.fnx - 1);
    cy = min(max((int)floor(((double)y - f.oy) * f.inv_cf), 0), f.fny - 1);
}

// (descending z, ascending original index) as one ascending 64-bit key
__global__ void __launch_bounds__(kThreads)
k_zkeys(const float4 *__restrict__ pts, uint32_t n, unsigned long long *__restrict__ key,
        uint32_t *__restrict__ val) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[i];
    uint32_t u = __float_as_uint(p.z);
    u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);   // ascending in z
    key[i] = ((unsigned long long)(~u) << 32) | __float_as_uint(p.w);
    val[i] = i;
}

// windows holding each point (in z order): count per point
__global__ void __launch_bounds__(kThreads)
k_win_count(const float4 *__restrict__ pts, const uint32_t *__restrict__ zord, uint32_t n,
            FineGeo f, uint32_t *__restrict__ pcount) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[zord[i]];
    int cx, cy;
    fine_cell(f, p.x, p.y, cx, cy);
    uint32_t c = 0;
    for (int wy = max(cy - f.reach, 0); wy <= min(cy + f.reach, f.fny - 1); ++wy)
        for (int wx = max(cx - f.reach, 0); wx <= min(cx + f.reach, f.fnx - 1); ++wx)
            if (in_window(f, (double)p.x, (double)p.y, wx, wy)) ++c;
    pcount[i] = c;
}

__global__ void __launch_bounds__(kThreads)
k_win_emit(const float4 *__restrict__ pts, const uint32_t *__restrict__ zord, uint32_t n,
           FineGeo f, const uint32_t *__restrict__ poff, uint32_t *__restrict__ wkey,
           uint32_t *__restrict__ rank) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = pts[zord[i]];
    int cx, cy;
    fine_cell(f, p.x, p.y, cx, cy);
    uint32_t o = poff[i];
    for (int wy = max(cy - f.reach, 0); wy <= min(cy + f.reach, f.fny - 1); ++wy)
        for (int wx = max(cx - f.reach, 0); wx <= min(cx + f.reach, f.fnx - 1); ++wx)
            if (in_window(f, (double)p.x, (double)p.y, wx, wy)) {
                wkey[o] = (uint32_t)wx + (uint32_t)f.fnx * (uint32_t)wy;
                rank[o] = i;
                ++o;
            }
}

// cstart[w] = first sorted pair of window w (lower bound in the sorted window keys), w <= nw
__global__ void __launch_bounds__(kThreads)
k_win_bounds(const uint32_t *__restrict__ wkey, uint32_t np, uint32_t nw,
             uint32_t *__restrict__ cstart) {
    const uint32_t w = blockIdx.x * kThreads + threadIdx.x;
    if (w > nw) return;
    uint32_t lo = 0, hi = np;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (wkey[mid] < w) lo = mid + 1;
        else hi = mid;
    }
    cstart[w] = lo;
}

// sorted pair k of window W lands at k + W (one sentinel ends each earlier window)
__global__ void __launch_bounds__(kThreads)
k_win_place(const float4 *__restrict__ pts, const uint32_t *__restrict__ zord,
            const uint32_t *__restrict__ wkey, const uint32_t *__restrict__ rank, uint32_t np,
            float4 *__restrict__ wpts) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= np) return;
    wpts[k + wkey[k]] = pts[zord[rank[k]]];
}

// records of one window, one thread per window: for coarse z corner iz, the window's points in
// coarse z cells iz, iz + 1 start at the first point with cz <= iz + 1 of the z-descending run
// (cz is non-increasing along it); no end is stored (see the header).  The z band is stored as
// probe thresholds in steps of kZq cells above the block floor: lo - T, hi + T with
// T = ceil((r + 2 mm) / c / kZq) folded in (0 / 255 unbounded; empty: lo 255, hi 0), so the
// probe is two compares.  (One thread per record with two binary searches each
// measured 1.7x slower: 17 levels re-search the same short run.)
__global__ void __launch_bounds__(kThreads)
k_frec(float4 *__restrict__ wpts, const uint32_t *__restrict__ cstart, CellMap m, double c,
       uint32_t fnx, uint32_t fny, uint32_t rz, uint32_t tsteps, int tile,
       int skip2, uint2 *__restrict__ frec, uint16_t *__restrict__ fband,
       uint32_t *__restrict__ fstart) {
    const uint32_t nw = fnx * fny, w = blockIdx.x * kThreads + threadIdx.x;
    // tiles of T x T records: 4 x 4 8-byte records (tile 1) or 8 x 8 split records (tile 2),
    // 128 bytes of probe data each
    const uint32_t sh = tile == 2 ? 3u : 2u, T = 1u << sh, TS = T * T;
    const uint32_t tx = (fnx + T - 1) >> sh, ty = (fny + T - 1) >> sh;
    const size_t plane = tile ? (size_t)tx * ty * TS : (size_t)nw;
    auto put = [&](size_t r, uint32_t start, uint32_t band) {
        if (tile == 2) {
            fband[r] = (uint16_t)band;
            fstart[r] = start;
        } else {
            frec[r] = make_uint2(start, band);
        }
    };
    if (tile && w < tx * ty * TS) {   // padding records of the tiles (never windows)
        const uint32_t t = w >> (2 * sh), sub = w & (TS - 1);
        const uint32_t px = (t % tx) * T + (sub & (T - 1)), py = (t / tx) * T + (sub >> sh);
        if (px >= fnx || py >= fny)
            for (uint32_t iz = 0; iz < rz; ++iz) put((size_t)iz * plane + w, 0u, 0x00FFu);
    }
    if (w >= nw) return;
    // record index of (w, iz): x-fastest, or T x T xy tiles
    const uint32_t wx = w % fnx, wy = w / fnx;
    const size_t base = tile ? ((size_t)((wy >> sh) * tx + (wx >> sh)) << (2 * sh)) |
                                   ((wy & (T - 1)) << sh) | (wx & (T - 1))
                             : (size_t)w;
    const uint32_t s = cstart[w] + w, e = cstart[w + 1] + w;   // e: the sentinel
    wpts[e] = make_float4(__int_as_float(0x7FC00000), __int_as_float(0x7FC00000), -INFINITY,
                          __uint_as_float(0xFFFFFFFFu));
    // one pass down the run: jt / jb advance monotonically, each entry's z and coarse z cell
    // loaded once per pointer (the walk of every level reuses them)
    uint32_t jt = s, jb = s, j2 = s, j3 = s;
    float zt = wpts[s].z, zb = zt, zlast = zt, z2 = zt, z3 = zt;
    int ct = s < e ? cell_z(m, zt) : -1, cb = ct;
    for (int iz = (int)rz - 1; iz >= 0; --iz) {
        while (jt < e && ct > iz + 1) {
            ++jt;
            zt = wpts[jt].z;
            ct = jt < e ? cell_z(m, zt) : -1;
        }
        if (jb < jt) {
            jb = jt;
            zb = zt;
            cb = ct;
        }
        while (jb < e && cb >= iz) {
            zlast = zb;
            ++jb;
            zb = wpts[jb].z;
            cb = jb < e ? cell_z(m, zb) : -1;
        }
        uint32_t band = 0x00FFu;   // empty
        if (jb > jt) {
            const uint32_t code = zband_code(zt, zlast, m.oz + (double)iz * c, c);
            const uint32_t lo = code & 255u, hi = code >> 8;
            const uint32_t lo2 = (lo == 0u || lo <= tsteps) ? 0u : lo - tsteps;
            const uint32_t hi2 = (hi == 255u) ? 255u : min(hi + tsteps, 255u);
            band = lo2 | (hi2 << 8);
        }
        // split records: the entries from jt that lie at or above oz + (iz + 1.5) c (at most
        // 15 of them) can be skipped by a query more than r below that height (march, FN 8).
        // skip2: two thresholds, iz + 1.375 and iz + 1.6875 (exact in float), at most 15 and 7
        // entries, with a 25-bit start (build_fine: below 2^25 entries)
        uint32_t word = jt;
        if (tile == 2) {
            if (j2 < jt) {
                j2 = jt;
                z2 = zt;
            }
            const double h2 = m.oz + ((double)iz + (skip2 ? 1.375 : 1.5)) * c;
            while (j2 < e && (double)z2 >= h2) z2 = wpts[++j2].z;
            if (skip2) {
                if (j3 < jt) {
                    j3 = jt;
                    z3 = zt;
                }
                const double h3 = m.oz + ((double)iz + 1.6875) * c;
                while (j3 < e && (double)z3 >= h3) z3 = wpts[++j3].z;
                word = jt | (min(j2 - jt, 15u) << 25) | (min(j3 - jt, 7u) << 29);
            } else {
                word = jt | (min(j2 - jt, 15u) << 28);
            }
        }
        put((size_t)iz * plane + base, word, band);
    }
}

// the fine-window entries packed to 12 bytes (x, y, z): a quarter less working set for the walks
__global__ void __launch_bounds__(kThreads)
k_pack3(const float4 *__restrict__ src, uint32_t n, float *__restrict__ dst) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = src[i];
    dst[3 * (size_t)i] = p.x;
    dst[3 * (size_t)i + 1] = p.y;
    dst[3 * (size_t)i + 2] = p.z;
}

}  // namespace

int build_fine(pcp_ctx *ctx, GridIndex &g) {
    if (g.fine_ok || g.fine_fail || !g.present || !g.occz_ok || g.n_pts == 0) return PCP_OK;
    hipStream_t st = ctx->stream;
    ProfScope prof(ctx, PCP_K_INDEX_BUILD);
    const GridView gv = g.view();
    const CellMap m{gv.ox, gv.oy, gv.oz, gv.inv_c, g.nx, g.ny, g.nz};
    const int F = std::max(2, std::min(ctx->terrain_fine, 8));
    const uint64_t fnx = (uint64_t)F * g.nx, fny = (uint64_t)F * g.ny;
    const uint64_t rz = (uint64_t)(g.nz > 1 ? g.nz - 1 : 0);
    // caps: 32-bit record byte offsets (< 2^29 records), 24-bit probe multiplies, window keys
    const int tile = ctx->fine_tile == 2 ? 2 : ctx->fine_tile ? 1 : 0;
    const uint64_t T = tile == 2 ? 8 : 4;
    const uint64_t nrec = tile ? ((fnx + T - 1) / T) * ((fny + T - 1) / T) * T * T * rz
                               : fnx * fny * rz;
    const uint64_t nw = fnx * fny;   // windows (the runs)
    const size_t band_bytes = ((size_t)nrec * 2 + 255) & ~(size_t)255;
    const size_t rec_bytes = tile == 2 ? band_bytes + (size_t)nrec * 4 : (size_t)nrec * sizeof(uint2);
    if (rz == 0 || nrec >= (1ull << 29) || fnx >= (1ull << 24) || fny * rz >= (1ull << 24)) {
        g.fine_fail = true;
        return PCP_OK;
    }
    FineGeo f{};
    f.ox = gv.ox;
    f.oy = gv.oy;
    f.cf = g.c / F;
    f.inv_cf = F * gv.inv_c;
    const double R = g.r_q + kQueryMargin;
    f.R2 = R * R;
    f.fnx = (int32_t)fnx;
    f.fny = (int32_t)fny;
    f.reach = (int32_t)std::ceil(R / f.cf);
    const uint32_t n = (uint32_t)g.n_pts;
    const unsigned gridn = (n + kThreads - 1) / kThreads;
    const float4 *pts = g.pts.as<const float4>();
    // 1. global z order
    size_t t1 = 0, t2 = 0;
    // rocPRIM's onesweep radix sort, called directly (no CUB-compatibility layer)
    (void)rocprim::radix_sort_pairs(nullptr, t1, (unsigned long long *)nullptr,
                                    (unsigned long long *)nullptr, (uint32_t *)nullptr,
                                    (uint32_t *)nullptr, n, 0u, 64u, st);
    PCP_HIP(ctx, ctx->scratch[2].ensure((size_t)n * 24 + 64));   // keys x2, vals x2
    unsigned long long *k0 = ctx->scratch[2].as<unsigned long long>(), *k1 = k0 + n;
    uint32_t *v0 = reinterpret_cast<uint32_t *>(k1 + n), *zord = v0 + n;
    hipLaunchKernelGGL(k_zkeys, dim3(gridn), dim3(kThreads), 0, st, pts, n, k0, v0);
    PCP_CHECK_LAUNCH(ctx);
    // 2. windows per point (pcount); points per window come from the sorted pairs (step 4)
    PCP_HIP(ctx, ctx->scratch[3].ensure((size_t)(n + 1) * 8 + (nw + 1) * 4 + 64));
    uint32_t *pcount = ctx->scratch[3].as<uint32_t>(), *poff = pcount + (n + 1);
    uint32_t *cstart = poff + (n + 1);
    // 3. scans
    const size_t tscan = scan_tmp_bytes(std::max<uint64_t>(n, nw)) +
                         (std::max<uint64_t>(n, nw) + 1) * sizeof(uint32_t);
    PCP_HIP(ctx, ctx->scratch[4].ensure(std::max(t1, tscan) + 256));
    if (rocprim::radix_sort_pairs(ctx->scratch[4].p, t1, k0, k1, v0, zord, n, 0u, 64u, st) !=
        hipSuccess)
        return set_err(ctx, PCP_E_HIP, "build_fine: z sort failed");
    hipLaunchKernelGGL(k_win_count, dim3(gridn), dim3(kThreads), 0, st, pts, zord, n, f, pcount);
    PCP_CHECK_LAUNCH(ctx);
    int rc = exclusive_scan_u32(ctx, pcount, poff, n, ctx->scratch[4].p);
    if (rc) return rc;
    uint32_t np = 0;
    if ((rc = read_small(ctx, &np, poff + n, 4, st))) return rc;
    // entries = pairs + one sentinel per window, addressed with 32-bit indices (<< 4 bytes)
    if (np == 0 || (uint64_t)np + nw >= (1ull << 28)) {
        g.fine_fail = true;
        return PCP_OK;
    }
    // 4. pairs (window, z rank), stable sort by window
    int wbits = 1;
    while ((1ull << wbits) < nw) ++wbits;
    (void)rocprim::radix_sort_pairs(nullptr, t2, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                    (uint32_t *)nullptr, (uint32_t *)nullptr, np, 0u,
                                    (unsigned)wbits, st);
    PCP_HIP(ctx, ctx->scratch[5].ensure((size_t)np * 16 + 64));
    uint32_t *wk0 = ctx->scratch[5].as<uint32_t>(), *wk1 = wk0 + np, *rk0 = wk1 + np,
             *rk1 = rk0 + np;
    PCP_HIP(ctx, ctx->scratch[6].ensure(t2 + 256));
    hipLaunchKernelGGL(k_win_emit, dim3(gridn), dim3(kThreads), 0, st, pts, zord, n, f,
                       (const uint32_t *)poff, wk0, rk0);
    PCP_CHECK_LAUNCH(ctx);
    if (rocprim::radix_sort_pairs(ctx->scratch[6].p, t2, wk0, wk1, rk0, rk1, np, 0u,
                                  (unsigned)wbits, st) != hipSuccess)
        return set_err(ctx, PCP_E_HIP, "build_fine: window sort failed");
    hipLaunchKernelGGL(k_win_bounds, dim3((unsigned)((nw + kThreads) / kThreads)), dim3(kThreads),
                       0, st, (const uint32_t *)wk1, np, (uint32_t)nw, cstart);
    PCP_CHECK_LAUNCH(ctx);
    // the copy is an optional speed-up: an allocation failure keeps the other layouts
    const size_t nent = (size_t)np + nw;
    const bool pack = ctx->fine_pack != 0;
    // packed: the float4 entries are built in scratch, then packed into wpts
    if ((pack && ctx->scratch[7].ensure(nent * sizeof(float4)) != hipSuccess) ||
        g.wpts.ensure(pack ? nent * 12 + 16 : nent * sizeof(float4)) != hipSuccess ||
        g.frec.ensure(rec_bytes) != hipSuccess) {
        (void)hipGetLastError();
        g.wpts.release();
        g.frec.release();
        g.fine_fail = true;
        return PCP_OK;
    }
    float4 *went = pack ? ctx->scratch[7].as<float4>() : g.wpts.as<float4>();
    hipLaunchKernelGGL(k_win_place, dim3((np + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                       pts, (const uint32_t *)zord, (const uint32_t *)wk1, (const uint32_t *)rk1,
                       np, went);
    PCP_CHECK_LAUNCH(ctx);
    // 5. records (and the sentinels), one thread per window; two skip thresholds need a 25-bit
    // walk start
    const bool skip2 = tile == 2 && ctx->fine_skip == 2 && nent < (1ull << 25);
    const uint32_t tsteps = (uint32_t)std::ceil((g.r_q + 2e-3) / g.c / (double)kZq);
    const uint64_t nthr = std::max<uint64_t>(nw, tile ? nrec / rz : 0);
    hipLaunchKernelGGL(k_frec, dim3((unsigned)((nthr + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       st, went, (const uint32_t *)cstart, m, g.c, (uint32_t)fnx,
                       (uint32_t)fny, (uint32_t)rz, tsteps, tile, skip2 ? 1 : 0,
                       g.frec.as<uint2>(),
                       g.frec.as<uint16_t>(),
                       reinterpret_cast<uint32_t *>(g.frec.as<char>() + band_bytes));
    PCP_CHECK_LAUNCH(ctx);
    if (pack) {
        hipLaunchKernelGGL(k_pack3, dim3((unsigned)((nent + kThreads - 1) / kThreads)),
                           dim3(kThreads), 0, st, (const float4 *)went, (uint32_t)nent,
                           g.wpts.as<float>());
        PCP_CHECK_LAUNCH(ctx);
    }
    g.wpack = pack ? 1 : 0;
    g.frx = (uint32_t)fnx;
    g.fry = (uint32_t)fny;
    g.frz = (uint32_t)rz;
    g.ffine = (float)F;
    g.ftile = tile;
    g.fskip = skip2 ? 2 : 1;
    g.fstart_off = tile == 2 ? band_bytes : 0;
    g.fine_ok = true;
    return PCP_OK;
}

}  // namespace pcp
