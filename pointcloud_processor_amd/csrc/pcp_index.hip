// pcp_index.hip -- uniform-grid spatial index build (replaces KdTreeFLANN::setInputCloud,
// virtual_lidar.cpp:172,187,201).  Layout in HBM (see DESIGN.md "Terrain index"):
//   pts   : float4[n]   x, y, z, bitcast(original point index), sorted by cell
//   start : u32[ncell+1] prefix offsets (cell c holds pts[start[c] .. start[c+1]) )
//   occ2  : u32[(ncell+31)/32] dilated occupancy (bit c = any point in cells c + {0,1}^3)
//   occz  : u16[ncell] z band of the same 2x2x2 block (z-sorted indices: the march's probe)
//   bstart: u32[ncell+1], bpts: float4[8 n] (terrain): each stencil corner's 2x2x2 block as
//           one run in descending z (every point appears in the blocks of its 8 corners)
#include <cfloat>
#include <cmath>
#include <cstring>

#include "pcp_internal.hpp"
#include "pcp_grid.hpp"

namespace pcp {

constexpr uint64_t kMaxCells = 1ull << 25;
constexpr int kThreads = 256;

GridView GridIndex::view() const {
    GridView v{};
    v.pts = pts.as<const float4>();
    v.start = start.as<const uint32_t>();
    v.occ2 = occ2_ok ? occ2.as<const uint32_t>() : nullptr;
    v.c = c;
    v.inv_c = c > 0 ? 1.0 / c : 0.0;
    v.ox = bmin[0] - c;   // one padding cell below the points
    v.oy = bmin[1] - c;
    v.oz = bmin[2] - c;
    const double rm = r_q + kQueryMargin;
    // the clip box also absorbs the float rounding of a sample position near the points
    double amax = 0.0;
    for (int a = 0; a < 3; ++a) amax = fmax(amax, fmax(fabs(bmin[a]), fabs(bmax[a])));
    const double rb = rm + 1e-6 * amax;
    v.lo_x = v.ox + rm;
    v.lo_y = v.oy + rm;
    v.lo_z = v.oz + rm;
    v.nx = nx;
    v.ny = ny;
    v.nz = nz;
    v.n_pts = (uint32_t)n_pts;
    v.bx0 = bmin[0] - rb;
    v.bx1 = bmax[0] + rb;
    v.by0 = bmin[1] - rb;
    v.by1 = bmax[1] + rb;
    v.bz0 = bmin[2] - rb;
    v.bz1 = bmax[2] + rb;
    v.flo_x = (float)v.lo_x;
    v.flo_y = (float)v.lo_y;
    v.flo_z = (float)v.lo_z;
    v.finv_c = (float)v.inv_c;
    v.fnx1 = (float)(nx - 1);
    v.fny1 = (float)(ny - 1);
    v.fnz1 = (float)(nz - 1);
    const double bb[6] = {v.bx0, v.bx1, v.by0, v.by1, v.bz0, v.bz1};
    for (int a = 0; a < 6; ++a) v.fb[a] = (float)bb[a];
    v.occz = occz_ok ? occz.as<const uint16_t>() : nullptr;
    v.bstart = blk_ok ? bstart.as<const uint32_t>() : nullptr;
    v.bpts = blk_ok ? bpts.as<const float4>() : nullptr;
    v.fzoff = (float)(rm * v.inv_c);
    v.fzt = (float)((r_q + 2e-3) * v.inv_c);
    v.frec = fine_ok ? frec.as<const uint2>() : nullptr;
    v.wpts = fine_ok ? wpts.as<const float4>() : nullptr;
    v.frx = fine_ok ? frx : 0u;
    v.fry = fine_ok ? fry : 0u;
    v.frz = fine_ok ? frz : 0u;
    v.ffine = fine_ok ? ffine : 0.0f;
    v.ftile = fine_ok ? ftile : 0;
    v.fband = (fine_ok && ftile == 2) ? frec.as<const uint16_t>() : nullptr;
    v.fzc = (float)c;
    v.wpack = fine_ok ? wpack : 0;
    v.fzo = (float)v.oz;
    v.fstart = (fine_ok && ftile == 2)
                   ? reinterpret_cast<const uint32_t *>(frec.as<const char>() + fstart_off)
                   : nullptr;
    v.fus_off = (float)(rm * v.inv_c / (double)kZq);
    v.fskip = fine_ok ? fskip : 1;
    return v;
}

float exit_dist(float r2) {
    float d = std::sqrt(r2);
    while (d * d < r2) d = std::nextafter(d, INFINITY);
    for (float p = std::nextafter(d, 0.0f); p * p >= r2; p = std::nextafter(d, 0.0f)) d = p;
    return d;
}

__device__ __forceinline__ float ld_f32(const unsigned char *base, uint32_t off) {
    return *reinterpret_cast<const float *>(base + off);
}

// extract x,y,z (4-byte aligned FLOAT32 fields) to float4 + per-block bbox of finite pts
__global__ void __launch_bounds__(kThreads)
k_extract(const unsigned char *__restrict__ raw, uint64_t n, uint32_t step, uint32_t ox,
          uint32_t oy, uint32_t oz, float4 *__restrict__ xyz, float *__restrict__ part,
          uint32_t *__restrict__ part_n, uint32_t *__restrict__ zero_p, uint64_t zero_n) {
    // the cell counters of the build, zeroed here instead of by a separate fill launch
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < zero_n;
         i += (uint64_t)gridDim.x * kThreads)
        zero_p[i] = 0;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    uint32_t cnt = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * kThreads) {
        const unsigned char *p = raw + i * step;
        const float x = ld_f32(p, ox), y = ld_f32(p, oy), z = ld_f32(p, oz);
        const bool fin = isfinite(x) && isfinite(y) && isfinite(z);
        xyz[i] = make_float4(x, y, z, __uint_as_float(fin ? (uint32_t)i : 0xFFFFFFFFu));
        if (fin) {
            ++cnt;
            mn[0] = fminf(mn[0], x); mx[0] = fmaxf(mx[0], x);
            mn[1] = fminf(mn[1], y); mx[1] = fmaxf(mx[1], y);
            mn[2] = fminf(mn[2], z); mx[2] = fmaxf(mx[2], z);
        }
    }
    // wave reduce then block reduce through LDS
    __shared__ float s[6][kThreads / 64];
    __shared__ uint32_t sc[kThreads / 64];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
            mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
        }
        cnt += __shfl_xor(cnt, o, 64);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        for (int a = 0; a < 3; ++a) { s[a][w] = mn[a]; s[3 + a][w] = mx[a]; }
        sc[w] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int ww = 1; ww < kThreads / 64; ++ww) {
            for (int a = 0; a < 3; ++a) {
                s[a][0] = fminf(s[a][0], s[a][ww]);
                s[3 + a][0] = fmaxf(s[3 + a][0], s[3 + a][ww]);
            }
            sc[0] += sc[ww];
        }
        for (int a = 0; a < 6; ++a) part[blockIdx.x * 6 + a] = s[a][0];
        part_n[blockIdx.x] = sc[0];
    }
}

// order-free reduction of the k_extract partials (min / max / count), one block
__global__ void __launch_bounds__(kThreads)
k_bbox_final(const float *__restrict__ part, const uint32_t *__restrict__ part_n, int nb,
             float *__restrict__ out, uint32_t *__restrict__ out_n) {
    float r[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    uint32_t c = 0;
    for (int b = threadIdx.x; b < nb; b += kThreads) {
        for (int a = 0; a < 3; ++a) {
            r[a] = fminf(r[a], part[b * 6 + a]);
            r[3 + a] = fmaxf(r[3 + a], part[b * 6 + 3 + a]);
        }
        c += part_n[b];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            r[a] = fminf(r[a], __shfl_xor(r[a], o, 64));
            r[3 + a] = fmaxf(r[3 + a], __shfl_xor(r[3 + a], o, 64));
        }
        c += __shfl_xor(c, o, 64);
    }
    __shared__ float s[6][kThreads / 64];
    __shared__ uint32_t sc[kThreads / 64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) {
        for (int a = 0; a < 6; ++a) s[a][w] = r[a];
        sc[w] = c;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int ww = 1; ww < kThreads / 64; ++ww) {
        for (int a = 0; a < 3; ++a) {
            s[a][0] = fminf(s[a][0], s[a][ww]);
            s[3 + a][0] = fmaxf(s[3 + a][0], s[3 + a][ww]);
        }
        sc[0] += sc[ww];
    }
    for (int a = 0; a < 6; ++a) out[a] = s[a][0];
    *out_n = sc[0];
}

// the active lanes of the wave holding the same 32-bit key as this lane.  Big cells (the 1.5 m
// normal index is a 3 m grid) put many points of a wave into one cell, where per-lane atomics on
// one counter serialize; one atomic per group of equal keys avoids that.
__device__ __forceinline__ uint64_t peer_mask(uint32_t key) {
    uint64_t same = __ballot(1);
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        const bool bit = (key >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        same &= bit ? bb : ~bb;
    }
    return same;
}

// a point's cell and its slot in the cell: the count's atomic hands out the slots (one atomic
// per group of lanes sharing the cell; the order inside a cell is free: z-sorted indices
// re-rank by (z, index), the others are queried order-free)
__device__ __forceinline__ void count_ranked(const CellMap &m, float x, float y, float z,
                                             bool fin, uint32_t *__restrict__ count, uint2 &cr) {
    const uint32_t c = fin ? cell_of(m, x, y, z) : 0xFFFFFFFFu;
    const uint64_t peers = peer_mask(c);
    const int lane = threadIdx.x & 63, leader = __ffsll((long long)peers) - 1;
    uint32_t base = 0;
    if (fin && lane == leader) base = atomicAdd(&count[c], (uint32_t)__popcll(peers));
    base = __shfl(base, leader, 64);
    cr = make_uint2(c, base + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull)));
}

// message-sized clouds (grid geometry from the host's bbox): extraction, cell and slot in one
// pass over the raw records
__global__ void __launch_bounds__(kThreads)
k_extract_count(const unsigned char *__restrict__ raw, uint64_t n, uint32_t step, uint32_t ox,
                uint32_t oy, uint32_t oz, CellMap m, float4 *__restrict__ xyz,
                uint32_t *__restrict__ count, uint2 *__restrict__ cr,
                unsigned char *__restrict__ raw_copy) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;   // (whole waves: the peer masks below see only live lanes)
    const unsigned char *p = raw + i * step;
    if (raw_copy) {   // the record into device memory on the way (step: 16-byte multiple <= 64)
        uint4 r[4];
        const uint32_t nq = step >> 4;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (k < nq) r[k] = reinterpret_cast<const uint4 *>(p)[k];
        unsigned char *d = raw_copy + i * step;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (k < nq) reinterpret_cast<uint4 *>(d)[k] = r[k];
        p = d;   // (this thread's own stores: x, y, z read back from them)
    }
    const float x = ld_f32(p, ox), y = ld_f32(p, oy), z = ld_f32(p, oz);
    const bool fin = isfinite(x) && isfinite(y) && isfinite(z);
    xyz[i] = make_float4(x, y, z, __uint_as_float(fin ? (uint32_t)i : 0xFFFFFFFFu));
    uint2 c;
    count_ranked(m, x, y, z, fin, count, c);
    cr[i] = c;
}

// the same after a device-side bbox (large clouds: k_extract + k_bbox_final first)
__global__ void __launch_bounds__(kThreads)
k_cell_count_ranked(const float4 *__restrict__ xyz, uint64_t n, CellMap m,
                    uint32_t *__restrict__ count, uint2 *__restrict__ cr) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const float4 p = xyz[i];
    const bool fin = __float_as_uint(p.w) != 0xFFFFFFFFu;
    uint2 c;
    count_ranked(m, p.x, p.y, p.z, fin, count, c);
    cr[i] = c;
}

// each point to its cell's start + its slot: no cursors, no atomics
__global__ void __launch_bounds__(kThreads)
k_cell_place(const float4 *__restrict__ xyz, uint64_t n, const uint2 *__restrict__ cr,
             const uint32_t *__restrict__ start, float4 *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint2 c = cr[i];
    if (c.x == 0xFFFFFFFFu) return;
    out[start[c.x] + c.y] = xyz[i];
}

// points of each cell in descending z: lets a query stop scanning a cell at the first point
// that is more than r below it (exact early exit, see scan_stencil).  One thread per point:
// position = cell start + the cell's points ahead of it (higher z, or equal z and earlier), so
// a cell of n points costs n^2 compares spread over n threads -- the 3 m cells of a 1.5 m
// radius index hold thousands of points (a per-cell insertion sort took 250 ms there).
__global__ void __launch_bounds__(kThreads)
k_cell_rank_z(const float4 *__restrict__ in, uint64_t n, CellMap m,
              const uint32_t *__restrict__ start, float4 *__restrict__ out) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const float4 p = in[k];
    const uint32_t c = cell_of(m, p.x, p.y, p.z);
    const uint32_t s = start[c], e = start[c + 1];
    // descending z, ties by original index (.w): the layout does not depend on the order
    // in which the scatter's atomics placed the points
    const uint32_t ok = __float_as_uint(p.w);
    uint32_t rank = 0;
    for (uint32_t j = s; j < e; ++j) {
        const float4 q = in[j];
        rank += (q.z > p.z || (q.z == p.z && __float_as_uint(q.w) < ok)) ? 1u : 0u;
    }
    out[s + rank] = p;
}

// z band per stencil corner (z-sorted cells: a cell's first point is its highest, its last
// the lowest).  Rounded outwards by one extra step and clamped to the open-ended codes, so
// zb + lo*kZq*c <= every point z <= zb + hi*kZq*c holds for the block's points whatever the
// rounding of their cell assignment (zb = the block's floor, oz + iz*c).
__device__ __forceinline__ uint16_t occz_at(const uint32_t *__restrict__ start,
                                            const float4 *__restrict__ pts, const CellMap &m,
                                            double c, int ix, int iy, int iz) {
    float zmax = -FLT_MAX, zmin = FLT_MAX;
    bool any = false;
    for (int dz = 0; dz < 2; ++dz)
        for (int dy = 0; dy < 2; ++dy) {
            const int y = iy + dy, z = iz + dz;
            if (y >= m.ny || z >= m.nz) continue;
            const uint64_t row = (uint64_t)m.nx * ((uint64_t)y + (uint64_t)m.ny * z);
            for (int dx = 0; dx < 2 && ix + dx < m.nx; ++dx) {
                const uint32_t s = start[row + ix + dx], e = start[row + ix + dx + 1];
                if (s < e) {
                    any = true;
                    zmax = fmaxf(zmax, pts[s].z);
                    zmin = fminf(zmin, pts[e - 1].z);
                }
            }
        }
    return any ? zband_code(zmax, zmin, m.oz + (double)iz * c, c) : (uint16_t)0x00FFu;
}

__global__ void __launch_bounds__(kThreads)
k_occz(const uint32_t *__restrict__ start, const float4 *__restrict__ pts, CellMap m, double c,
       uint64_t ncell, uint16_t *__restrict__ occz) {
    const uint64_t lin = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (lin >= ncell) return;
    const int ix = (int)(lin % m.nx);
    const int iy = (int)((lin / m.nx) % m.ny);
    const int iz = (int)(lin / ((uint64_t)m.nx * m.ny));
    occz[lin] = occz_at(start, pts, m, c, ix, iy, iz);
}

// the same bands for a sparse grid (far more cells than points; the array preset to the empty
// code 0x00FF): the first point of each occupied cell writes the bands of the 8 corners whose
// 2x2x2 block holds that cell -- every corner with a point in its block, and no other, differs
// from the preset.  A corner shared by several occupied cells gets the same value from each.
__global__ void __launch_bounds__(kThreads)
k_occz_sparse(const uint32_t *__restrict__ start, const float4 *__restrict__ pts, CellMap m,
              double c, uint64_t npts, uint16_t *__restrict__ occz) {
    // thread = (point, corner): the corners of one cell are independent (one occz_at each, no
    // chain of eight)
    const uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    const uint64_t j = t >> 3;
    const int d = (int)(t & 7);
    if (j >= npts) return;
    const float4 p = pts[j];
    const uint32_t cc = cell_of(m, p.x, p.y, p.z);
    if (start[cc] != (uint32_t)j) return;
    const int ix = (int)(cc % (uint32_t)m.nx);
    const int iy = (int)((cc / (uint32_t)m.nx) % (uint32_t)m.ny);
    const int iz = (int)(cc / ((uint32_t)m.nx * (uint32_t)m.ny));
    const int tx = ix - (d & 1), ty = iy - ((d >> 1) & 1), tz = iz - (d >> 2);
    if (tx < 0 || ty < 0 || tz < 0) return;
    const uint64_t lin = (uint64_t)tx + (uint64_t)m.nx * ((uint64_t)ty + (uint64_t)m.ny * tz);
    occz[lin] = occz_at(start, pts, m, c, tx, ty, tz);
}

// dilated occupancy: bit for lower corner (ix,iy,iz) = any point in the 2x2x2 block
__global__ void __launch_bounds__(kThreads)
k_occ2(const uint32_t *__restrict__ start, CellMap m, uint64_t ncell, uint32_t *__restrict__ occ2) {
    // one thread per cell (its 4 block rows are independent loads), a wave's 64 bits by ballot
    const uint64_t c = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    bool any = false;
    if (c < ncell) {
        const int ix = (int)(c % m.nx);
        const int iy = (int)((c / m.nx) % m.ny);
        const int iz = (int)(c / ((uint64_t)m.nx * m.ny));
        const int x1 = min(ix + 2, m.nx);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int y = iy + (r & 1), z = iz + (r >> 1);
            if (y < m.ny && z < m.nz) {
                const uint64_t row = (uint64_t)m.nx * ((uint64_t)y + (uint64_t)m.ny * z);
                any |= start[row + x1] > start[row + ix];
            }
        }
    }
    const uint64_t bits = __ballot(any);
    const uint64_t w = c >> 5;   // the wave's first word (64-cell aligned)
    const uint64_t nw = (ncell + 31) / 32;
    if ((threadIdx.x & 63) == 0 && w < nw) occ2[w] = (uint32_t)bits;
    if ((threadIdx.x & 63) == 0 && w + 1 < nw) occ2[w + 1] = (uint32_t)(bits >> 32);
}

// points per stencil corner's 2x2x2 block (0 for corners on the upper border: stencil_cell
// never returns them)
__global__ void __launch_bounds__(kThreads)
k_blk_count(const uint32_t *__restrict__ start, CellMap m, uint64_t ncell,
            uint32_t *__restrict__ cnt) {
    const uint64_t lin = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (lin >= ncell) return;
    const int ix = (int)(lin % m.nx);
    const int iy = (int)((lin / m.nx) % m.ny);
    const int iz = (int)(lin / ((uint64_t)m.nx * m.ny));
    uint32_t n = 0;
    if (ix < m.nx - 1 && iy < m.ny - 1 && iz < m.nz - 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint64_t row = lin + (uint64_t)(r & 1) * m.nx + (uint64_t)(r >> 1) * m.nx * m.ny;
            n += start[row + 2] - start[row];
        }
    }
    cnt[lin] = n;
}

// (z descending, original index ascending) -- the order of k_cell_rank_z, as one comparison
__device__ __forceinline__ bool zbefore(float az, uint32_t ai, float bz, uint32_t bi) {
    return az > bz || (az == bz && ai < bi);
}

// block-major fill, one thread per point p of cell C (cells already z-sorted): p's place in
// corner K's block is the number of block points ahead of it = the sum over K's 8 cells D of
// rank_D(p) (points of D ahead of p; its own position for D = C).  The 27 cells around C cover
// the blocks of all 8 corners that contain C; their ranks are counted once and summed per corner.
// Consecutive threads are consecutive points of one cell, so a wave reads the same neighbour
// runs (shared lines).
__global__ void __launch_bounds__(kThreads)
k_blk_fill(const float4 *__restrict__ pts, uint64_t n, const uint32_t *__restrict__ start,
           CellMap m, const uint32_t *__restrict__ bstart, float4 *__restrict__ bpts) {
    const uint64_t k = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const float4 p = pts[k];
    const uint32_t pi = __float_as_uint(p.w);
    const uint32_t c = cell_of(m, p.x, p.y, p.z);
    const int nx = m.nx, ny = m.ny, nz = m.nz;
    const int ix = (int)(c % (uint32_t)nx);
    const int iy = (int)((c / (uint32_t)nx) % (uint32_t)ny);
    const int iz = (int)(c / ((uint32_t)nx * (uint32_t)ny));
    const uint32_t nxy = (uint32_t)nx * (uint32_t)ny;
    uint32_t rk[27];   // rank of p in cell C + (dx, dy, dz), index (dz+1)*9 + (dy+1)*3 + (dx+1)
#pragma unroll
    for (int t = 0; t < 27; ++t) {
        const int dx = t % 3 - 1, dy = (t / 3) % 3 - 1, dz = t / 9 - 1;
        uint32_t r = 0;
        if (dx == 0 && dy == 0 && dz == 0) {
            r = (uint32_t)k - start[c];
        } else if (ix + dx >= 0 && ix + dx < nx && iy + dy >= 0 && iy + dy < ny && iz + dz >= 0 &&
                   iz + dz < nz) {
            const uint32_t d = (uint32_t)((int)c + dx + dy * nx + dz * (int)nxy);
            const uint32_t s = start[d], e = start[d + 1];
            // descending z: the points ahead of p form a prefix of the run
            for (uint32_t j = s; j < e; ++j) {
                const float4 q = pts[j];
                if (!zbefore(q.z, __float_as_uint(q.w), p.z, pi)) break;
                ++r;
            }
        }
        rk[t] = r;
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) {   // corner K = C - (ax, ay, az)
        const int ax = a & 1, ay = (a >> 1) & 1, az = a >> 2;
        const int kx = ix - ax, ky = iy - ay, kz = iz - az;
        if (kx < 0 || ky < 0 || kz < 0 || kx >= nx - 1 || ky >= ny - 1 || kz >= nz - 1) continue;
        uint32_t pos = 0;
#pragma unroll
        for (int b = 0; b < 8; ++b) {   // the block's cells K + (bx, by, bz) = C + (b - a)
            const int dx = (b & 1) - ax, dy = ((b >> 1) & 1) - ay, dz = (b >> 2) - az;
            pos += rk[(dz + 1) * 9 + (dy + 1) * 3 + (dx + 1)];
        }
        const uint32_t K = c - (uint32_t)ax - (uint32_t)ay * (uint32_t)nx - (uint32_t)az * nxy;
        bpts[bstart[K] + pos] = p;
    }
}

// z bands of grids with more than this many cells per point: only around the occupied cells
constexpr uint64_t kSparseCells = 32;

// clouds up to this size get their bbox from the host (build_index)
constexpr uint64_t kHostBboxMax = 1ull << 17;

// min / max of the finite points and their count, as k_extract + k_bbox_final compute them.
// Records with x, y, z adjacent and 16 readable bytes from x (the 16- and 32-byte PointXYZ /
// PointXYZRGB layouts): one 4-wide load per point, four points' min / max chains in flight
// (~3x the scalar loop; every C5 frame takes four of these on the host between launches).  Only
// finite points enter, so the vector min / max equal fmin / fmax (a +-0 tie can pick the other
// zero, which no grid geometry below can see: bmin - c, bmax - bmin are the same either way)
typedef float HostF4 __attribute__((ext_vector_type(4)));
typedef int HostI4 __attribute__((ext_vector_type(4)));
static void host_bbox(const pcp_cloud_view &v, float bb[10], uint32_t &nfin) {
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    uint32_t c = 0;
    const unsigned char *raw = static_cast<const unsigned char *>(v.data);
    uint64_t i0 = 0;
    static const bool vec = !std::getenv("PCP_HOST_BBOX_SCALAR");   // (A/B: the scalar loop)
    if (vec && v.off_y == v.off_x + 4 && v.off_z == v.off_x + 8 &&
        v.off_x + 16 <= v.point_step) {
        constexpr int U = 4;
        HostF4 vmn[U], vmx[U];
        for (int u = 0; u < U; ++u) {
            vmn[u] = HostF4(FLT_MAX);
            vmx[u] = HostF4(-FLT_MAX);
        }
        const unsigned char *px = raw + v.off_x;
        for (; i0 + U <= v.n; i0 += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                HostF4 p;
                memcpy(&p, px + (i0 + u) * v.point_step, 16);
                const HostI4 f = (p - p) == HostF4(0.0f);   // finite lanes
                if (!(f.x & f.y & f.z)) continue;
                ++c;
                vmn[u] = p < vmn[u] ? p : vmn[u];
                vmx[u] = p > vmx[u] ? p : vmx[u];
            }
        }
        for (int u = 0; u < U; ++u)
            for (int a = 0; a < 3; ++a) {
                mn[a] = std::fmin(mn[a], vmn[u][a]);
                mx[a] = std::fmax(mx[a], vmx[u][a]);
            }
    }
    for (uint64_t i = i0; i < v.n; ++i) {
        const unsigned char *p = raw + i * v.point_step;
        float x, y, z;
        memcpy(&x, p + v.off_x, 4);
        memcpy(&y, p + v.off_y, 4);
        memcpy(&z, p + v.off_z, 4);
        if (!(std::isfinite(x) && std::isfinite(y) && std::isfinite(z))) continue;
        ++c;
        mn[0] = std::fmin(mn[0], x); mx[0] = std::fmax(mx[0], x);
        mn[1] = std::fmin(mn[1], y); mx[1] = std::fmax(mx[1], y);
        mn[2] = std::fmin(mn[2], z); mx[2] = std::fmax(mx[2], z);
    }
    for (int a = 0; a < 3; ++a) {
        bb[a] = mn[a];
        bb[3 + a] = mx[a];
    }
    nfin = c;
}

// the grid over a float bbox (bb[0..2] min, bb[3..5] max; g.r_q set): edge c > 2 (r_q +
// margin) so a query box spans <= 2 cells per axis, grown while the grid is too large.
// Returns the cell count
static uint64_t grid_geometry(GridIndex &g, const float bb[6]) {
    for (int a = 0; a < 3; ++a) {
        g.bmin[a] = bb[a];
        g.bmax[a] = bb[3 + a];
    }
    double c = 2.0 * (g.r_q + kCellMargin);
    uint64_t ncell = 0;
    for (;;) {
        int64_t d[3];
        for (int a = 0; a < 3; ++a)
            d[a] = (int64_t)std::floor((g.bmax[a] - (g.bmin[a] - c)) / c) + 2;
        ncell = (uint64_t)d[0] * (uint64_t)d[1] * (uint64_t)d[2];
        if (ncell <= kMaxCells && d[0] < (1 << 30) && d[1] < (1 << 30) && d[2] < (1 << 30)) {
            g.nx = (int32_t)d[0];
            g.ny = (int32_t)d[1];
            g.nz = (int32_t)d[2];
            break;
        }
        c *= 1.25;
    }
    g.c = c;
    return ncell;
}

// two order-free indices of one message-sized cloud (the excavation area's normal-radius and
// lattice-radius grids) from ONE pass over its raw records: extraction, both cells and slots,
// and the caller's per-point preparation (prep_pts: the points by input index as (x, y, z, 0);
// prep_nrm: NaN normals of the non-finite points) -- k_extract_count, k_cell_place and
// k_area_prep of three launches each ... in two
__global__ void __launch_bounds__(kThreads)
k_extract_count2(const unsigned char *__restrict__ raw, uint64_t n, uint32_t step, uint32_t ox,
                 uint32_t oy, uint32_t oz, CellMap ma, CellMap mb, float4 *__restrict__ xyz,
                 uint32_t *__restrict__ cnt_a, uint2 *__restrict__ cr_a,
                 uint32_t *__restrict__ cnt_b, uint2 *__restrict__ cr_b,
                 float4 *__restrict__ prep_pts, float *__restrict__ prep_nrm) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;   // (whole waves: the peer masks below see only live lanes)
    const unsigned char *p = raw + i * step;
    const float x = ld_f32(p, ox), y = ld_f32(p, oy), z = ld_f32(p, oz);
    const bool fin = isfinite(x) && isfinite(y) && isfinite(z);
    xyz[i] = make_float4(x, y, z, __uint_as_float(fin ? (uint32_t)i : 0xFFFFFFFFu));
    uint2 c;
    count_ranked(ma, x, y, z, fin, cnt_a, c);
    cr_a[i] = c;
    count_ranked(mb, x, y, z, fin, cnt_b, c);
    cr_b[i] = c;
    if (prep_pts) {
        prep_pts[i] = make_float4(x, y, z, 0.0f);
        if (!fin) prep_nrm[3 * i] = prep_nrm[3 * i + 1] = prep_nrm[3 * i + 2] = NAN;
    }
}

__global__ void __launch_bounds__(kThreads)
k_cell_place2(const float4 *__restrict__ xyz, uint64_t n, const uint2 *__restrict__ cr_a,
              const uint32_t *__restrict__ start_a, float4 *__restrict__ out_a,
              const uint2 *__restrict__ cr_b, const uint32_t *__restrict__ start_b,
              float4 *__restrict__ out_b) {
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    const uint2 a = cr_a[i], b = cr_b[i];
    if (a.x == 0xFFFFFFFFu) return;   // (non-finite: in neither index)
    const float4 p = xyz[i];
    out_a[start_a[a.x] + a.y] = p;
    out_b[start_b[b.x] + b.y] = p;
}

int build_index_pair(pcp_ctx *ctx, GridIndex &ga, double ra, GridIndex &gb, double rb,
                     const pcp_cloud_view &v, const unsigned char **raw_io, float4 *prep_pts,
                     float *prep_nrm, bool *paired) {
    *paired = false;
    const uint64_t n = v.n;
    if (n == 0 || n > kHostBboxMax || !ctx->index_pair) return PCP_OK;   // (the two builds)
    float bb_h[10];
    uint32_t nfin = 0;
    host_bbox(v, bb_h, nfin);
    if (nfin == 0) return PCP_OK;
    hipStream_t st = ctx->stream;
    ProfScope prof(ctx, PCP_K_INDEX_BUILD);
    for (GridIndex *g : {&ga, &gb}) {
        g->present = false;
        g->occz_ok = g->occ2_ok = g->blk_ok = g->blk_fail = g->fine_ok = g->fine_fail = false;
    }
    // the raw bytes device-readable (as build_index: given, or read in place from the ring)
    const uint64_t raw_bytes = n * (uint64_t)v.point_step;
    const unsigned char *raw = raw_io ? *raw_io : nullptr;
    bool pinned = false;
    if (!raw && ctx->zc_in && raw_bytes <= kPinDirectMax) {
        const HostPiece pc{0, v.data, raw_bytes};
        const void *dv = nullptr;
        if (int rc0 = pin_stage(ctx, &pc, 1, raw_bytes, &dv)) return rc0;
        raw = static_cast<const unsigned char *>(dv);
        pinned = true;
    }
    if (!raw) {
        PCP_HIP(ctx, ctx->stage.ensure(raw_bytes));
        if (int rc0 = upload_async(ctx, ctx->stage.p, v.data, raw_bytes, st)) return rc0;
        raw = ctx->stage.as<unsigned char>();
    }
    if (raw_io) *raw_io = raw;
    ga.r_q = ra;
    gb.r_q = rb;
    ga.n_pts = gb.n_pts = nfin;
    const uint64_t nca = grid_geometry(ga, bb_h), ncb = grid_geometry(gb, bb_h);
    const GridView va = ga.view(), vb = gb.view();
    const CellMap ma{va.ox, va.oy, va.oz, va.inv_c, ga.nx, ga.ny, ga.nz};
    const CellMap mb{vb.ox, vb.oy, vb.oz, vb.inv_c, gb.nx, gb.ny, gb.nz};
    // both grids' counters: zero between builds (each scan clears its own behind it)
    const size_t cba = (nca + 1) * sizeof(uint32_t), cbb = (ncb + 1) * sizeof(uint32_t);
    if (ctx->cell_cnt.cap < cba || ctx->cell_cnt_dirty) {
        PCP_HIP(ctx, ctx->cell_cnt.ensure(cba));
        PCP_HIP(ctx, hipMemsetAsync(ctx->cell_cnt.p, 0, ctx->cell_cnt.cap, st));
        ctx->cell_cnt_dirty = false;
    }
    if (ctx->cell_cnt2.cap < cbb || ctx->cell_cnt2_dirty) {
        PCP_HIP(ctx, ctx->cell_cnt2.ensure(cbb));
        PCP_HIP(ctx, hipMemsetAsync(ctx->cell_cnt2.p, 0, ctx->cell_cnt2.cap, st));
        ctx->cell_cnt2_dirty = false;
    }
    uint32_t *cnt_a = ctx->cell_cnt.as<uint32_t>(), *cnt_b = ctx->cell_cnt2.as<uint32_t>();
    PCP_HIP(ctx, ctx->scratch[0].ensure(n * sizeof(float4)));
    PCP_HIP(ctx, ctx->scratch[2].ensure(2 * n * sizeof(uint2)));
    uint2 *cr_a = ctx->scratch[2].as<uint2>(), *cr_b = cr_a + n;
    const unsigned gridn = (unsigned)((n + kThreads - 1) / kThreads);
    ctx->cell_cnt_dirty = ctx->cell_cnt2_dirty = true;
    hipLaunchKernelGGL(k_extract_count2, dim3(gridn), dim3(kThreads), 0, st, raw, n, v.point_step,
                       v.off_x, v.off_y, v.off_z, ma, mb, ctx->scratch[0].as<float4>(), cnt_a,
                       cr_a, cnt_b, cr_b, prep_pts, prep_nrm);
    PCP_CHECK_LAUNCH(ctx);
    if (pinned && !raw_io) pin_release(ctx, st);
    PCP_HIP(ctx, ga.start.ensure(cba));
    PCP_HIP(ctx, gb.start.ensure(cbb));
    const uint64_t ncm = std::max(nca, ncb);
    PCP_HIP(ctx, ctx->scratch[4].ensure(scan_tmp_bytes(ncm) + (ncm + 1) * sizeof(uint32_t)));
    if (int rc = exclusive_scan_u32_pair(ctx, cnt_a, ga.start.as<uint32_t>(), nca, cnt_a, cnt_b,
                                         gb.start.as<uint32_t>(), ncb, cnt_b, ctx->scratch[4].p,
                                         true))
        return rc;
    ctx->cell_cnt_dirty = ctx->cell_cnt2_dirty = false;
    PCP_HIP(ctx, ga.pts.ensure((size_t)nfin * sizeof(float4)));
    PCP_HIP(ctx, gb.pts.ensure((size_t)nfin * sizeof(float4)));
    hipLaunchKernelGGL(k_cell_place2, dim3(gridn), dim3(kThreads), 0, st,
                       ctx->scratch[0].as<const float4>(), n, (const uint2 *)cr_a,
                       ga.start.as<const uint32_t>(), ga.pts.as<float4>(), (const uint2 *)cr_b,
                       gb.start.as<const uint32_t>(), gb.pts.as<float4>());
    PCP_CHECK_LAUNCH(ctx);
    ga.present = gb.present = true;
    *paired = true;
    return PCP_OK;
}

int build_index(pcp_ctx *ctx, GridIndex &g, const pcp_cloud_view &v, double r_q, bool zsort,
                bool occ, const unsigned char **raw_io, unsigned char *raw_copy) {
    const uint64_t n = v.n;
    hipStream_t st = ctx->stream;
    // the query kernels address points and cells with 32-bit byte offsets (pcp_stencil.hpp)
    if (n >= (1ull << 28))
        return set_err(ctx, PCP_E_INVALID, "index cloud of %llu points exceeds 2^28",
                       (unsigned long long)n);
    ProfScope prof(ctx, PCP_K_INDEX_BUILD);
    // Invalidate everything derived from the previous cloud first: an early return below (e.g.
    // an allocation failure after the new geometry is written) must not leave the old block
    // copy or z bands paired with the new grid.  present is set again only on success.
    g.present = false;
    g.occz_ok = false;
    g.occ2_ok = false;
    g.blk_ok = false;
    g.blk_fail = false;
    g.fine_ok = false;
    g.fine_fail = false;
    // 1. the raw AoS bytes (the PointCloud2 data blob), device-readable: given by the caller,
    //    read in place from the pinned ring (message-sized), or DMA'd into ctx->stage
    const uint64_t raw_bytes = n * (uint64_t)v.point_step;
    const unsigned char *raw = raw_io ? *raw_io : nullptr;
    bool pinned = false;
    if (!raw && n && ctx->zc_in && raw_bytes <= kPinDirectMax) {
        const HostPiece pc{0, v.data, raw_bytes};
        const void *dv = nullptr;
        if (int rc0 = pin_stage(ctx, &pc, 1, raw_bytes, &dv)) return rc0;
        raw = static_cast<const unsigned char *>(dv);
        pinned = true;
    }
    if (!raw) {
        PCP_HIP(ctx, ctx->stage.ensure(raw_bytes));
        if (int rc0 = upload_async(ctx, ctx->stage.p, v.data, raw_bytes, st)) return rc0;
        raw = ctx->stage.as<unsigned char>();
    }
    // raw_copy: fused into the extraction (message-sized clouds, 16-byte records), else a
    // device copy first
    const bool host_bb = n <= kHostBboxMax;
    const bool fuse_copy = raw_copy && host_bb && n && (v.point_step & 15u) == 0 &&
                           v.point_step <= 64 &&
                           ((reinterpret_cast<uintptr_t>(raw) | reinterpret_cast<uintptr_t>(raw_copy)) & 15u) == 0;
    if (raw_copy && n && !fuse_copy) {
        if (int rc0 = copy_pinned_async(ctx, raw_copy, raw, raw_bytes, st)) return rc0;
        raw = raw_copy;
    }
    if (raw_io) *raw_io = raw_copy && n ? raw_copy : raw;
    // the extraction is the index's only reader of the raw bytes
    auto release_raw = [&]() {
        if (pinned && !raw_io) pin_release(ctx, st);
    };
    // 2. extract + bbox
    const int nb = (int)std::min<uint64_t>((n + kThreads - 1) / kThreads, 1024);
    PCP_HIP(ctx, ctx->scratch[0].ensure(n * sizeof(float4)));
    PCP_HIP(ctx, ctx->scratch[1].ensure((size_t)nb * 6 * sizeof(float) + 64 + nb * 4));
    PCP_HIP(ctx, ctx->stats_d.ensure(64));
    float *part = ctx->scratch[1].as<float>();
    uint32_t *part_n = reinterpret_cast<uint32_t *>(part + nb * 6);
    float bb_h[10];
    uint32_t nfin;
    // a message-sized cloud: the grid geometry from the host's copy of the same bytes (the
    // same float min / max over the finite points, order-free) -- no round trip through the
    // stream; the extraction is launched below, fused with the cell count
    if (host_bb) {
        host_bbox(v, bb_h, nfin);
    } else {
        hipLaunchKernelGGL(k_extract, dim3(nb), dim3(kThreads), 0, st, raw, n, v.point_step,
                           v.off_x, v.off_y, v.off_z, ctx->scratch[0].as<float4>(), part, part_n,
                           nullptr, (uint64_t)0);
        PCP_CHECK_LAUNCH(ctx);
        release_raw();
        float *bb_d = ctx->stats_d.as<float>();
        hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(kThreads), 0, st, part, part_n, nb, bb_d,
                           reinterpret_cast<uint32_t *>(bb_d + 8));
        PCP_CHECK_LAUNCH(ctx);
        if (int rc0 = read_small(ctx, bb_h, bb_d, sizeof(bb_h), st)) return rc0;
        memcpy(&nfin, &bb_h[8], 4);
    }
    g.r_q = r_q;
    g.n_pts = nfin;
    if (nfin == 0) {   // a tree over zero valid points: never returns neighbours
        // (no extraction to carry the copy the caller reads from)
        if (fuse_copy)
            if (int rc0 = copy_pinned_async(ctx, raw_copy, raw, raw_bytes, st)) return rc0;
        release_raw();
        g.c = 1.0;
        g.nx = g.ny = g.nz = 1;
        for (int a = 0; a < 3; ++a) g.bmin[a] = g.bmax[a] = 0.0;
        PCP_HIP(ctx, g.pts.ensure(16));
        PCP_HIP(ctx, g.start.ensure(16));
        PCP_HIP(ctx, g.occ2.ensure(16));
        PCP_HIP(ctx, hipMemsetAsync(g.start.p, 0, 16, st));
        PCP_HIP(ctx, hipMemsetAsync(g.occ2.p, 0, 16, st));
        g.occ2_ok = true;
        // one empty z band (lo 255, hi 0) for the single cell
        PCP_HIP(ctx, g.occz.ensure(16));
        PCP_HIP(ctx, hipMemsetAsync(g.occz.p, 0xFF, 1, st));
        PCP_HIP(ctx, hipMemsetAsync(static_cast<char *>(g.occz.p) + 1, 0, 1, st));
        g.occz_ok = zsort;
        g.present = true;
        return PCP_OK;
    }
    // 3. grid geometry
    const uint64_t ncell = grid_geometry(g, bb_h);
    const double c = g.c;
    const GridView gv = g.view();
    CellMap m{gv.ox, gv.oy, gv.oz, gv.inv_c, g.nx, g.ny, g.nz};
    // 4. each point's cell and slot in it.  The counters are all zero between builds (the scan
    //    below clears what this build counts), so nothing zeroes them here; a new or grown
    //    buffer, or one left dirty by a build that stopped early, is cleared first
    const size_t cnt_b = (ncell + 1) * sizeof(uint32_t);
    if (ctx->cell_cnt.cap < cnt_b || ctx->cell_cnt_dirty) {
        PCP_HIP(ctx, ctx->cell_cnt.ensure(cnt_b));
        PCP_HIP(ctx, hipMemsetAsync(ctx->cell_cnt.p, 0, ctx->cell_cnt.cap, st));
        ctx->cell_cnt_dirty = false;
    }
    uint32_t *cnt = ctx->cell_cnt.as<uint32_t>();
    PCP_HIP(ctx, ctx->scratch[2].ensure(n * sizeof(uint2)));
    uint2 *cr = ctx->scratch[2].as<uint2>();
    const unsigned gridn = (unsigned)((n + kThreads - 1) / kThreads);
    ctx->cell_cnt_dirty = true;
    if (host_bb) {   // one pass over the raw records: extraction, cell, slot
        hipLaunchKernelGGL(k_extract_count, dim3(gridn), dim3(kThreads), 0, st, raw, n,
                           v.point_step, v.off_x, v.off_y, v.off_z, m,
                           ctx->scratch[0].as<float4>(), cnt, cr,
                           fuse_copy ? raw_copy : (unsigned char *)nullptr);
        PCP_CHECK_LAUNCH(ctx);
        release_raw();
    } else {
        hipLaunchKernelGGL(k_cell_count_ranked, dim3(gridn), dim3(kThreads), 0, st,
                           ctx->scratch[0].as<const float4>(), n, m, cnt, cr);
        PCP_CHECK_LAUNCH(ctx);
    }
    // 5. prefix -> start; the scan clears the counters behind it (and, for a mostly empty
    // z-sorted grid, presets its z bands: no memset launch in front of k_occz_sparse)
    PCP_HIP(ctx, g.start.ensure((ncell + 1) * sizeof(uint32_t)));
    PCP_HIP(ctx, ctx->scratch[4].ensure(scan_tmp_bytes(ncell) + (ncell + 1) * sizeof(uint32_t)));
    const bool sparse_z = zsort && ncell > kSparseCells * (uint64_t)nfin;
    if (zsort) PCP_HIP(ctx, g.occz.ensure(ncell * sizeof(uint16_t)));
    int rc = exclusive_scan_u32(ctx, cnt, g.start.as<uint32_t>(), ncell, ctx->scratch[4].p, cnt,
                                true, sparse_z ? g.occz.as<uint16_t>() : nullptr);
    if (rc) return rc;
    ctx->cell_cnt_dirty = false;
    // 6. every point to its cell's start + its slot
    PCP_HIP(ctx, g.pts.ensure((size_t)nfin * sizeof(float4)));
    // (with zsort the points land in a temporary and the rank pass writes g.pts)
    if (zsort) PCP_HIP(ctx, ctx->scratch[5].ensure((size_t)nfin * sizeof(float4)));
    float4 *scat = zsort ? ctx->scratch[5].as<float4>() : g.pts.as<float4>();
    hipLaunchKernelGGL(k_cell_place, dim3(gridn), dim3(kThreads), 0, st,
                       ctx->scratch[0].as<const float4>(), n, (const uint2 *)cr,
                       g.start.as<const uint32_t>(), scat);
    PCP_CHECK_LAUNCH(ctx);
    // 7. descending z inside each cell (the ray-march indices only)
    if (zsort) {
        hipLaunchKernelGGL(k_cell_rank_z, dim3((unsigned)((nfin + kThreads - 1) / kThreads)),
                           dim3(kThreads), 0, st, (const float4 *)scat, (uint64_t)nfin, m,
                           g.start.as<const uint32_t>(), g.pts.as<float4>());
        PCP_CHECK_LAUNCH(ctx);
    }
    // 8. dilated occupancy (one pass over every cell: only for indices that stencil_any queries)
    g.occ2_ok = false;
    if (occ) {
        const uint64_t nw = (ncell + 31) / 32;
        PCP_HIP(ctx, g.occ2.ensure(nw * sizeof(uint32_t)));
        hipLaunchKernelGGL(k_occ2, dim3((unsigned)((ncell + kThreads - 1) / kThreads)),
                           dim3(kThreads), 0, st, g.start.as<const uint32_t>(), m, ncell,
                           g.occ2.as<uint32_t>());
        PCP_CHECK_LAUNCH(ctx);
        g.occ2_ok = true;
    }
    // 8b. z band per stencil corner (the fan march's probe), z-sorted indices only
    g.occz_ok = false;
    if (zsort) {
        if (sparse_z) {   // mostly empty: the scan preset every band, now the occupied cells'
            hipLaunchKernelGGL(k_occz_sparse, dim3((unsigned)((8 * (uint64_t)nfin + kThreads - 1) / kThreads)),
                               dim3(kThreads), 0, st, g.start.as<const uint32_t>(),
                               g.pts.as<const float4>(), m, c, (uint64_t)nfin,
                               g.occz.as<uint16_t>());
        } else {
            hipLaunchKernelGGL(k_occz, dim3((unsigned)((ncell + kThreads - 1) / kThreads)),
                               dim3(kThreads), 0, st, g.start.as<const uint32_t>(),
                               g.pts.as<const float4>(), m, c, ncell, g.occz.as<uint16_t>());
        }
        PCP_CHECK_LAUNCH(ctx);
        g.occz_ok = true;
    }
    // no synchronisation: the index is used by later work on the same stream
    g.present = true;
    return PCP_OK;
}

// block-major copy: count per corner -> prefix -> fill (every point lands in the blocks of its
// 8 corners, ~8 n entries; not built past the 2^28 point cap -- the scans fall back to the
// per-cell runs)
int build_blocks(pcp_ctx *ctx, GridIndex &g) {
    if (g.blk_ok || g.blk_fail || !g.present || !g.occz_ok || g.n_pts == 0) return PCP_OK;
    hipStream_t st = ctx->stream;
    ProfScope prof(ctx, PCP_K_INDEX_BUILD);
    const GridView gv = g.view();
    const CellMap m{gv.ox, gv.oy, gv.oz, gv.inv_c, g.nx, g.ny, g.nz};
    const uint64_t ncell = (uint64_t)g.nx * (uint64_t)g.ny * (uint64_t)g.nz;
    PCP_HIP(ctx, ctx->scratch[3].ensure((ncell + 1) * sizeof(uint32_t)));
    PCP_HIP(ctx, ctx->scratch[4].ensure(scan_tmp_bytes(ncell) + (ncell + 1) * sizeof(uint32_t)));
    uint32_t *cnt = ctx->scratch[3].as<uint32_t>();
    hipLaunchKernelGGL(k_blk_count, dim3((unsigned)((ncell + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, g.start.as<const uint32_t>(), m, ncell, cnt);
    PCP_CHECK_LAUNCH(ctx);
    PCP_HIP(ctx, g.bstart.ensure((ncell + 1) * sizeof(uint32_t)));
    int rc = exclusive_scan_u32(ctx, cnt, g.bstart.as<uint32_t>(), ncell, ctx->scratch[4].p);
    if (rc) return rc;
    uint32_t nb_tot = 0;
    if ((rc = read_small(ctx, &nb_tot, g.bstart.as<uint32_t>() + ncell, 4, st))) return rc;
    if (nb_tot == 0 || nb_tot >= (1u << 28)) {   // past the 32-bit offset cap: never retry
        g.blk_fail = true;
        return PCP_OK;
    }
    // the copy is an optional speed-up: if it cannot be allocated, the queries keep the
    // per-cell runs (scan_stencil) instead of failing, and no later query retries
    if (g.bpts.ensure((size_t)nb_tot * sizeof(float4)) != hipSuccess) {
        (void)hipGetLastError();
        g.bpts.release();
        g.blk_fail = true;
        return PCP_OK;
    }
    const uint64_t n = g.n_pts;
    hipLaunchKernelGGL(k_blk_fill, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads),
                       0, st, g.pts.as<const float4>(), n, g.start.as<const uint32_t>(), m,
                       g.bstart.as<const uint32_t>(), g.bpts.as<float4>());
    PCP_CHECK_LAUNCH(ctx);
    g.blk_ok = true;
    return PCP_OK;
}

int terrain_blocks_before_query(pcp_ctx *ctx) {
    GridIndex &t = ctx->terrain;
    if (ctx->terrain_blocks <= 0 || t.blk_ok || t.fine_ok || t.blk_fail || !t.present)
        return PCP_OK;
    ++ctx->terrain_queries;
    if (ctx->terrain_blocks == 1 && ctx->terrain_queries < 2) return PCP_OK;
    if (ctx->terrain_fine && !t.fine_fail) {
        if (int rc = build_fine(ctx, t)) return rc;
        if (t.fine_ok) return PCP_OK;
    }
    return build_blocks(ctx, t);   // the 2x2x2 block copy (also past the fine copy's caps)
}

int set_terrain_from(pcp_ctx *ctx, const pcp_cloud_view *terrain, const unsigned char *raw_pre) {
    if (!ctx) return PCP_E_INVALID;
    int rc = check_view(ctx, terrain, "pcp_set_terrain");
    if (rc) return rc;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    ctx->terrain_cloud_n = terrain->n;
    if (terrain->n == 0) return PCP_OK;   // terrainCallback: no rebuild on an empty cloud
    // the march probes the z bands; occupancy bits only for the fan's A/B variant 2
    const unsigned char *raw = raw_pre;
    rc = build_index(ctx, ctx->terrain, *terrain, kRayRadius, true, ctx->fan_batch == 2,
                     raw ? &raw : nullptr);
    ctx->terrain_queries = 0;
    prof_resolve(ctx);
    return rc;
}

}  // namespace pcp

using namespace pcp;

extern "C" {

int pcp_set_terrain(pcp_ctx *ctx, const pcp_cloud_view *terrain) {
    return set_terrain_from(ctx, terrain, nullptr);
}

int pcp_set_aux_cloud(pcp_ctx *ctx, const pcp_cloud_view *aux) {
    if (!ctx) return PCP_E_INVALID;
    int rc = check_view(ctx, aux, "pcp_set_aux_cloud");
    if (rc) return rc;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    ctx->aux_cloud_n = aux->n;
    if (aux->n == 0) return PCP_OK;
    rc = build_index(ctx, ctx->aux, *aux, kRelaxedRadius);
    prof_resolve(ctx);
    return rc;
}

int pcp_terrain_info(pcp_ctx *ctx, pcp_index_info *info) {
    if (!ctx || !info) return PCP_E_INVALID;
    const GridIndex &g = ctx->terrain;
    info->n_points = g.n_pts;
    info->cell = g.c;
    info->nx = g.nx;
    info->ny = g.ny;
    info->nz = g.nz;
    for (int a = 0; a < 3; ++a) {
        info->bmin[a] = g.bmin[a];
        info->bmax[a] = g.bmax[a];
    }
    info->scan_layout = g.fine_ok ? 2 : g.blk_ok ? 1 : 0;
    info->fine_tile = g.fine_ok ? g.ftile : 0;
    return PCP_OK;
}

}  // extern "C"
