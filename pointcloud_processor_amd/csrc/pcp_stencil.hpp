// pcp_stencil.hpp -- device helpers shared by the kernels that query a GridIndex: FLANN's
// radius predicate and the float stencil corner (Terrain index).
#pragma once
#pragma clang fp contract(off)

#include "pcp_internal.hpp"

namespace pcp {

// a terrain point's x, y, z (the .w index is not needed by the test: 12-byte loads)
struct P3 {
    float x, y, z;
};
__device__ __forceinline__ P3 ld_p3(const float4 *pts, uint32_t i) {
    const float *f = reinterpret_cast<const float *>(pts + i);
    return P3{f[0], f[1], f[2]};
}

// FLANN L2_Simple<float>: result += diff*diff over x, y, z; returned iff result < r2
template <class PT>
__device__ __forceinline__ bool flann_within(float qx, float qy, float qz, const PT &p,
                                             float r2) {
    const float d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
    float acc = 0.0f;
    acc = acc + d0 * d0;
    acc = acc + d1 * d1;
    acc = acc + d2 * d2;
    return acc < r2;
}

// The same corner in float.  Exact in outcome: a corner off by one (the value within the float
// error of a cell boundary) still holds every point within r of q while the error is below the
// query margin m (the block keeps >= m of slack on the low side and c - 2r - m on the high
// side); the rounding here is ~1e-5 m against m = 1e-3 m.  The same holds at the grid border,
// where the off-by-one block is padding / outside (empty).
__device__ __forceinline__ bool stencil_cell3_f(const GridView &g, float qx, float qy, float qz,
                                                uint32_t &ix, uint32_t &iy, uint32_t &iz) {
    const float fx = (qx - g.flo_x) * g.finv_c;
    const float fy = (qy - g.flo_y) * g.finv_c;
    const float fz = (qz - g.flo_z) * g.finv_c;
    if (!(fx >= 0.0f && fx < g.fnx1 && fy >= 0.0f && fy < g.fny1 && fz >= 0.0f && fz < g.fnz1))
        return false;
    ix = (uint32_t)fx;
    iy = (uint32_t)fy;
    iz = (uint32_t)fz;
    return true;
}

// The same test as one predicate (no short-circuit chain: one exec mask instead of three nested
// branches).  The indices are only meaningful when it returns true.
__device__ __forceinline__ bool stencil_cell3_fb(const GridView &g, float qx, float qy, float qz,
                                                 uint32_t &ix, uint32_t &iy, uint32_t &iz) {
    const float fx = (qx - g.flo_x) * g.finv_c;
    const float fy = (qy - g.flo_y) * g.finv_c;
    const float fz = (qz - g.flo_z) * g.finv_c;
    const bool ok = (fx >= 0.0f) & (fx < g.fnx1) & (fy >= 0.0f) & (fy < g.fny1) & (fz >= 0.0f) &
                    (fz < g.fnz1);
    ix = ok ? (uint32_t)fx : 0u;
    iy = ok ? (uint32_t)fy : 0u;
    iz = ok ? (uint32_t)fz : 0u;
    return ok;
}

// Loads at 32-bit byte offsets from a kernel-argument base: one voffset VGPR and the base in
// SGPRs (global_load ... v, s[base:base+1]) instead of a 64-bit address add per load.  Valid
// while the arrays stay below 4 GiB: build_index caps an index at 2^28 points and 2^25 cells.
__device__ __forceinline__ uint32_t ld_u32o(const uint32_t *base, uint32_t i) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(base) + (i << 2));
}
// three consecutive directory entries (cells c, c+1, c+2 of one stencil row) in ONE load
// instruction: one L1 tag lookup per lane instead of three (the fan kernel is bound by the
// texture address / data path, one tag lookup per distinct line per lane and instruction)
struct U3 {
    uint32_t a, b, c;
};
__device__ __forceinline__ U3 ld_u3o(const uint32_t *base, uint32_t i) {
    return *reinterpret_cast<const U3 *>(reinterpret_cast<const char *>(base) + (i << 2));
}
// two consecutive directory entries (a block's start and end) in one load
__device__ __forceinline__ uint2 ld_u2o(const uint32_t *base, uint32_t i) {
    const uint32_t *p =
        reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(base) + (i << 2));
    return make_uint2(p[0], p[1]);
}
// one 8-byte record (the fine-window directory: {start, band | count << 16}; build_fine caps
// the directory below 2^29 records)
__device__ __forceinline__ uint2 ld_rec(const uint2 *base, uint32_t i) {
    return *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(base) + (i << 3));
}
__device__ __forceinline__ uint32_t ld_u16o(const uint16_t *base, uint32_t i) {
    return *reinterpret_cast<const uint16_t *>(reinterpret_cast<const char *>(base) + (i << 1));
}
__device__ __forceinline__ P3 ld_p3o(const float4 *pts, uint32_t i) {
    const float *f =
        reinterpret_cast<const float *>(reinterpret_cast<const char *>(pts) + (i << 4));
    return P3{f[0], f[1], f[2]};
}

}  // namespace pcp
