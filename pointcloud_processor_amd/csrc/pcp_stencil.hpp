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

}  // namespace pcp
