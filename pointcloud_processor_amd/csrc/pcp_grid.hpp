// pcp_grid.hpp -- device helpers of the grid index builds (pcp_index.hip, pcp_fine.hip)
#pragma once
#pragma clang fp contract(off)

#include "pcp_internal.hpp"

namespace pcp {

struct CellMap {
    double ox, oy, oz, inv_c;
    int32_t nx, ny, nz;
};

__device__ __forceinline__ uint32_t cell_of(const CellMap &m, float x, float y, float z) {
    int ix = (int)floor(((double)x - m.ox) * m.inv_c);
    int iy = (int)floor(((double)y - m.oy) * m.inv_c);
    int iz = (int)floor(((double)z - m.oz) * m.inv_c);
    // points lie in [1, n-2] by construction; clamp defensively
    ix = min(max(ix, 0), m.nx - 1);
    iy = min(max(iy, 0), m.ny - 1);
    iz = min(max(iz, 0), m.nz - 1);
    return (uint32_t)ix + (uint32_t)m.nx * ((uint32_t)iy + (uint32_t)m.ny * (uint32_t)iz);
}

// a point's z cell (cell_of's z)
__device__ __forceinline__ int cell_z(const CellMap &m, float z) {
    const int iz = (int)floor(((double)z - m.oz) * m.inv_c);
    return min(max(iz, 0), m.nz - 1);
}

// u16 z band lo | hi << 8 of points with z in [zmin, zmax] above a block floor zb (cell edge c)
__device__ __forceinline__ uint32_t zband_code(float zmax, float zmin, double zb, double c) {
    const double step = (double)kZq * c;
    const double h = ceil(((double)zmax - zb) / step) + 1.0;
    const double l = floor(((double)zmin - zb) / step) - 1.0;
    const uint32_t hi = h >= 255.0 ? 255u : (uint32_t)fmax(h, 1.0);
    const uint32_t lo = l <= 0.0 ? 0u : (uint32_t)fmin(l, 254.0);
    return lo | (hi << 8);
}

}  // namespace pcp
