// pcp_rigid.hpp -- the float SE(3) of tf2::doTransform(PointCloud2) (Eigen Affine3f): shared
// by the merger (pcp_filter.hip) and the drivable-area grid (pcp_drivable.hip).
#pragma once
#pragma clang fp contract(off)

#include <cstdint>

#include "pcp_internal.hpp"

namespace pcp {

// ---- SE(3) + colour (tf2::doTransform + processRobotCloud loop) ------------------------------
struct Rigid {
    float m00, m01, m02, m10, m11, m12, m20, m21, m22, tx, ty, tz;
    uint32_t rgba;
};

inline Rigid make_rigid(const pcp_rigid &t, const uint8_t rgb[3]) {
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
__device__ __forceinline__ void xform_pt(const Rigid &r, float x, float y, float z, float &X,
                                         float &Y, float &Z) {
    X = ((r.m00 * x + r.m01 * y) + r.m02 * z) + r.tx;
    Y = ((r.m10 * x + r.m11 * y) + r.m12 * z) + r.ty;
    Z = ((r.m20 * x + r.m21 * y) + r.m22 * z) + r.tz;
}

__device__ __forceinline__ void xform_store(const Rigid &r, float x, float y, float z, float4 *o) {
    float X, Y, Z;
    xform_pt(r, x, y, z, X, Y, Z);
    o[0] = make_float4(X, Y, Z, 1.0f);
    o[1] = make_float4(__uint_as_float(r.rgba), 0.f, 0.f, 0.f);
}

}  // namespace pcp
