/* pcp_libm.h -- the float libm calls of pcl::eigen33 (computeRoots: atan2f, cosf, sinf, sqrtf)
 * as the reference's platform computes them, so that the GPU's PCA normals are bit-identical to
 * a CPU build of the reference on Ubuntu 22.04 / glibc 2.35 (ROS 2 Humble, README.md:9) -- and to
 * the oracle, which calls that glibc.  C and HIP (host + device) from one text: the CPU suite
 * checks this text against the running glibc (tests/test_libm.py), the GPU compiles the same.
 *
 * Restated algorithms (public, not the reference's code):
 *  - atan2f / atanf: glibc 2.35 sysdeps/ieee754/flt-32/e_atan2f.c + s_atanf.c (the fdlibm float
 *    versions; no ifunc variants on x86_64: every multiply and add rounds separately).
 *  - sinf / cosf: glibc 2.35 sysdeps/ieee754/flt-32/s_sinf.c / s_cosf.c + sincosf.h (double
 *    polynomials over __sincosf_table); x86_64 selects the FMA build of both by ifunc on
 *    FMA-capable CPUs, whose compiler contracts each `a + b * c` of the polynomials and
 *    `x - n * hpi` of the reduction into one fma -- reproduced here with explicit fma() when
 *    PCP_LIBM_SINCOS_FMA is 1 (the default; 0 restates the SSE2 build).
 *    Only |x| < 120 is restated (computeRoots' angle lies in [0, pi/3]).
 *  - sqrtf and float division: correctly rounded on both sides (IEEE); written through double,
 *    which is exact-then-rounded-once for both operations at float precision.
 * Compile with -ffp-contract=off: every other operation must round on its own.
 *
 * Notices of the restated upstream code (its constants and control flow are reproduced here):
 *
 *   atanf / atan2f (fdlibm, as carried by glibc):
 *   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
 *   Developed at SunPro, a Sun Microsystems, Inc. business.
 *   Permission to use, copy, modify, and distribute this software is freely granted, provided
 *   that this notice is preserved.
 *
 *   sinf / cosf / sincosf.h (Arm optimized-routines, as carried by glibc 2.35):
 *   Copyright (c) 2018 Arm Ltd.  Contributed to the GNU C Library, which distributes it under
 *   the GNU Lesser General Public License v2.1 or later; upstream Arm optimized-routines
 *   license the same code under SPDX-License-Identifier: MIT OR Apache-2.0 WITH LLVM-exception.
 */
#ifndef PCP_LIBM_H
#define PCP_LIBM_H

#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define PCP_LM static __host__ __device__ __forceinline__
#else
#define PCP_LM static inline
#endif

#ifndef PCP_LIBM_SINCOS_FMA
#define PCP_LIBM_SINCOS_FMA 1
#endif

PCP_LM uint32_t pcp_lm_asu(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
PCP_LM float pcp_lm_asf(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
/* correctly rounded float division and square root */
PCP_LM float pcp_lm_div(float a, float b) { return (float)((double)a / (double)b); }
PCP_LM float pcp_lm_sqrt(float a) { return (float)sqrt((double)a); }

/* ---- atanf (s_atanf.c) ------------------------------------------------------------------ */
PCP_LM float pcp_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f,
                             1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f,
                             7.5497894159e-08f};
    const float aT[11] = {3.3333334327e-01f,  -2.0000000298e-01f, 1.4285714924e-01f,
                          -1.1111110449e-01f, 9.0908870101e-02f,  -7.6918758452e-02f,
                          6.6610731184e-02f,  -5.8335702866e-02f, 4.9768779427e-02f,
                          -3.6531571299e-02f, 1.6285819933e-02f};
    const int32_t hx = (int32_t)pcp_lm_asu(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) { /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) { /* |x| < 0.4375 */
        if (ix < 0x31000000) return x; /* |x| < 2^-29 */
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {     /* |x| < 1.1875 */
            if (ix < 0x3f300000) { /* 7/16 <= |x| < 11/16 */
                id = 0;
                x = pcp_lm_div(2.0f * x - 1.0f, 2.0f + x);
            } else { /* 11/16 <= |x| < 19/16 */
                id = 1;
                x = pcp_lm_div(x - 1.0f, x + 1.0f);
            }
        } else {
            if (ix < 0x401c0000) { /* |x| < 2.4375 */
                id = 2;
                x = pcp_lm_div(x - 1.5f, 1.0f + 1.5f * x);
            } else { /* 2.4375 <= |x| < 2^25 */
                id = 3;
                x = pcp_lm_div(-1.0f, x);
            }
        }
    }
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const float s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const float r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}

/* ---- atan2f (e_atan2f.c) ------------------------------------------------------------------ */
PCP_LM float pcp_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    const int32_t hx = (int32_t)pcp_lm_asu(x), hy = (int32_t)pcp_lm_asu(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y; /* NaN */
    if (hx == 0x3f800000) return pcp_atanf(y);            /* x = 1 */
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      /* 2 sign(x) + sign(y) */
    if (iy == 0) {
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0f * pi_o_4 + tiny;
            default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60)
        z = pi_o_2 + 0.5f * pi_lo; /* |y/x| > 2^60 */
    else if (hx < 0 && k < -60)
        z = 0.0f;                  /* |y|/x < -2^60 */
    else
        z = pcp_atanf(fabsf(pcp_lm_div(y, x)));
    switch (m) {
    case 0: return z;
    case 1: return pcp_lm_asf(pcp_lm_asu(z) ^ 0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

/* ---- sinf / cosf (s_sinf.c, s_cosf.c, sincosf.h) ------------------------------------------ */
#if PCP_LIBM_SINCOS_FMA
#define PCP_LM_MAD(a, b, c) fma((a), (b), (c)) /* c + a * b, contracted */
#else
#define PCP_LM_MAD(a, b, c) ((c) + (a) * (b))
#endif
/* __sincosf_table[t]: c0 .. c4, s1 .. s3 (t = 1: the cos coefficients negated) */
PCP_LM double pcp_lm_sincos_poly(double x, double x2, int t, int n) {
    const double sg = t ? -1.0 : 1.0;
    if ((n & 1) == 0) {
        const double s1c = -0x1.555545995a603p-3, s2c = 0x1.1107605230bc4p-7,
                     s3c = -0x1.994eb3774cf24p-13;
        const double x3 = x * x2;
        const double s1 = PCP_LM_MAD(x2, s3c, s2c);
        const double x7 = x3 * x2;
        const double s = PCP_LM_MAD(x3, s1c, x);
        return PCP_LM_MAD(x7, s1, s);
    }
    const double c0 = sg * 0x1p0, c1 = sg * -0x1.ffffffd0c621cp-2, c2 = sg * 0x1.55553e1068f19p-5,
                 c3 = sg * -0x1.6c087e89a359dp-10, c4 = sg * 0x1.99343027bf8c3p-16;
    const double x4 = x2 * x2;
    const double h2 = PCP_LM_MAD(x2, c4, c3);   /* c3 + x2 c4 */
    const double h1 = PCP_LM_MAD(x2, c1, c0);   /* c0 + x2 c1 */
    const double x6 = x4 * x2;
    const double c = PCP_LM_MAD(x4, c2, h1);    /* h1 + x4 c2 */
    return PCP_LM_MAD(x6, h2, c);               /* c + x6 h2 */
}
PCP_LM uint32_t pcp_lm_abstop12(float x) { return (pcp_lm_asu(x) >> 20) & 0x7ff; }
/* reduce_fast: n = round(x 2 / pi), x - n pi / 2 */
PCP_LM double pcp_lm_reduce(double x, int *np) {
    const double hpi_inv = 0x1.45F306DC9C883p+23, hpi = 0x1.921FB54442D18p0;
    const double r = x * hpi_inv;
    const int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return PCP_LM_MAD(-(double)n, hpi, x);
}
PCP_LM float pcp_sinf(float y) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (pcp_lm_abstop12(y) < pcp_lm_abstop12(pio4)) {
        if (pcp_lm_abstop12(y) < pcp_lm_abstop12(0x1p-12f)) return y;
        return (float)pcp_lm_sincos_poly(x, x * x, 0, 0);
    }
    int n;
    x = pcp_lm_reduce(x, &n);
    const double sign[4] = {1.0, -1.0, -1.0, 1.0};
    const double s = sign[n & 3];
    return (float)pcp_lm_sincos_poly(x * s, x * x, (n & 2) ? 1 : 0, n);
}
PCP_LM float pcp_cosf(float y) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (pcp_lm_abstop12(y) < pcp_lm_abstop12(pio4)) {
        if (pcp_lm_abstop12(y) < pcp_lm_abstop12(0x1p-12f)) return 1.0f;
        return (float)pcp_lm_sincos_poly(x, x * x, 0, 1);
    }
    int n;
    x = pcp_lm_reduce(x, &n);
    const double sign[4] = {1.0, -1.0, -1.0, 1.0};
    const double s = sign[n & 3];
    return (float)pcp_lm_sincos_poly(x * s, x * x, (n & 2) ? 1 : 0, n ^ 1);
}
#undef PCP_LM_MAD

#endif /* PCP_LIBM_H */
