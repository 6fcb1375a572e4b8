/* pcp_crmath.h -- correctly rounded double atan2 from a faithful first result, for the device
 * (ocml's atan2 is within an ulp; glibc's, which the reference and the oracle call, rounds
 * correctly in all but rare cases -- tools/libm_cr_check.py).  C and HIP (host + device) from
 * one text: the CPU suite checks it against the running glibc (tests/test_crmath.py).
 *
 * pcp_cr_atan2_fix(y, x, r): r is atan2(y, x) to within one ulp.  The true angle t lies between
 * r's neighbours; it is compared with the two midpoints m = r -+ ulp / 2 through the sign of
 *     sin(t - m) = (y cos m - x sin m) / |(x, y)|
 * with cos m and sin m in double-double (Cody-Waite reduction by pi / 2 in three parts, Taylor
 * series to t^31 for |t| <= pi / 4), so the sign is decided unless t lies within ~2^-100 of a
 * midpoint.  Zeros, infinities, NaNs and |r| < 2^-900 return r unchanged.
 * (The same construction for the scoring's acos and sin, virtual_lidar.cpp:700-705, lives in
 * tests/libm/crmath_extra.h: checked on the CPU, not used by a kernel, because glibc misrounds
 * those near ties more often than ocml disagrees with it -- DESIGN.md §8.)
 * Compile with -ffp-contract=off: the error-free transformations need every operation rounded
 * on its own (fma() is called explicitly where one is meant).
 */
#ifndef PCP_CRMATH_H
#define PCP_CRMATH_H

#include <math.h>

#if defined(__HIPCC__)
#define PCP_CR static __host__ __device__ __forceinline__
#else
#define PCP_CR static inline
#endif

typedef struct {
    double hi, lo;
} pcp_dd;

PCP_CR pcp_dd pcp_dd_make(double hi, double lo) {
    pcp_dd r;
    r.hi = hi;
    r.lo = lo;
    return r;
}

PCP_CR pcp_dd pcp_two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return pcp_dd_make(s, (a - (s - bb)) + (b - bb));
}

PCP_CR pcp_dd pcp_fast_two_sum(double a, double b) {   /* |a| >= |b| or a == 0 */
    const double s = a + b;
    return pcp_dd_make(s, b - (s - a));
}

PCP_CR pcp_dd pcp_two_prod(double a, double b) {
    const double p = a * b;
    return pcp_dd_make(p, fma(a, b, -p));
}

PCP_CR pcp_dd pcp_dd_add(pcp_dd a, pcp_dd b) {
    pcp_dd s = pcp_two_sum(a.hi, b.hi);
    const pcp_dd t = pcp_two_sum(a.lo, b.lo);
    s = pcp_fast_two_sum(s.hi, s.lo + t.hi);
    return pcp_fast_two_sum(s.hi, s.lo + t.lo);
}

PCP_CR pcp_dd pcp_dd_neg(pcp_dd a) { return pcp_dd_make(-a.hi, -a.lo); }

PCP_CR pcp_dd pcp_dd_mul(pcp_dd a, pcp_dd b) {
    const pcp_dd p = pcp_two_prod(a.hi, b.hi);
    return pcp_fast_two_sum(p.hi, p.lo + (a.hi * b.lo + a.lo * b.hi));
}

PCP_CR pcp_dd pcp_dd_mul_d(pcp_dd a, double b) {
    const pcp_dd p = pcp_two_prod(a.hi, b);
    return pcp_fast_two_sum(p.hi, p.lo + a.lo * b);
}

PCP_CR pcp_dd pcp_dd_div_d(pcp_dd a, double d) {   /* d a small positive integer */
    const double q1 = a.hi / d;
    const pcp_dd p = pcp_two_prod(q1, d);
    const double r = ((a.hi - p.hi) - p.lo) + a.lo;
    return pcp_fast_two_sum(q1, r / d);
}

/* (-1)^k / (2k + 1)! and (-1)^k / (2k)! as double-doubles (exact fractions rounded twice) */
#if defined(__cplusplus)
#define PCP_CR_CONST static constexpr
#else
#define PCP_CR_CONST static const
#endif
PCP_CR_CONST double kPcpSinC[15][2] = {
    {1.0, 0.0},
    {-0.16666666666666666, -9.25185853854297e-18},
    {0.008333333333333333, 1.1564823173178714e-19},
    {-0.0001984126984126984, -1.7209558293420705e-22},
    {2.7557319223985893e-06, -1.858393274046472e-22},
    {-2.505210838544172e-08, 1.448814070935912e-24},
    {1.6059043836821613e-10, 1.2585294588752098e-26},
    {-7.647163731819816e-13, -7.03872877733453e-30},
    {2.8114572543455206e-15, 1.6508842730861433e-31},
    {-8.22063524662433e-18, -2.2141894119604265e-34},
    {1.9572941063391263e-20, -1.3643503830087908e-36},
    {-3.868170170630684e-23, 8.843177655482344e-40},
    {6.446950284384474e-26, -1.9330404233703465e-42},
    {-9.183689863795546e-29, -1.4303150396787322e-45},
    {1.1309962886447716e-31, 1.0498015412959506e-47}};
PCP_CR_CONST double kPcpCosC[15][2] = {
    {1.0, 0.0},
    {-0.5, 0.0},
    {0.041666666666666664, 2.3129646346357427e-18},
    {-0.001388888888888889, 5.300543954373577e-20},
    {2.48015873015873e-05, 2.1511947866775882e-23},
    {-2.755731922398589e-07, -2.3767714622250297e-23},
    {2.08767569878681e-09, -1.20734505911326e-25},
    {-1.1470745597729725e-11, -2.0655512752830745e-28},
    {4.779477332387385e-14, 4.399205485834081e-31},
    {-1.5619206968586225e-16, -1.1910679660273754e-32},
    {4.110317623312165e-19, 1.4412973378659527e-36},
    {-8.896791392450574e-22, 7.911402614872376e-38},
    {1.6117375710961184e-24, -3.6846573564509766e-41},
    {-2.4795962632247976e-27, 1.2953730964765229e-43},
    {3.279889237069838e-30, 1.5117542744029879e-46}};

/* sin and cos of a double-double m, |m| <= 4 (atan2's range and a little) */
PCP_CR void pcp_dd_sincos(pcp_dd m, pcp_dd *s_out, pcp_dd *c_out) {
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17,
                 P3 = -1.4973849048591698e-33;   /* pi / 2 = P1 + P2 + P3 */
    const double k = nearbyint(m.hi / P1);
    pcp_dd t = pcp_dd_add(m, pcp_dd_make(-k * P1, 0.0));   /* k * P1 exact for |k| <= 3 */
    t = pcp_dd_add(t, pcp_dd_neg(pcp_two_prod(k, P2)));
    t = pcp_dd_add(t, pcp_dd_make(-k * P3, 0.0));
    const pcp_dd t2 = pcp_dd_mul(t, t);
    /* Horner in t^2 over the tables (|t| <= pi / 4: the 15th terms are below 2^-108) */
    pcp_dd s = pcp_dd_make(kPcpSinC[14][0], kPcpSinC[14][1]);
    pcp_dd c = pcp_dd_make(kPcpCosC[14][0], kPcpCosC[14][1]);
#if defined(__HIPCC__)
#pragma unroll
#endif
    for (int j = 13; j >= 0; --j) {
        s = pcp_dd_add(pcp_dd_mul(s, t2), pcp_dd_make(kPcpSinC[j][0], kPcpSinC[j][1]));
        c = pcp_dd_add(pcp_dd_mul(c, t2), pcp_dd_make(kPcpCosC[j][0], kPcpCosC[j][1]));
    }
    s = pcp_dd_mul(s, t);
    const int q = ((int)k % 4 + 4) % 4;
    switch (q) {
    case 0: *s_out = s; *c_out = c; break;
    case 1: *s_out = c; *c_out = pcp_dd_neg(s); break;
    case 2: *s_out = pcp_dd_neg(s); *c_out = pcp_dd_neg(c); break;
    default: *s_out = pcp_dd_neg(c); *c_out = s; break;
    }
}

/* sign of y cos m - x sin m, i.e. of sin(atan2(y, x) - m) */
PCP_CR int pcp_cr_side(double y, double x, pcp_dd m) {
    pcp_dd s, c;
    pcp_dd_sincos(m, &s, &c);
    const pcp_dd e = pcp_dd_add(pcp_dd_mul_d(c, y), pcp_dd_neg(pcp_dd_mul_d(s, x)));
    const double v = e.hi != 0.0 ? e.hi : e.lo;
    return (v > 0.0) - (v < 0.0);
}

PCP_CR double pcp_cr_atan2_fix(double y, double x, double r) {
    if (!(isfinite(y) && isfinite(x) && isfinite(r)) || y == 0.0 || x == 0.0 || r == 0.0)
        return r;
    /* angles near the underflow range (|y / x| < 2^-900): the double-double terms underflow */
    if (fabs(r) < 0x1p-900) return r;
    const double lo = nextafter(r, -INFINITY), hi = nextafter(r, INFINITY);
    /* sin / cos at r once; at the midpoints m = r + h (h = half the exact gap to a neighbour)
     * sin m = S + h C - h^2 / 2 S, cos m = C - h S - h^2 / 2 C (the h^3 terms are ~2^-160) */
    pcp_dd S, C;
    pcp_dd_sincos(pcp_dd_make(r, 0.0), &S, &C);
    const pcp_dd yC = pcp_dd_mul_d(C, y), xS = pcp_dd_mul_d(S, x);
    const pcp_dd yS = pcp_dd_mul_d(S, y), xC = pcp_dd_mul_d(C, x);
    const pcp_dd e0 = pcp_dd_add(yC, pcp_dd_neg(xS));   /* y cos r - x sin r */
    const pcp_dd e1 = pcp_dd_add(yS, xC);               /* d/dh of -(y cos m - x sin m) */
    for (int side = 0; side < 2; ++side) {
        const double h = 0.5 * ((side ? hi : lo) - r);
        /* y cos m - x sin m = e0 - h e1 - h^2 / 2 e0 */
        pcp_dd e = pcp_dd_add(e0, pcp_dd_neg(pcp_dd_mul_d(e1, h)));
        e = pcp_dd_add(e, pcp_dd_make(-0.5 * h * h * e0.hi, 0.0));
        const double v = e.hi != 0.0 ? e.hi : e.lo;
        if (side == 0 && v < 0.0) return lo;
        if (side == 1 && v > 0.0) return hi;
    }
    return r;
}

#endif /* PCP_CRMATH_H */
