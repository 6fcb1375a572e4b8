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
 * The scoring's acos and sin (evaluateCellScore, virtual_lidar.cpp:689-700) the same way
 * (round 6): pcp_cr_acos_fix(d, r) from ocml's acos, pcp_cr_sin(a) from the double-double sin.
 * Measured per cell (tests/test_gpu_parity.py::test_parity_bar_per_cell, 91-candidate tick):
 * ocml's acos / sin made 9 % of the positive cell scores differ from glibc's (up to 8 ulps where
 * pi / 2 - theta is small, 2:1 downward); glibc rounds these correctly but for rare near ties.
 * Compile with -ffp-contract=off: the error-free transformations need every operation rounded
 * on its own (fma() is called explicitly where one is meant).
 */
#ifndef PCP_CRMATH_H
#define PCP_CRMATH_H

#include <math.h>
#include <string.h>

#if defined(__HIPCC__)
#define PCP_CR static __host__ __device__ __forceinline__
#define PCP_CR_COLD static __host__ __device__ __attribute__((noinline))
#else
#define PCP_CR static inline
#define PCP_CR_COLD static __attribute__((noinline))
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

/* acos(d) for 0 < d < 1 from a faithful first result r: acos is decreasing, so the true angle
 * lies below the midpoint m = r + h (h = half the gap to a neighbour) exactly when d > cos m,
 * with cos m = C - h S - h^2 / 2 C from ONE double-double sin / cos at r (the h^3 terms are
 * ~2^-160).  Other d (0, 1, outside, NaN) and r = 0 return r unchanged. */
PCP_CR double pcp_cr_acos_fix(double d, double r) {
    if (!(d > 0.0 && d < 1.0) || !isfinite(r) || r == 0.0) return r;
    const double lo = nextafter(r, -INFINITY), hi = nextafter(r, INFINITY);
    pcp_dd S, C;
    pcp_dd_sincos(pcp_dd_make(r, 0.0), &S, &C);
    for (int side = 0; side < 2; ++side) {
        const double h = 0.5 * ((side ? hi : lo) - r);
        pcp_dd cm = pcp_dd_add(C, pcp_dd_neg(pcp_dd_mul_d(S, h)));
        cm = pcp_dd_add(cm, pcp_dd_make(-0.5 * h * h * C.hi, 0.0));
        const pcp_dd e = pcp_dd_add(pcp_dd_make(d, 0.0), pcp_dd_neg(cm));   /* d - cos m */
        const double v = e.hi != 0.0 ? e.hi : e.lo;
        if (side == 0 && v > 0.0) return lo;
        if (side == 1 && v < 0.0) return hi;
    }
    return r;
}

/* sin(a) for 2^-500 <= |a| <= 4: the double-double value rounded once (its normalised high
 * part) -- correct unless sin(a) lies within ~2^-100 relative of a midpoint; other a: sin(a) */
PCP_CR double pcp_cr_sin(double a) {
    if (!isfinite(a) || fabs(a) > 4.0 || fabs(a) < 0x1p-500) return sin(a);
    pcp_dd s, c;
    pcp_dd_sincos(pcp_dd_make(a, 0.0), &s, &c);
    return s.hi + s.lo;
}

/* ---- the scoring's sin(pi / 2 - acos(d)) at speed (round 6) -------------------------------
 * A two-phase (Ziv) evaluation.  Phase 1: sin / cos from the table of k pi / 512
 * (pcp_crmath_tab.h, tools/gen/crmath_table.py) and short polynomials in |t| <= pi / 1024, good
 * to ~2^-70 absolute; each rounding decision is taken only when the value lies more than
 * PCP_CR_FAST_MARGIN from the decision's boundary, else phase 2 (pcp_cr_acos_fix +
 * pcp_cr_sin above, ~2^-100) decides.  tests/test_crmath.py checks phase 1's decisions against
 * phase 2 and the result against glibc's sin(M_PI / 2 - acos(d)). */
#include "pcp_crmath_tab.h"

/* phase 1's decision margins: absolute for d - cos m (values <= 1), relative for a rounding */
#define PCP_CR_FAST_MARGIN 0x1p-74
#define PCP_CR_FAST_MARGIN_REL 0x1p-66

/* sin / cos of 0 <= x <= 1.61 as double-doubles, |error| below ~2^-84 (absolute; relative for
 * sin of x < pi / 1024): the table's k pi / 512, t = x - k pi / 512 in double-double,
 * sin t = t + t^3 (-1/6 + t^2/120 - t^4/5040), cos t = 1 - u / 2 + u^2 / 24 - u^3 / 720 with
 * u = t^2 in double-double (the terms past those are below 2^-90 for |t| <= pi / 1024) */
PCP_CR void pcp_fast_sincos(double x, pcp_dd *s_out, pcp_dd *c_out) {
    int k = (int)nearbyint(x * (512.0 / 3.141592653589793));
    k = k < 0 ? 0 : (k > PCP_CR_TAB_N - 1 ? PCP_CR_TAB_N - 1 : k);
    const double kd = (double)k;
    /* t = x - k (Q1 + Q2 + Q3): k Q1, k Q2 exact; x - k Q1 exact (Sterbenz) */
    const double t1 = x - kd * PCP_CR_Q1;
    const pcp_dd t2 = pcp_two_sum(t1, -(kd * PCP_CR_Q2));
    const pcp_dd t = pcp_fast_two_sum(t2.hi, t2.lo - kd * PCP_CR_Q3);
    const pcp_dd u2 = pcp_two_prod(t.hi, t.hi);
    const pcp_dd u = pcp_fast_two_sum(u2.hi, u2.lo + 2.0 * t.hi * t.lo);   /* t^2 */
    const double ud = u.hi;
    /* sin t = t + st, st = t^3 (-1/6 + ...) (|st| < 2^-27 |t|: double suffices) */
    const double st = t.hi * ud * (-1.0 / 6.0 + ud * (1.0 / 120.0 + ud * (-1.0 / 5040.0)));
    /* cos t = 1 + ct, ct = -u / 2 (double-double) + u^2 (1/24 - u / 720) */
    const pcp_dd ct = pcp_dd_add(pcp_dd_make(-0.5 * u.hi, -0.5 * u.lo),
                                 pcp_dd_make(ud * ud * (1.0 / 24.0 + ud * (-1.0 / 720.0)), 0.0));
    const pcp_dd sint = pcp_dd_add(t, pcp_dd_make(st, 0.0));
    const pcp_dd Sk = pcp_dd_make(kPcpSinCos512[k][0], kPcpSinCos512[k][1]);
    const pcp_dd Ck = pcp_dd_make(kPcpSinCos512[k][2], kPcpSinCos512[k][3]);
    /* sin x = Sk + Sk ct + Ck sin t, cos x = Ck + Ck ct - Sk sin t */
    *s_out = pcp_dd_add(pcp_dd_add(Sk, pcp_dd_mul(Sk, ct)), pcp_dd_mul(Ck, sint));
    *c_out = pcp_dd_add(pcp_dd_add(Ck, pcp_dd_mul(Ck, ct)), pcp_dd_neg(pcp_dd_mul(Sk, sint)));
}

/* neighbours of a positive finite double (bit steps; no call into libm) */
PCP_CR double pcp_next_up(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double(__double_as_longlong(x) + 1);
#else
    long long b;
    memcpy(&b, &x, 8);
    ++b;
    memcpy(&x, &b, 8);
    return x;
#endif
}
PCP_CR double pcp_next_down(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __longlong_as_double(__double_as_longlong(x) - 1);
#else
    long long b;
    memcpy(&b, &x, 8);
    --b;
    memcpy(&x, &b, 8);
    return x;
#endif
}

/* the double nearest v = hi + lo (v > 0, lo normalised below hi's ulp), if v lies more than
 * margin * v from a rounding boundary: *ok = 1; else *ok = 0 */
PCP_CR double pcp_round_dd_checked(pcp_dd v, double margin, int *ok) {
    const double R = v.hi + v.lo;
    const double res = (v.hi - R) + v.lo;   /* v - R */
    const double half = 0.5 * (res > 0.0 ? pcp_next_up(R) - R : R - pcp_next_down(R));
    *ok = fabs(fabs(res) - half) > margin * R;
    return R;
}

/* phase 2 (rare: one call, kept out of line so that its registers do not weigh on the fast
 * path's occupancy) */
PCP_CR_COLD double pcp_score_sin_part_exact(double d, double r) {
    return pcp_cr_sin(1.5707963267948966 - pcp_cr_acos_fix(d, r));
}

/* evaluateCellScore's sin(M_PI / 2 - theta), theta = acos(d), as glibc evaluates it (both
 * functions rounded correctly), from a faithful first result r of acos(d).  phase_out
 * (nullable): 1 when phase 1 decided, 2 when phase 2 did.  Straight-line: every lane of a
 * wave runs the same instructions but for the rare phase 2. */
PCP_CR double pcp_score_sin_part(double d, double r, int *phase_out) {
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17;   /* pi / 2 = P1 + P2 + ~1e-33 */
    if (phase_out) *phase_out = 2;
    if (!(d > 0x1p-20 && d < 1.0) || !(r > 0.0 && r < 1.6)) return pcp_score_sin_part_exact(d, r);
    pcp_dd S, C;
    pcp_fast_sincos(r, &S, &C);
    /* d - cos(r + h) at both midpoints, cos(r + h) = C - S h - C h^2 / 2: d - C.hi is exact
     * (Sterbenz: d ~ cos r), and the terms in h (|h| < 2^-53) are exact to ~2^-106 in double */
    const double lo = pcp_next_down(r), hi = pcp_next_up(r);
    const double hl = 0.5 * (lo - r), hh = 0.5 * (hi - r);
    const double dCh = d - C.hi;
    const double el = dCh + (S.hi * hl + (0.5 * hl * hl * C.hi - C.lo));
    const double eh = dCh + (S.hi * hh + (0.5 * hh * hh * C.hi - C.lo));
    if (fabs(el) <= PCP_CR_FAST_MARGIN || fabs(eh) <= PCP_CR_FAST_MARGIN)
        return pcp_score_sin_part_exact(d, r);
    /* acos decreases: d above cos(lower midpoint) -> lo; below cos(upper midpoint) -> hi */
    const double th = el > 0.0 ? lo : (eh < 0.0 ? hi : r);
    /* a = P1 - th rounded: P1 - th = a + e exactly, pi / 2 = P1 + P2 + P3, so
     * a = pi / 2 - (th + e + P2 + P3) and sin(a) = cos(r + delta), delta = (th - r) + e + P2
     * (|delta| < 2^-51; P3 and S.lo delta are below 2^-104): cos(r + delta) = C - S delta -
     * C delta^2 / 2.  C's absolute error (~2^-84) is relative to sin(a) ~ a: below a = 2^-8,
     * sin(a) = a + a^3 (-1/6 + a^2/120 - a^4/5040) directly (a exact; the correction's error
     * is below 2^-71 of a, the a^9 term below 2^-90) */
    const pcp_dd ea = pcp_two_sum(P1, -th);
    const double a = ea.hi;
    pcp_dd v;
    if (a < 0x1p-8) {
        const double u = a * a;
        v = pcp_fast_two_sum(a, a * u * (-1.0 / 6.0 + u * (1.0 / 120.0 + u * (-1.0 / 5040.0))));
    } else {
        const double delta = (th - r) + (ea.lo + P2);
        v = pcp_fast_two_sum(C.hi, C.lo - (S.hi * delta + 0.5 * C.hi * delta * delta));
    }
    int ok = 0;
    const double R = pcp_round_dd_checked(v, PCP_CR_FAST_MARGIN_REL, &ok);
    if (!ok) return pcp_score_sin_part_exact(d, r);
    if (phase_out) *phase_out = 1;
    return R;
}

#endif /* PCP_CRMATH_H */
