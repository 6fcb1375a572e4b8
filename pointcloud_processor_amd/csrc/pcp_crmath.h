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
 * pcp_cr_acos_fix(d, r) and pcp_cr_sin(a): the same for the scoring's acos and sin
 * (virtual_lidar.cpp:700-705); checked on the CPU and not used by a kernel: glibc misrounds
 * those near ties more often than ocml disagrees with it.
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

/* sin and cos of a double-double m, |m| <= 4 (atan2's range and a little) */
PCP_CR void pcp_dd_sincos(pcp_dd m, pcp_dd *s_out, pcp_dd *c_out) {
    const double P1 = 1.5707963267948966, P2 = 6.123233995736766e-17,
                 P3 = -1.4973849048591698e-33;   /* pi / 2 = P1 + P2 + P3 */
    const double k = nearbyint(m.hi / P1);
    pcp_dd t = pcp_dd_add(m, pcp_dd_make(-k * P1, 0.0));   /* k * P1 exact for |k| <= 3 */
    t = pcp_dd_add(t, pcp_dd_neg(pcp_two_prod(k, P2)));
    t = pcp_dd_add(t, pcp_dd_make(-k * P3, 0.0));
    const pcp_dd t2 = pcp_dd_mul(t, t);
    /* sin t = t (1 - t^2/(2 3) (1 - t^2/(4 5) (...))), cos t = 1 - t^2/(1 2) (1 - ...) */
    pcp_dd s = pcp_dd_make(1.0, 0.0), c = pcp_dd_make(1.0, 0.0);
    for (int j = 15; j >= 1; --j) {
        s = pcp_dd_add(pcp_dd_make(1.0, 0.0),
                       pcp_dd_neg(pcp_dd_div_d(pcp_dd_mul(t2, s), (double)((2 * j) * (2 * j + 1)))));
        c = pcp_dd_add(pcp_dd_make(1.0, 0.0),
                       pcp_dd_neg(pcp_dd_div_d(pcp_dd_mul(t2, c), (double)((2 * j - 1) * (2 * j)))));
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
    /* the midpoints as double-doubles: r and half the (exact) gap to each neighbour */
    if (pcp_cr_side(y, x, pcp_fast_two_sum(r, 0.5 * (lo - r))) < 0) return lo;
    if (pcp_cr_side(y, x, pcp_fast_two_sum(r, 0.5 * (hi - r))) > 0) return hi;
    return r;
}

/* acos(d) for 0 < d < 1 from a faithful first result r: acos is decreasing, so the true angle
 * lies below the midpoint m exactly when d > cos m (cos m in double-double) */
PCP_CR double pcp_cr_acos_fix(double d, double r) {
    if (!(d > 0.0 && d < 1.0) || !isfinite(r) || r == 0.0) return r;
    const double lo = nextafter(r, -INFINITY), hi = nextafter(r, INFINITY);
    pcp_dd s, c;
    pcp_dd_sincos(pcp_fast_two_sum(r, 0.5 * (lo - r)), &s, &c);
    if (pcp_dd_add(pcp_dd_make(d, 0.0), pcp_dd_neg(c)).hi > 0.0) return lo;
    pcp_dd_sincos(pcp_fast_two_sum(r, 0.5 * (hi - r)), &s, &c);
    if (pcp_dd_add(pcp_dd_make(d, 0.0), pcp_dd_neg(c)).hi < 0.0) return hi;
    return r;
}

/* sin(a) for |a| <= 4, a >= 2^-500: the double-double value rounded once (its normalised high
 * part) -- correct unless sin(a) lies within ~2^-100 relative of a midpoint */
PCP_CR double pcp_cr_sin(double a) {
    if (!isfinite(a) || fabs(a) > 4.0 || fabs(a) < 0x1p-500) return sin(a);
    pcp_dd s, c;
    pcp_dd_sincos(pcp_dd_make(a, 0.0), &s, &c);
    return s.hi + s.lo;
}

#endif /* PCP_CRMATH_H */
