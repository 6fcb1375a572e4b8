/* crmath_extra.h -- correctly rounded acos / sin built on pcp_crmath.h's double-double sin /
 * cos, for the CPU check only (tests/test_crmath.py via crmath_check.c).  Not product code: no
 * kernel calls them (glibc misrounds acos / sin near ties more often than ocml disagrees with
 * it, so correct rounding would move the scoring AWAY from the reference). */
#ifndef PCP_CRMATH_EXTRA_H
#define PCP_CRMATH_EXTRA_H

#include "pcp_crmath.h"

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

#endif /* PCP_CRMATH_EXTRA_H */
