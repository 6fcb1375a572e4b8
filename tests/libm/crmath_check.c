/* crmath_check.c -- pcp_crmath.h against the running glibc (tests/test_crmath.py).
 * For N argument pairs: glibc's atan2 g, a first result r0 in {g's lower neighbour, g, g's
 * upper neighbour} (a faithful device result), and pcp_cr_atan2_fix(y, x, r0) must give g.
 * Half the pairs span the candidate generator's magnitudes (metres), a quarter tiny / huge
 * ratios, a quarter arbitrary finite bit patterns (those whose angle is below 2^-900 are
 * outside the fix's domain and skipped); then acos and sin the same way.  Prints one
 * "<fn> checked mismatches skipped" line per function. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pcp_crmath.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}
static double uni(double a, double b) { return a + (b - a) * ((rnd() >> 11) * 0x1.0p-53); }
static double bits(void) {
    for (;;) {
        uint64_t u = rnd();
        double d;
        memcpy(&d, &u, 8);
        if (isfinite(d) && d != 0.0) return d;
    }
}

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    long bad = 0, skipped = 0;
    for (long i = 0; i < n; ++i) {
        double y, x;
        const int kind = (int)(i & 3);
        if (kind < 2) {
            y = uni(-60.0, 60.0);
            x = uni(-60.0, 60.0);
        } else if (kind == 2) {
            y = uni(-1.0, 1.0) * ldexp(1.0, (int)(rnd() % 80) - 40);
            x = uni(-1.0, 1.0) * ldexp(1.0, (int)(rnd() % 80) - 40);
        } else {
            y = bits();
            x = bits();
        }
        const double g = atan2(y, x);
        if (fabs(g) < 0x1p-900) {   /* outside the fix's domain (it returns r0) */
            ++skipped;
            continue;
        }
        const int pick = (int)(rnd() % 3);
        const double r0 = pick == 0 ? nextafter(g, -INFINITY) : pick == 1 ? g : nextafter(g, INFINITY);
        const double r = pcp_cr_atan2_fix(y, x, r0);
        if (memcmp(&r, &g, 8) != 0) {
            if (bad < 5) fprintf(stderr, "y %a x %a glibc %a got %a (r0 %a)\n", y, x, g, r, r0);
            ++bad;
        }
    }
    printf("atan2 %ld %ld %ld\n", n - skipped, bad, skipped);
    /* acos over (0, 1) and sin over the scoring's pi / 2 - acos(..) in [0, pi / 2] */
    long bad_acos = 0, bad_sin = 0;
    for (long i = 0; i < n; ++i) {
        const double d = uni(0.0, 1.0);
        if (d == 0.0) continue;
        const double g = acos(d);
        const int pick = (int)(rnd() % 3);
        const double r0 = pick == 0 ? nextafter(g, -INFINITY) : pick == 1 ? g : nextafter(g, INFINITY);
        const double r = pcp_cr_acos_fix(d, r0);
        if (memcmp(&r, &g, 8) != 0) ++bad_acos;
        const double a = uni(0x1p-20, 1.5707963267948966);
        const double gs = sin(a), rs = pcp_cr_sin(a);
        if (memcmp(&rs, &gs, 8) != 0) ++bad_sin;
    }
    printf("acos %ld %ld 0\n", n, bad_acos);
    printf("sin %ld %ld 0\n", n, bad_sin);
    /* the scoring's composite (pcp_score_sin_part, round 6): against glibc's
     * sin(M_PI / 2 - acos(d)), and phase 1's decisions against phase 2's (the exact path) */
    long bad_spa = 0, disagree = 0, slow = 0;
    for (long i = 0; i < n; ++i) {
        const int kind = (int)(i % 4);
        const double d = kind == 0 ? uni(0x1p-20, 0.01) : kind == 3 ? uni(0.99, 1.0) : uni(0.0, 1.0);
        if (!(d > 0.0 && d < 1.0)) continue;
        const double ga = acos(d);
        const double g = sin(M_PI / 2 - ga);
        const int pick = (int)(rnd() % 3);
        const double r0 = pick == 0 ? nextafter(ga, -INFINITY) : pick == 2 ? nextafter(ga, INFINITY) : ga;
        int ph = 0;
        const double got = pcp_score_sin_part(d, r0, &ph);
        const double exact = pcp_cr_sin(1.5707963267948966 - pcp_cr_acos_fix(d, r0));
        if (memcmp(&got, &g, 8) != 0) ++bad_spa;
        if (memcmp(&got, &exact, 8) != 0) ++disagree;
        if (ph != 1) ++slow;
    }
    printf("spa %ld %ld %ld %ld\n", n, bad_spa, disagree, slow);
    return 0;
}
