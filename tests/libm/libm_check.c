/* Checks pointcloud_processor_amd/csrc/pcp_libm.h (the GPU's restatement of glibc's float
 * atan2f / sinf / cosf, used by the exact PCA normals) against the glibc it runs on, bit for bit.
 * usage: libm_check STRIDE N_ATAN2  -> prints "sin_cos n mism_sin mism_cos\natan2 n mism\n" */
#include <stdio.h>
#include <stdlib.h>

#include "pcp_libm.h"

int main(int argc, char **argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 10) : 1;
    const long n_at = argc > 2 ? strtol(argv[2], 0, 10) : 1000000;
    long n = 0, ms = 0, mc = 0;
    /* every stride-th float of [0, 1.1]: computeRoots' angle lies in [0, pi / 3] */
    const uint32_t hi = pcp_lm_asu(1.1f);
    for (uint32_t u = 0; u <= hi; u += stride) {
        const float t = pcp_lm_asf(u);
        ms += pcp_lm_asu(pcp_sinf(t)) != pcp_lm_asu(sinf(t));
        mc += pcp_lm_asu(pcp_cosf(t)) != pcp_lm_asu(cosf(t));
        ++n;
    }
    printf("sin_cos %ld %ld %ld\n", n, ms, mc);
    long ma = 0;
    uint64_t s = 88172645463325252ull;
    for (long i = 0; i < n_at; ++i) {
        float y, x;
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        if (i & 1) { /* any bit pattern (NaN, inf, subnormal, zero included) */
            y = pcp_lm_asf((uint32_t)s);
            x = pcp_lm_asf((uint32_t)(s >> 32));
        } else { /* the magnitudes computeRoots feeds it: sqrt(-q), half_b */
            y = ldexpf((float)(s & 0xffffff) / 16777216.0f, (int)((s >> 24) % 48) - 36);
            x = ldexpf((float)((s >> 32) & 0xffffff) / 16777216.0f - 0.5f, (int)((s >> 56) % 48) - 36);
        }
        const float a = pcp_atan2f(y, x), b = atan2f(y, x);
        if (pcp_lm_asu(a) != pcp_lm_asu(b) && !(a != a && b != b)) ++ma;
    }
    printf("atan2 %ld %ld\n", n_at, ma);
    return 0;
}
