// Cost of the scoring's sin(pi/2 - acos(d)) on gfx950: ocml's functions vs pcp_score_sin_part
// (two-phase correctly rounded) vs the exact path alone, one lane per argument, N arguments.
// hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../pointcloud_processor_amd/csrc -o cr_mb cr_mb.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "pcp_crmath.h"

template <int MODE>
__global__ void k(const double *in, double *out, int n, int *phase2) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double d = in[i];
    double v;
    if (MODE == 0) v = sin(1.5707963267948966 - acos(d));
    else if (MODE == 1) {
        int ph = 1;
        v = pcp_score_sin_part(d, acos(d), &ph);
        if (ph != 1) atomicAdd(phase2, 1);
    } else if (MODE == 2) v = pcp_cr_sin(1.5707963267948966 - pcp_cr_acos_fix(d, acos(d)));
    else if (MODE == 3) {   // the table-driven sin / cos alone
        pcp_dd S, C;
        pcp_fast_sincos(acos(d), &S, &C);
        v = S.hi + C.lo;
    } else if (MODE == 4) {   // acos + 4 nextafter
        const double r = acos(d);
        v = nextafter(r, 1e9) + nextafter(r, -1e9) + nextafter(d, 1e9) + nextafter(d, -1e9);
    } else {   // the double-double sin / cos (Taylor to t^31)
        pcp_dd S, C;
        pcp_dd_sincos(pcp_dd_make(acos(d), 0.0), &S, &C);
        v = S.hi + C.lo;
    }
    out[i] = v;
}

int main() {
    const int n = 1 << 20;
    std::vector<double> h(n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = (double)(s >> 11) * 0x1.0p-53;
    }
    double *in, *out; int *p2;
    hipMalloc(&in, n * 8); hipMalloc(&out, n * 8); hipMalloc(&p2, 4);
    hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice);
    hipMemset(p2, 0, 4);
    const char *names[6] = {"ocml sin(pi/2 - acos)", "pcp_score_sin_part", "exact path only", "fast sincos + acos", "acos + 4 nextafter", "dd sincos (Taylor) + acos"};
    for (int mode = 0; mode < 6; ++mode) {
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            for (int r = 0; r < 10; ++r) {
                if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
                if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
                if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
                if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
                if (mode == 4) hipLaunchKernelGGL(k<4>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
                if (mode == 5) hipLaunchKernelGGL(k<5>, dim3(n / 256), dim3(256), 0, 0, in, out, n, p2);
            }
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b);
            if (rep) printf("%-24s %.3f us per launch of %d (%.2f ns per argument)\n", names[mode], ms * 100.0, n, ms * 1e5 / n);
        }
    }
    int ph2 = 0; hipMemcpy(&ph2, p2, 4, hipMemcpyDeviceToHost);
    printf("phase-2 arguments (20 launches of pcp_score_sin_part): %d of %d\n", ph2, 20 * n);
    return 0;
}
