// Dependent f64 add latency on gfx950 (the row-sum chain floor, pcp_vlidar.hip row_group_body).
// hipcc --offload-arch=gfx950 -O3 -o chain chain.hip; measured: ~6 clocks per dependent
// v_add_f64, 2.6 ns wall per add on one wave with 4 or 16 active lanes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
// dependent f64 add chain latency: one wave, N adds, operands in VGPRs
__global__ void k_chain(const double* in, double* out, long long* cyc, int iters) {
    double v[32];
    for (int i = 0; i < 32; ++i) v[i] = in[threadIdx.x * 32 + i];
    double acc = 0.0;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) acc += v[i];
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
// two interleaved independent chains (issue-bound check)
__global__ void k_chain2(const double* in, double* out, long long* cyc, int iters) {
    double v[32];
    for (int i = 0; i < 32; ++i) v[i] = in[threadIdx.x * 32 + i];
    double a = 0.0, b = 1.0;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) { a += v[i]; b += v[31 - i]; }
    }
    long long t1 = clock64();
    out[threadIdx.x] = a + b;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
int main(int argc, char **argv) {
    // argv[1]: iterations of 32 adds (default 20000: the launch is < 1 % of the interval)
    double *in, *out; long long* cyc;
    hipMalloc(&in, 64 * 32 * 8); hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
    hipMemset(in, 0, 64 * 32 * 8);
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    double ns64 = 0.0, tk64 = 0.0;
    for (int lanes : {64, 16, 4}) {
        for (int k = 0; k < 2; ++k) {
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(k_chain, dim3(1), dim3(lanes), 0, 0, in, out, cyc, iters);
            else hipLaunchKernelGGL(k_chain2, dim3(1), dim3(lanes), 0, 0, in, out, cyc, iters);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            const double n = 32.0 * iters * (k ? 2 : 1);
            const double ns = ms * 1e6 / (32.0 * iters);
            printf("lanes %d chains %d: %.2f clock64 ticks/add, wall %.3f ms = %.3f ns per dependent add\n",
                   lanes, k + 1, c / n, ms, ns);
            if (lanes == 64 && k == 0) { ns64 = ns; tk64 = c / n; }
        }
    }
    // the row-sum chain floor of k_sum_flags (one lane per row: C dependent adds per row)
    printf("{\"ns_per_dependent_f64_add\": %.4f, \"clock64_ticks_per_add\": %.3f, \"iters\": %d, "
           "\"wave_lanes\": 64}\n", ns64, tk64, iters);
    return 0;
}
