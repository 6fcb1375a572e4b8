// FETCH_SIZE calibration for divergent gathers on gfx950 (profiles/r04_fetch_calibration.json):
// a table of T bytes is read once per launch, every 128-byte line exactly once, in one of these
// shapes (kernel names carry the shape, so rocprofv3's per-dispatch FETCH_SIZE rows separate):
//   k_stream16   lane i reads 16 B at 16 i (coalesced streaming: the guide's calibrated case)
//   k_gather<W>  lane i reads W bytes (W = 2, 4, 12, 16) at the start of line perm(i): every lane
//                of a wave on its own line, the lines in a scrambled order (the fan's probes,
//                walk starts and point records are W = 2, 4, 12)
// Known quantity: lines touched = T / 128 per launch.  Run once plain (launch times, printed as
// JSON lines) and once per counter under rocprofv3 --pmc FETCH_SIZE; tools/gather_cal.py joins
// them.  Two table sizes: 64 MiB (Infinity-Cache resident after the first launch, the fan's
// regime: its ~170 MB copy stays resident) and 2 GiB (HBM).
//   hipcc --offload-arch=gfx950 -O3 -o gather_fetch gather_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

__global__ void __launch_bounds__(256) k_stream16(const uint4 *__restrict__ t, unsigned long long n16,
                                                  unsigned *__restrict__ out) {
    unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x;
    unsigned s = 0;
    for (; i < n16; i += (unsigned long long)gridDim.x * 256) {
        const uint4 v = t[i];
        s += v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345678u) out[0] = s;   // practically never true: no stores
}

template <int W>
__global__ void __launch_bounds__(256) k_gather(const unsigned char *__restrict__ t,
                                                unsigned long long nlines,
                                                unsigned *__restrict__ out) {
    const unsigned long long mask = nlines - 1;
    unsigned s = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < nlines;
         i += (unsigned long long)gridDim.x * 256) {
        // a bijection of [0, nlines): odd multiplier, low bits
        const unsigned long long line = (i * 0x9E3779B97F4A7C15ull) & mask;
        const unsigned char *p = t + (line << 7);
        if constexpr (W == 2) {
            s += *reinterpret_cast<const unsigned short *>(p);
        } else if constexpr (W == 4) {
            s += *reinterpret_cast<const unsigned *>(p);
        } else if constexpr (W == 12) {
            const float *f = reinterpret_cast<const float *>(p);
            s += __float_as_uint(f[0]) ^ __float_as_uint(f[1]) ^ __float_as_uint(f[2]);
        } else {
            const uint4 v = *reinterpret_cast<const uint4 *>(p);
            s += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (s == 0x12345678u) out[0] = s;
}

template <class F>
static float time_ms(F launch, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();   // warm (and fills the Infinity Cache for a resident table)
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
    const unsigned long long sizes[2] = {64ull << 20, 2ull << 30};
    unsigned *out;
    CK(hipMalloc(&out, 64));
    for (unsigned long long T : sizes) {
        unsigned char *t;
        CK(hipMalloc(&t, T));
        CK(hipMemset(t, 0x5A, T));   // non-zero bytes (no compressible pattern assumed)
        const unsigned long long nlines = T >> 7;
        const unsigned grid = 256 * 64;   // 64 blocks per CU, grid-stride
        auto report = [&](const char *name, int w, float ms) {
            std::printf("{\"kernel\": \"%s\", \"lane_bytes\": %d, \"table_bytes\": %llu, "
                        "\"lines\": %llu, \"ms\": %.6f, \"lines_per_s\": %.6e}\n",
                        name, w, T, nlines, ms, nlines / (ms * 1e-3));
            std::fflush(stdout);
        };
        report("k_stream16", 16, time_ms([&] {
                   hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(256), 0, 0,
                                      (const uint4 *)t, T / 16, out);
               }, reps));
        report("k_gather<2>", 2, time_ms([&] {
                   hipLaunchKernelGGL(k_gather<2>, dim3(grid), dim3(256), 0, 0, t, nlines, out);
               }, reps));
        report("k_gather<4>", 4, time_ms([&] {
                   hipLaunchKernelGGL(k_gather<4>, dim3(grid), dim3(256), 0, 0, t, nlines, out);
               }, reps));
        report("k_gather<12>", 12, time_ms([&] {
                   hipLaunchKernelGGL(k_gather<12>, dim3(grid), dim3(256), 0, 0, t, nlines, out);
               }, reps));
        report("k_gather<16>", 16, time_ms([&] {
                   hipLaunchKernelGGL(k_gather<16>, dim3(grid), dim3(256), 0, 0, t, nlines, out);
               }, reps));
        CK(hipDeviceSynchronize());
        CK(hipFree(t));
    }
    CK(hipFree(out));
    return 0;
}
