// Ceiling of divergent lane-loads on gfx950 -- the bound the fan kernel's roofline is quoted
// against (bench.py _fan_roofline; profiles/r05_gather_ceiling.json via tools/gather_ceiling.sh).
//
// The fan kernel (pcp_vlidar.hip k_raycast_fan_xcd) is one wave per workgroup, 8 waves per SIMD,
// and every lane of its probe / walk-start / point-record loads reads its own cache line: 2-byte
// z-band thresholds, 4-byte walk starts, 12-byte (x, y, z) window entries, each lane's next
// address depending on what it loaded before (a probe decides the walk, a walk entry the next).
// This kernel reproduces that shape and nothing else:
//   * one 64-lane wave per workgroup, 8 waves per SIMD (256 CUs x 4 SIMDs x 8 = 8,192 resident),
//     a grid of 4 such rounds;
//   * each lane runs C independent dependent chains (C = 1, 2, 4: loads in flight per lane);
//     step k of a chain loads W bytes (W = 2, 4, 12: one ushort, one uint, three floats) at the
//     start of a pseudo-random 128-byte line whose index is a hash of the chain's previous value
//     (tables of >= 16,384 lines: every lane of a wave on its own line; the L1-sized ones below
//     share lines the way the fan's loads do), the load's data feeding the next address like
//     the fan's walks;
//   * tables of 8 KiB and 16 KiB (L1-resident: random lines shared by ~1.6 / ~1.3 lanes of a
//     64-lane load -- the fan's loads measure 1.57 lanes per L1 tag and hit L1 82 % of the time,
//     profiles/r05_fan_gather_path.json), 2 MiB (L2-resident in every XCD: every lane its own
//     line, an L1 miss each), 16 MiB and 96 MiB (the fan's fine-window copy: Infinity-Cache
//     resident), filled with random bits;
//   * A active lanes per wave (64, or 24: the fan's loads average 24 active lanes per
//     instruction -- its walks diverge), the others idle for the whole launch.
// Lane-loads per launch = waves x A x C x steps (exact: no lane exits early).  Time = HIP events
// around `reps` back-to-back launches after a warm-up launch.  The clock the chip held under the
// load: lane 0 of every wave reads clock64() (shader clock) and wall_clock64() (the constant
// real-time counter, hipDeviceAttributeWallClockRate kHz) at its start and end; the median of
// dclock / dwall over the waves is the shader clock in MHz.  Per CU and cycle =
// lane-loads/s / 256 / clock.
//   hipcc --offload-arch=gfx950 -O3 -o gather_ceiling gather_ceiling.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

constexpr int kSteps = 256;   // dependent loads per chain and launch

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int W>
__device__ __forceinline__ uint32_t load_w(const unsigned char *__restrict__ t, uint32_t line) {
    const unsigned char *p = t + ((size_t)line << 7);
    if constexpr (W == 2) {
        return *reinterpret_cast<const unsigned short *>(p);
    } else if constexpr (W == 4) {
        return *reinterpret_cast<const uint32_t *>(p);
    } else {
        const float *f = reinterpret_cast<const float *>(p);
        return __float_as_uint(f[0]) ^ __float_as_uint(f[1]) ^ __float_as_uint(f[2]);
    }
}

template <int W, int C>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_gather_chain(const unsigned char *__restrict__ t, uint32_t line_mask, uint32_t active,
               unsigned long long *__restrict__ clk, uint32_t *__restrict__ sink) {
    const uint64_t c0 = clock64(), w0 = wall_clock64();
    uint32_t s = 0;
    if (threadIdx.x < active) {
        uint32_t x[C];
#pragma unroll
        for (int c = 0; c < C; ++c) x[c] = mix(blockIdx.x * 64u + threadIdx.x + 0x9e3779b9u * (c + 1));
        for (int k = 0; k < kSteps; ++k) {
            uint32_t v[C];
#pragma unroll
            for (int c = 0; c < C; ++c) v[c] = load_w<W>(t, x[c] & line_mask);
#pragma unroll
            for (int c = 0; c < C; ++c) x[c] = mix(x[c] + v[c]);
        }
#pragma unroll
        for (int c = 0; c < C; ++c) s ^= x[c];
    }
    const uint64_t c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = w1 - w0;
    }
    if (s == 0x12345678u) sink[0] = s;   // practically never: keeps the chains live
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 10;
    int dev = 0, ncu = 0, wall_khz = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, dev));
    const unsigned waves = (unsigned)ncu * 4 * 8 * 4;   // 4 rounds of 8 waves per SIMD
    const size_t sizes[5] = {8u << 10, 16u << 10, 2u << 20, 16u << 20, 96u << 20};
    unsigned long long *clk;
    uint32_t *sink;
    CK(hipMalloc(&clk, (size_t)waves * 16));
    CK(hipMalloc(&sink, 64));
    std::vector<unsigned long long> hclk((size_t)waves * 2);
    for (size_t T : sizes) {
        unsigned char *t;
        CK(hipMalloc(&t, T));
        {
            std::vector<uint32_t> h(T / 4);
            uint64_t s = 0x243f6a8885a308d3ull;
            for (auto &v : h) {
                s = s * 6364136223846793005ull + 1442695040888963407ull;
                v = (uint32_t)(s >> 32);
            }
            CK(hipMemcpy(t, h.data(), T, hipMemcpyHostToDevice));
        }
        const uint32_t mask = (uint32_t)(T >> 7) - 1;   // power-of-two line counts
        auto run = [&](const char *name, int w, int c, uint32_t act, auto kern) {
            auto launch = [&] {
                hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, t, mask, act, clk, sink);
            };
            launch();   // warm: caches filled, clocks up
            CK(hipDeviceSynchronize());
            hipEvent_t a, b;
            CK(hipEventCreate(&a));
            CK(hipEventCreate(&b));
            CK(hipEventRecord(a));
            for (int r = 0; r < reps; ++r) launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            CK(hipEventDestroy(a));
            CK(hipEventDestroy(b));
            ms /= reps;
            CK(hipMemcpy(hclk.data(), clk, hclk.size() * 8, hipMemcpyDeviceToHost));
            std::vector<double> f;
            f.reserve(waves);
            for (unsigned i = 0; i < waves; ++i)
                if (hclk[2 * i + 1]) f.push_back((double)hclk[2 * i] / hclk[2 * i + 1] * wall_khz * 1e-3);
            std::sort(f.begin(), f.end());
            const double mhz = f.empty() ? 0.0 : f[f.size() / 2];
            const double lanes = (double)waves * act * c * kSteps;
            const double rate = lanes / (ms * 1e-3);
            std::printf("{\"kernel\": \"%s\", \"lane_bytes\": %d, \"chains_per_lane\": %d, "
                        "\"active_lanes\": %u, \"table_bytes\": %zu, \"waves\": %u, \"cus\": %d, "
                        "\"lane_loads\": %.0f, \"ms\": %.6f, \"lane_loads_per_s\": %.6e, "
                        "\"clock_mhz\": %.1f, \"per_cu_per_cycle\": %.4f}\n",
                        name, w, c, act, T, waves, ncu, lanes, ms, rate, mhz,
                        mhz > 0 ? rate / ncu / (mhz * 1e6) : 0.0);
            std::fflush(stdout);
        };
        for (uint32_t act : {64u, 24u}) {
            run("k_gather_chain<2,1>", 2, 1, act, k_gather_chain<2, 1>);
            run("k_gather_chain<2,4>", 2, 4, act, k_gather_chain<2, 4>);
            run("k_gather_chain<4,1>", 4, 1, act, k_gather_chain<4, 1>);
            run("k_gather_chain<4,4>", 4, 4, act, k_gather_chain<4, 4>);
            run("k_gather_chain<12,1>", 12, 1, act, k_gather_chain<12, 1>);
            run("k_gather_chain<12,4>", 12, 4, act, k_gather_chain<12, 4>);
        }
        CK(hipFree(t));
    }
    CK(hipFree(clk));
    CK(hipFree(sink));
    return 0;
}
