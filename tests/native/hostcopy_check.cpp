// The split host copy (pointcloud_processor_amd/csrc/pcp_hostcopy.hip) on the CPU: every size
// around the split threshold, unaligned sources, bytes past the end untouched, 1,200 jobs through
// the helper threads; prints the copy time of a 60k-point scan with and without the helpers.
// Built host-only by hipcc (no GPU call): tests/test_hostcopy.py.
#include <cstdio>
#include <cstring>
#include <vector>
#include <chrono>
#include "pcp_internal.hpp"
int main() {
    pcp_ctx *ctx = new pcp_ctx();
    std::vector<char> a(4 << 20), b(4 << 20);
    for (size_t i = 0; i < a.size(); ++i) a[i] = (char)(i * 131 + 7);
    size_t sizes[] = {1000, 262144, 262145, 960512, 3 * 1024 * 1024 + 17, 4 << 20};
    for (int rep = 0; rep < 200; ++rep)
        for (size_t n : sizes) {
            std::memset(b.data(), 0, b.size());
            pcp::host_copy(ctx, b.data(), a.data() + (rep % 7), n);
            if (std::memcmp(b.data(), a.data() + (rep % 7), n) != 0 || b[n] != 0) { std::printf("FAIL %zu\n", n); return 1; }
        }
    for (int t : {0, 3}) {
        ctx->copy_threads = t;
        auto t0 = std::chrono::steady_clock::now();
        for (int rep = 0; rep < 500; ++rep) pcp::host_copy(ctx, b.data(), a.data(), 960512);
        double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 500;
        std::printf("threads %d: %.1f us per 960 KB copy\n", t, us);
    }
    pcp::host_copy_release(ctx);
    std::printf("ok\n");
}
