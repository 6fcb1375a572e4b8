// pcp_hostcopy.hip -- host-side copies of message-sized buffers into and out of libpcp's pinned
// memory, split over a few helper threads (host code only).
//
// Every C5 frame moves ~3 MB through host memcpy: each callback's message into the pinned ring
// (the kernels read it there, pin_stage / upload_*), and each result out of its pinned landing
// into the caller's array.  One core copies ~25 GB/s, so a 60k-point scan (960 KB) costs ~40 us
// on the critical path between callbacks.  Copies of at least kSplitMin bytes are split into
// kParts parts, claimed by the calling thread and the helper threads alike (a helper that is
// asleep or preempted leaves its share to the others instead of stalling the copy).  Helpers spin on
// a job generation for a short while after each job (a streaming chain's next copy is ~100 us
// away) and then sleep on a condition variable (a 10 Hz node's helpers sleep between frames).
// PCP_COPY_THREADS=0 turns the helpers off (plain memcpy), N sets their count (default 3).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "pcp_internal.hpp"

namespace pcp {

namespace {
constexpr size_t kSplitMin = 256u << 10;
constexpr int kMaxHelpers = 7;
constexpr auto kSpin = std::chrono::microseconds(300);
// the parts of a job are claimed (one CAS on {job, next part}), the caller included, and each
// claimed part decrements `pending` once, which the caller waits for.  Every part is non-empty:
// with k parts of per = ceil(n / k) rounded up to 4 KiB < n / k + 4096 bytes, the last part
// starts at (k - 1) per < n whenever n > k (k - 1) 4096 (2 k 4096 did not imply it)
static_assert(kSplitMin > (size_t)(kMaxHelpers + 1) * kMaxHelpers * 4096, "parts must be non-empty");
static_assert(kMaxHelpers + 1 < 0xffff, "part count and index fit the claim word's 16-bit fields");

inline void cpu_relax() { __builtin_ia32_pause(); }
}  // namespace

struct CopyPool {
    struct Part {
        char *d = nullptr;
        const char *s = nullptr;
        size_t n = 0;
    };
    explicit CopyPool(int helpers) {
        for (int i = 0; i < helpers; ++i) th_.emplace_back([this, i] { run(i + 1); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_.store(true, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int parts() const { return (int)th_.size() + 1; }
    void copy(void *dst, const void *src, size_t n) {
        const int k = parts();
        // parts on 4 KiB boundaries (whole pages per thread)
        const size_t per = ((n + k - 1) / k + 4095) & ~(size_t)4095;
        int used = 0;
        for (int i = 0; i < k; ++i) {
            const size_t o = std::min(n, (size_t)i * per), e = std::min(n, o + per);
            part_[i] = Part{static_cast<char *>(dst) + o, static_cast<const char *>(src) + o, e - o};
            if (e > o) used = i + 1;
        }
        pending_.store(used, std::memory_order_relaxed);
        const uint64_t g = ++job_;
        // publishes the parts; the job's part count travels in the same word as its id, so a
        // late helper can never pair job g's id with another job's count
        claim_.store((g << 32) | ((uint64_t)used << 16), std::memory_order_release);
        {
            std::lock_guard<std::mutex> l(mu_);
            gen_.store(g, std::memory_order_release);
        }
        cv_.notify_all();
        // the parts are claimed, not assigned: the caller takes whatever the helpers have not
        // started, so a helper that is asleep or preempted (a busy host's timeslice: ms) delays
        // nothing it has not begun
        work(g);
        while (pending_.load(std::memory_order_acquire) > 0) cpu_relax();
    }

   private:
    // copy parts of job g until none is left unclaimed (a claim is one CAS on {job, parts, next
    // part}: job << 32 | used << 16 | next)
    void work(uint64_t g) {
        uint64_t c = claim_.load(std::memory_order_acquire);
        for (;;) {
            const uint32_t next = (uint32_t)c & 0xffffu, used = ((uint32_t)c >> 16) & 0xffffu;
            if ((c >> 32) != g || next >= used) return;
            if (!claim_.compare_exchange_weak(c, c + 1, std::memory_order_acq_rel,
                                              std::memory_order_acquire))
                continue;
            const Part p = part_[next];
            std::memcpy(p.d, p.s, p.n);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
            c = claim_.load(std::memory_order_acquire);
        }
    }
    void run(int) {
        uint64_t seen = 0;
        for (;;) {
            auto t0 = std::chrono::steady_clock::now();
            uint64_t g;
            for (int it = 0;; ++it) {
                g = gen_.load(std::memory_order_acquire);
                if (g != seen || stop_.load(std::memory_order_acquire)) break;
                if ((it & 255) == 255 && std::chrono::steady_clock::now() - t0 > kSpin) {
                    std::unique_lock<std::mutex> l(mu_);
                    cv_.wait(l, [&] {
                        return gen_.load(std::memory_order_acquire) != seen ||
                               stop_.load(std::memory_order_acquire);
                    });
                    t0 = std::chrono::steady_clock::now();
                }
                cpu_relax();
            }
            if (stop_.load(std::memory_order_acquire)) return;
            seen = g;
            work(g);   // (a late helper finds the job's parts claimed and goes back to waiting)
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<bool> stop_{false};
    std::atomic<uint64_t> claim_{0};   // job << 32 | parts << 16 | next unclaimed part
    uint64_t job_ = 0;                 // (the caller's; one copy at a time per pool)
    Part part_[kMaxHelpers + 1];
};

void host_copy(pcp_ctx *ctx, void *dst, const void *src, size_t bytes) {
    if (bytes < kSplitMin || ctx->copy_threads <= 0) {
        std::memcpy(dst, src, bytes);
        return;
    }
    if (!ctx->copy_pool) ctx->copy_pool = new (std::nothrow) CopyPool(std::min(ctx->copy_threads, kMaxHelpers));
    if (!ctx->copy_pool) {
        std::memcpy(dst, src, bytes);
        return;
    }
    ctx->copy_pool->copy(dst, src, bytes);
}

void host_copy_release(pcp_ctx *ctx) {
    delete ctx->copy_pool;
    ctx->copy_pool = nullptr;
}

}  // namespace pcp
