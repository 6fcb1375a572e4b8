// pcp_context.hip -- context, errors, profiling, device helpers, prefix scan.
#include <cmath>
#include <cstdio>
#include <dlfcn.h>
#include <execinfo.h>
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <new>

#include "pcp_internal.hpp"

namespace pcp {

int set_err(pcp_ctx *ctx, int code, const char *fmt, ...) {
    if (ctx) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        ctx->err = buf;
    }
    return code;
}

int hip_fail(pcp_ctx *ctx, hipError_t e, const char *what, const char *file, int line) {
    const int code = (e == hipErrorOutOfMemory) ? PCP_E_NOMEM : PCP_E_HIP;
    return set_err(ctx, code, "HIP error %d (%s) in %s at %s:%d", (int)e, hipGetErrorString(e),
                   what, file, line);
}

int check_view(pcp_ctx *ctx, const pcp_cloud_view *v, const char *what) {
    if (!v) return set_err(ctx, PCP_E_INVALID, "%s: null cloud view", what);
    if (v->n == 0) return PCP_OK;
    if (!v->data) return set_err(ctx, PCP_E_INVALID, "%s: null data with n=%llu", what,
                                 (unsigned long long)v->n);
    if (v->point_step < 12 || (v->point_step & 3) || (v->off_x & 3) || (v->off_y & 3) ||
        (v->off_z & 3) || v->off_x + 4 > v->point_step || v->off_y + 4 > v->point_step ||
        v->off_z + 4 > v->point_step)
        return set_err(ctx, PCP_E_INVALID,
                       "%s: unsupported layout point_step=%u offsets=(%u,%u,%u) (FLOAT32 "
                       "fields, 4-byte aligned)",
                       what, v->point_step, v->off_x, v->off_y, v->off_z);
    if (v->n > 0xFFFFFFF0ull) return set_err(ctx, PCP_E_INVALID, "%s: too many points", what);
    return PCP_OK;
}

static std::atomic<uint64_t> g_reallocs{0}, g_pinned_reallocs{0}, g_alloc_bytes{0};
__attribute__((noinline)) void note_realloc(size_t bytes, bool pinned) {
    (pinned ? g_pinned_reallocs : g_reallocs).fetch_add(1, std::memory_order_relaxed);
    g_alloc_bytes.fetch_add(bytes, std::memory_order_relaxed);
    // PCP_ALLOC_TRACE=1: the allocation site as an offset into libpcp (addr2line -e libpcp.so)
    static const bool trace = std::getenv("PCP_ALLOC_TRACE") != nullptr;
    if (trace) {
        void *fr[6];
        const int nf = backtrace(fr, 6);
        std::fprintf(stderr, "pcp realloc %s %zu B at", pinned ? "pinned" : "device", bytes);
        for (int i = 1; i < nf; ++i) {
            Dl_info di{};
            const uintptr_t base = dladdr(fr[i], &di) ? (uintptr_t)di.dli_fbase : 0;
            std::fprintf(stderr, " +0x%zx", (size_t)((uintptr_t)fr[i] - base));
        }
        std::fprintf(stderr, "\n");
    }
}
uint64_t alloc_count(int which) {
    return which == 0 ? g_reallocs.load() : which == 1 ? g_pinned_reallocs.load() : g_alloc_bytes.load();
}

// the next ring slot, never the one pin_stage holds (kernels may still read it)
static int next_slot(pcp_ctx *ctx) {
    int k = ctx->up_next;
    if (k == ctx->pin_held) k = (k + 1) % pcp_ctx::kUpRing;
    ctx->up_next = (k + 1) % pcp_ctx::kUpRing;
    return k;
}

// host (pinned) -> device copy by a kernel on the stream itself: no copy-engine hand-off
// before the next kernel (a DMA's submission and the engine switch cost ~15 + ~14 us here)
__global__ void __launch_bounds__(256)
k_copy_pinned(const unsigned char *__restrict__ src, unsigned char *__restrict__ dst,
              uint64_t bytes) {
    const uint64_t n16 = bytes >> 4;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
    if (blockIdx.x == 0 && threadIdx.x < (bytes & 15))
        dst[(n16 << 4) + threadIdx.x] = src[(n16 << 4) + threadIdx.x];
}

int copy_pinned_async(pcp_ctx *ctx, void *dst_d, const void *src_pinned, size_t bytes,
                      hipStream_t st) {
    if (!bytes) return PCP_OK;
    // both 16-byte aligned (device allocations and pinned slots are; offsets are the caller's)
    if (!ctx->copy_kernel || (((uintptr_t)dst_d | (uintptr_t)src_pinned) & 15u)) {
        PCP_HIP(ctx, hipMemcpyAsync(dst_d, src_pinned, bytes, hipMemcpyHostToDevice, st));
        return PCP_OK;
    }
    const uint64_t n16 = (bytes + 15) / 16;
    const unsigned g = (unsigned)std::min<uint64_t>((n16 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_copy_pinned, dim3(g), dim3(256), 0, st,
                       static_cast<const unsigned char *>(src_pinned),
                       static_cast<unsigned char *>(dst_d), (uint64_t)bytes);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

int copy_to_pinned_async(pcp_ctx *ctx, void *dst_pinned, const void *src_d, size_t bytes,
                         hipStream_t st) {
    if (!bytes) return PCP_OK;
    if (!ctx->copy_kernel || (((uintptr_t)dst_pinned | (uintptr_t)src_d) & 15u)) {
        PCP_HIP(ctx, hipMemcpyAsync(dst_pinned, src_d, bytes, hipMemcpyDeviceToHost, st));
        return PCP_OK;
    }
    const uint64_t n16 = (bytes + 15) / 16;
    const unsigned g = (unsigned)std::min<uint64_t>((n16 + 255) / 256, 1024);
    hipLaunchKernelGGL(k_copy_pinned, dim3(g), dim3(256), 0, st,
                       static_cast<const unsigned char *>(src_d),
                       static_cast<unsigned char *>(dst_pinned), (uint64_t)bytes);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

// slot s must hold `bytes`: when it has to grow, every slot of the ring grows with it (their
// earlier transfers drained first), so a stream of same-sized messages pays the pinned
// allocations once, on its first message, not on each slot's first turn
static int ring_ensure(pcp_ctx *ctx, int s, size_t bytes) {
    if (bytes <= ctx->up_buf[s].cap) return PCP_OK;
    for (int k = 0; k < pcp_ctx::kUpRing; ++k) {
        if (k == ctx->pin_held || ctx->up_buf[k].cap >= bytes) continue;
        if (ctx->up_used[k]) PCP_HIP(ctx, hipEventSynchronize(ctx->up_ev[k]));
        PCP_HIP(ctx, ctx->up_buf[k].ensure(bytes));
    }
    return PCP_OK;
}

int upload_async(pcp_ctx *ctx, void *dst_d, const void *src_h, size_t bytes, hipStream_t st) {
    if (bytes == 0) return PCP_OK;
    if (bytes > kUploadPinnedMax) {
        PCP_HIP(ctx, hipMemcpyAsync(dst_d, src_h, bytes, hipMemcpyHostToDevice, st));
        return PCP_OK;
    }
    const int k = next_slot(ctx);
    if (ctx->up_used[k]) PCP_HIP(ctx, hipEventSynchronize(ctx->up_ev[k]));   // its last DMA
    if (!ctx->up_ev[k]) PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->up_ev[k], hipEventDisableTiming));
    if (int rc = ring_ensure(ctx, k, bytes)) return rc;
    host_copy(ctx, ctx->up_buf[k].p, src_h, bytes);
    if (int rc = copy_pinned_async(ctx, dst_d, ctx->up_buf[k].p, bytes, st)) return rc;
    PCP_HIP(ctx, hipEventRecord(ctx->up_ev[k], st));
    ctx->up_used[k] = true;
    return PCP_OK;
}

int upload_pieces(pcp_ctx *ctx, void *dst_d, const HostPiece *pc, int k, size_t bytes,
                  hipStream_t st) {
    if (bytes == 0) return PCP_OK;
    if (bytes > kUploadPinnedMax) {   // pageable, piece by piece
        for (int i = 0; i < k; ++i)
            if (pc[i].bytes)
                PCP_HIP(ctx, hipMemcpyAsync(static_cast<char *>(dst_d) + pc[i].off, pc[i].src,
                                            pc[i].bytes, hipMemcpyHostToDevice, st));
        return PCP_OK;
    }
    const int s = next_slot(ctx);
    if (ctx->up_used[s]) PCP_HIP(ctx, hipEventSynchronize(ctx->up_ev[s]));
    if (!ctx->up_ev[s]) PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->up_ev[s], hipEventDisableTiming));
    if (int rc = ring_ensure(ctx, s, bytes)) return rc;
    for (int i = 0; i < k; ++i)
        if (pc[i].bytes) host_copy(ctx, static_cast<char *>(ctx->up_buf[s].p) + pc[i].off,
                                   pc[i].src, pc[i].bytes);
    if (int rc = copy_pinned_async(ctx, dst_d, ctx->up_buf[s].p, bytes, st)) return rc;
    PCP_HIP(ctx, hipEventRecord(ctx->up_ev[s], st));
    ctx->up_used[s] = true;
    return PCP_OK;
}

int pin_stage(pcp_ctx *ctx, const HostPiece *pc, int k, size_t bytes, const void **dev) {
    if (ctx->pin_held >= 0) {   // an unreleased slot (an error path): drain, then drop it
        PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
        ctx->pin_held = -1;
    }
    const int s = next_slot(ctx);
    if (ctx->up_used[s]) PCP_HIP(ctx, hipEventSynchronize(ctx->up_ev[s]));
    ctx->up_used[s] = false;
    if (!ctx->up_ev[s]) PCP_HIP(ctx, hipEventCreateWithFlags(&ctx->up_ev[s], hipEventDisableTiming));
    if (int rc = ring_ensure(ctx, s, bytes + 256)) return rc;
    for (int i = 0; i < k; ++i)
        if (pc[i].bytes) host_copy(ctx, static_cast<char *>(ctx->up_buf[s].p) + pc[i].off,
                                   pc[i].src, pc[i].bytes);
    ctx->pin_held = s;
    *dev = ctx->up_buf[s].p;
    return PCP_OK;
}

void pin_release(pcp_ctx *ctx, hipStream_t st) {
    const int s = ctx->pin_held;
    if (s < 0) return;
    ctx->pin_held = -1;
    if (hipEventRecord(ctx->up_ev[s], st) == hipSuccess) {
        ctx->up_used[s] = true;
    } else {   // no event: make sure no kernel still reads the slot
        (void)hipStreamSynchronize(st);
    }
}

int read_small(pcp_ctx *ctx, void *dst, const void *src_d, size_t bytes, hipStream_t st) {
    if (bytes > 4096) return set_err(ctx, PCP_E_INVALID, "read_small: %zu bytes", bytes);
    PCP_HIP(ctx, ctx->small_host.ensure(4096));
    PCP_HIP(ctx, hipMemcpyAsync(ctx->small_host.p, src_d, bytes, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    std::memcpy(dst, ctx->small_host.p, bytes);
    return PCP_OK;
}

void fan_tables(int32_t n_az, int32_t n_el, double el_min, double el_max, double *ca, double *sa,
                double *ce, double *se) {
    // identical expression order to oracle/pcp_oracle.c:orc_fan_tables (glibc libm)
    for (int32_t i = 0; i < n_az; ++i) {
        const double a = 2.0 * kPi * (double)i / (double)n_az;
        ca[i] = std::cos(a);
        sa[i] = std::sin(a);
    }
    for (int32_t j = 0; j < n_el; ++j) {
        const double e = el_min + (el_max - el_min) * ((double)j + 0.5) / (double)n_el;
        ce[j] = std::cos(e);
        se[j] = std::sin(e);
    }
}

std::vector<double> step_table(double end) {
    // virtual_lidar.cpp:765-796: step = 0.5; while (step < end) { ...; step += 0.3; }
    std::vector<double> s;
    double step = 0.5;   // repeated addition, not 0.5 + 0.3 k
    while (step < end) {
        s.push_back(step);
        step = step + kRayStep;
        if (s.size() > (1u << 24)) break;
    }
    return s;
}

// ---- profiling -------------------------------------------------------------------------
static hipEvent_t take_event(pcp_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

ProfScope::ProfScope(pcp_ctx *c, int k, hipStream_t s) : ctx(c), kid(k), st(s ? s : c->stream) {
    if (!ctx->prof || kid < 0 || ctx->capturing) return;
    a = take_event(ctx);
    b = take_event(ctx);
    if (a) (void)hipEventRecord(a, st);
}

ProfScope::~ProfScope() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    ctx->pending.push_back({kid, a, b});
}

KernelTimer::KernelTimer(pcp_ctx *c, int k) : ctx(c), kid(k) {
    if (!ctx->prof || kid < 0 || ctx->capturing) return;
    a = take_event(ctx);
    b = take_event(ctx);
    if (!a || !b) a = b = nullptr;
}

KernelTimer::~KernelTimer() {
    if (a && b) ctx->pending.push_back({kid, a, b});
}

void prof_count(pcp_ctx *ctx, int kid) {
    if (kid >= 0 && kid < PCP_K_COUNT) ctx->slots[kid].launches += 1;
}

void prof_resolve(pcp_ctx *ctx) {
    // calls that return without a stream synchronisation (index builds) leave events in
    // flight: those stay pending until a later call finds them complete
    std::vector<PendingEvent> keep;
    for (auto &pe : ctx->pending) {
        if (hipEventQuery(pe.b) == hipErrorNotReady) {
            keep.push_back(pe);
            continue;
        }
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pe.a, pe.b) == hipSuccess) {
            ctx->slots[pe.kid].total_ms += ms;
            ctx->slots[pe.kid].launches += 1;
        }
        ctx->event_pool.push_back(pe.a);
        ctx->event_pool.push_back(pe.b);
    }
    ctx->pending.swap(keep);
}

// ---- exclusive scan (uint32) ----------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;   // 2048

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    return v;
}

// block-wide exclusive scan of one value per thread; returns exclusive prefix, *total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *lds4, uint32_t *total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t incl = wave_incl_scan(v);
    if (lane == 63) lds4[wid] = incl;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kScanThreads / 64; ++w) {
        const uint32_t s = lds4[w];
        if (w < wid) off += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return off + incl - v;
}

__global__ void __launch_bounds__(kScanThreads)
k_scan_tile_sums(const uint32_t *__restrict__ in, uint64_t n, uint32_t *__restrict__ sums) {
    __shared__ uint32_t lds4[4];
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t k = base + (uint64_t)i * kScanThreads + threadIdx.x;
        if (k < n) s += in[k];
    }
    uint32_t tot;
    (void)block_excl_scan(s, lds4, &tot);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// scans each tile locally (thread owns kScanItems consecutive items), adds tile offset;
// out2 (may be null, may be `in` itself: every thread reads its own items before it writes
// them) receives a second copy of out[0 .. n)
__device__ __forceinline__ void scan_tile(const uint32_t *in, uint64_t n, uint32_t off,
                                          uint32_t *__restrict__ out, uint32_t *out2, int zero2,
                                          uint16_t *__restrict__ preset16, uint32_t tile,
                                          bool last_tile) {
    __shared__ uint32_t lds4[4];
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    // a thread's 8 items whole: two 16-byte loads and stores instead of 8 single words at a
    // 32-byte lane stride (4x the cache-line visits per wave) -- when the arrays are 16-byte
    // aligned (item offsets are multiples of 8; the recursion's partial-sum arrays may not be)
    const bool al = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out) |
                      reinterpret_cast<uintptr_t>(out2)) & 15u) == 0;
    const bool whole = al && base + kScanItems <= n;
    static_assert(kScanItems == 8, "two uint4 per thread");
    uint32_t v[kScanItems];
    uint32_t s = 0;
    if (whole) {
        const uint4 a = reinterpret_cast<const uint4 *>(in + base)[0];
        const uint4 b = reinterpret_cast<const uint4 *>(in + base)[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) {
            const uint64_t k = base + i;
            v[i] = (k < n) ? in[k] : 0u;
        }
    }
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) s += v[i];
    uint32_t tot;
    uint32_t run = block_excl_scan(s, lds4, &tot) + off;
    uint32_t o[kScanItems];
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        o[i] = run;
        run += v[i];
    }
    if (whole) {
        reinterpret_cast<uint4 *>(out + base)[0] = make_uint4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<uint4 *>(out + base)[1] = make_uint4(o[4], o[5], o[6], o[7]);
        if (out2) {   // zero2: leave out2 (= in) cleared
            const uint4 z = make_uint4(0u, 0u, 0u, 0u);
            reinterpret_cast<uint4 *>(out2 + base)[0] = zero2 ? z : make_uint4(o[0], o[1], o[2], o[3]);
            reinterpret_cast<uint4 *>(out2 + base)[1] = zero2 ? z : make_uint4(o[4], o[5], o[6], o[7]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < kScanItems; ++i) {
            const uint64_t k = base + i;
            if (k < n) {
                out[k] = o[i];
                if (out2) out2[k] = zero2 ? 0u : o[i];
            }
        }
    }
    if (preset16)
#pragma unroll
        for (int i = 0; i < kScanItems; ++i)
            if (base + i < n) preset16[base + i] = 0x00FFu;
    // out[n] written by the last tile's last thread
    if (last_tile && threadIdx.x == kScanThreads - 1) out[n] = run;
}

__global__ void __launch_bounds__(kScanThreads)
k_scan_tiles(const uint32_t *in, uint64_t n, const uint32_t *__restrict__ offs,
             uint32_t *__restrict__ out, uint32_t *out2, int zero2, uint16_t *__restrict__ preset16) {
    scan_tile(in, n, offs ? offs[blockIdx.x] : 0u, out, out2, zero2, preset16, blockIdx.x,
              blockIdx.x == gridDim.x - 1);
}

// two one-tile scans in one launch (block 0: a, block 1: b; a grid index's pair of builds)
struct ScanOne {
    const uint32_t *in;
    uint64_t n;
    uint32_t *out, *out2;
};
__global__ void __launch_bounds__(kScanThreads) k_scan_pair(ScanOne a, ScanOne b, int zero2) {
    const ScanOne &q = blockIdx.x ? b : a;
    scan_tile(q.in, q.n, 0u, q.out, q.out2, zero2, nullptr, 0u, true);
}

// one-pass exclusive scan: tiles take tickets in arrival order (a tile waits only for tiles
// already running), publish their aggregate, then look back over their predecessors' status
// words 64 at a time (wave 0, one per lane) until an inclusive prefix; a status word is one
// 64-bit agent-scope store {value, epoch << 2 | flag} (flag 1 aggregate, 2 inclusive), so a
// reader sees the value with its flag and the previous call's words (older epoch) as absent
__global__ void __launch_bounds__(kScanThreads)
k_scan_onepass(const uint32_t *in, uint64_t n, uint32_t *out, uint32_t *out2, int zero2,
               unsigned long long *state, uint32_t *ticket, uint32_t ticket_base, uint32_t epoch,
               uint16_t *__restrict__ preset16) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t sh_tile, sh_prefix;
    if (threadIdx.x == 0) sh_tile = atomicAdd(ticket, 1u) - ticket_base;
    __syncthreads();
    const uint32_t tile = sh_tile;
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint32_t v[kScanItems], s = 0;
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t k = base + i;
        v[i] = (k < n) ? in[k] : 0u;
        s += v[i];
    }
    uint32_t agg;
    const uint32_t ex_local = block_excl_scan(s, lds4, &agg);
    const uint64_t tag = (uint64_t)(epoch << 2);
    auto publish = [&](uint32_t flag, uint32_t val) {
        __hip_atomic_store(&state[tile], ((tag | flag) << 32) | val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    };
    if (threadIdx.x == 0) publish(tile == 0 ? 2u : 1u, agg);
    if (tile > 0 && threadIdx.x < 64) {
        const int lane = threadIdx.x;
        uint32_t prefix = 0;
        int64_t top = (int64_t)tile - 1;   // the window's first (nearest) predecessor
        for (;;) {
            const int64_t j = top - lane;
            uint64_t w = 0;
            uint32_t flag = 2;   // (lanes past tile 0: an empty inclusive prefix)
            if (j >= 0) {
                for (;;) {
                    w = __hip_atomic_load(&state[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if ((uint32_t)(w >> 34) == (epoch & 0x3fffffffu) && ((w >> 32) & 3u) != 0u)
                        break;
                    __builtin_amdgcn_s_sleep(1);
                }
                flag = (uint32_t)(w >> 32) & 3u;
            }
            const uint32_t val = (uint32_t)w;
            // the nearest inclusive lane ends the walk: add the lanes up to it
            const uint64_t inc = __ballot(flag == 2u);
            const int stop = inc ? __ffsll((unsigned long long)inc) - 1 : 64;
            uint32_t part = lane <= stop ? val : 0u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
            prefix += part;
            if (inc) break;
            top -= 64;
        }
        if (lane == 0) {
            publish(2u, prefix + agg);
            sh_prefix = prefix;
        }
    }
    __syncthreads();
    uint32_t run = ex_local + (tile > 0 ? sh_prefix : 0u);
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
        const uint64_t k = base + i;
        if (k < n) {
            out[k] = run;
            if (out2) out2[k] = zero2 ? 0u : run;
            if (preset16) preset16[k] = 0x00FFu;
        }
        run += v[i];
    }
    // out[n] = the total, by the last tile's last thread (its items past n are zero)
    if (tile == gridDim.x - 1 && threadIdx.x == kScanThreads - 1) out[n] = run;
}

size_t scan_tmp_bytes(uint64_t n) {
    size_t bytes = 0;
    while (n > (uint64_t)kScanTile) {
        const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
        bytes += (tiles + 1) * 2 * sizeof(uint32_t) + 256;
        n = tiles;
    }
    return bytes + 256;
}

int exclusive_scan_u32(pcp_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n, void *tmp,
                       uint32_t *out2, bool zero2, uint16_t *preset16) {
    if (n == 0) {
        PCP_HIP(ctx, hipMemsetAsync(out, 0, sizeof(uint32_t), ctx->stream));
        return PCP_OK;
    }
    const uint64_t tiles = (n + kScanTile - 1) / kScanTile;
    // one pass only where the look-back is one window (tiles <= 64: tile 0's inclusive prefix
    // in every tile's first window); longer scans walk windows of aggregates back to tile 0,
    // which measured slower than the three short launches (terrain grids, ~430 tiles)
    if (tiles > 1 && tiles <= 64 && ctx->scan_onepass) {
        const size_t cap0 = ctx->scan_state.cap;
        PCP_HIP(ctx, ctx->scan_state.ensure(tiles * sizeof(unsigned long long) + 64));
        if (++ctx->scan_epoch >= (1u << 30) || ctx->scan_state.cap != cap0) {   // wrap / new buffer
            PCP_HIP(ctx, hipMemsetAsync(ctx->scan_state.p, 0, ctx->scan_state.cap, ctx->stream));
            ctx->scan_epoch = 1;
            ctx->scan_ticket = 0;
        }
        unsigned long long *state = ctx->scan_state.as<unsigned long long>();
        uint32_t *ticket = reinterpret_cast<uint32_t *>(ctx->scan_state.as<char>() + ctx->scan_state.cap - 64);
        hipLaunchKernelGGL(k_scan_onepass, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream,
                           in, n, out, out2, zero2 ? 1 : 0, state, ticket, ctx->scan_ticket,
                           ctx->scan_epoch, preset16);
        PCP_CHECK_LAUNCH(ctx);
        ctx->scan_ticket += (uint32_t)tiles;
        return PCP_OK;
    }
    if (tiles == 1) {
        hipLaunchKernelGGL(k_scan_tiles, dim3(1), dim3(kScanThreads), 0, ctx->stream, in, n,
                           (const uint32_t *)nullptr, out, out2, zero2 ? 1 : 0, preset16);
        PCP_CHECK_LAUNCH(ctx);
        return PCP_OK;
    }
    uint32_t *sums = static_cast<uint32_t *>(tmp);
    uint32_t *sums_scan = sums + tiles + 1;
    void *next = reinterpret_cast<char *>(tmp) + (tiles + 1) * 2 * sizeof(uint32_t) + 256;
    hipLaunchKernelGGL(k_scan_tile_sums, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream,
                       in, n, sums);
    PCP_CHECK_LAUNCH(ctx);
    int rc = exclusive_scan_u32(ctx, sums, sums_scan, tiles, next);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_tiles, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream, in,
                       n, (const uint32_t *)sums_scan, out, out2, zero2 ? 1 : 0, preset16);
    PCP_CHECK_LAUNCH(ctx);
    return PCP_OK;
}

}  // namespace pcp

// the library's device exclusive scan on a host array (diagnostic entry point: the one-pass
// look-back form against the three-launch form, tests/test_gpu_parity.py::test_exclusive_scan_*)
extern "C" int pcp_debug_exclusive_scan(pcp_ctx *ctx, const uint32_t *in, uint64_t n,
                                        uint32_t *out) {
    using namespace pcp;
    if (!ctx || (n && !in) || !out) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    DevBuf din, dout, dtmp;
    PCP_HIP(ctx, din.ensure((n + 1) * sizeof(uint32_t)));
    PCP_HIP(ctx, dout.ensure((n + 1) * sizeof(uint32_t)));
    PCP_HIP(ctx, dtmp.ensure(scan_tmp_bytes(n) + 256));
    int rc = PCP_OK;
    hipError_t e = n ? hipMemcpyAsync(din.p, in, n * sizeof(uint32_t), hipMemcpyHostToDevice,
                                      ctx->stream)
                     : hipSuccess;
    if (e == hipSuccess)
        rc = exclusive_scan_u32(ctx, din.as<const uint32_t>(), dout.as<uint32_t>(), n, dtmp.p);
    if (e == hipSuccess && rc == PCP_OK)
        e = hipMemcpyAsync(out, dout.p, (n + 1) * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    din.release();
    dout.release();
    dtmp.release();
    if (rc) return rc;
    if (e != hipSuccess) return hip_fail(ctx, e, "pcp_debug_exclusive_scan", __FILE__, __LINE__);
    return PCP_OK;
}

namespace pcp {
// exclusive_scan_u32 of two arrays (out2 / zero2 as there, no preset); two one-tile scans
// (a message-sized cloud's pair of grids) are one launch
int exclusive_scan_u32_pair(pcp_ctx *ctx, const uint32_t *in_a, uint32_t *out_a, uint64_t n_a,
                            uint32_t *out2_a, const uint32_t *in_b, uint32_t *out_b, uint64_t n_b,
                            uint32_t *out2_b, void *tmp, bool zero2) {
    if (n_a && n_b && n_a <= (uint64_t)kScanTile && n_b <= (uint64_t)kScanTile && ctx->scan_pair) {
        hipLaunchKernelGGL(k_scan_pair, dim3(2), dim3(kScanThreads), 0, ctx->stream,
                           ScanOne{in_a, n_a, out_a, out2_a}, ScanOne{in_b, n_b, out_b, out2_b},
                           zero2 ? 1 : 0);
        PCP_CHECK_LAUNCH(ctx);
        return PCP_OK;
    }
    if (int rc = exclusive_scan_u32(ctx, in_a, out_a, n_a, tmp, out2_a, zero2)) return rc;
    return exclusive_scan_u32(ctx, in_b, out_b, n_b, tmp, out2_b, zero2);
}

}  // namespace pcp

using namespace pcp;

// ======================================================================================
// C ABI: context
// ======================================================================================
extern "C" {

int pcp_abi_version(void) { return PCP_ABI_VERSION; }

int pcp_alloc_stats(uint64_t *device_reallocs, uint64_t *pinned_reallocs, uint64_t *bytes) {
    if (device_reallocs) *device_reallocs = alloc_count(0);
    if (pinned_reallocs) *pinned_reallocs = alloc_count(1);
    if (bytes) *bytes = alloc_count(2);
    return PCP_OK;
}

int pcp_device_count(int *n) {
    if (!n) return PCP_E_INVALID;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return PCP_OK;
}

int pcp_create(int device, pcp_ctx **out) {
    if (!out) return PCP_E_INVALID;
    *out = nullptr;
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c <= 0) return PCP_E_HIP;
    if (device < 0 || device >= c) return PCP_E_INVALID;
    if (hipSetDevice(device) != hipSuccess) return PCP_E_HIP;
    pcp_ctx *ctx = new (std::nothrow) pcp_ctx();
    if (!ctx) return PCP_E_NOMEM;
    ctx->device = device;
    if (const char *fb = std::getenv("PCP_FAN_BATCH")) ctx->fan_batch = std::atoi(fb);
    if (const char *fw = std::getenv("PCP_FAN_NPW")) {
        const int v = std::atoi(fw);
        ctx->fan_npw = (v == 2 || v == 4 || v == 8 || v == 16 || v == 32) ? v : 1;
    }
    if (const char *ho = std::getenv("PCP_FAN_HOST_OUT")) ctx->fan_host_out = std::atoi(ho) != 0;
    if (const char *ne = std::getenv("PCP_NORMALS_EXACT")) ctx->normals_exact = std::atoi(ne) != 0;
    if (const char *sw = std::getenv("PCP_SCORE_WIDE")) ctx->score_wide = std::atoi(sw) != 0;
    if (const char *wr = std::getenv("PCP_SCORE_WIDE_RAYS")) ctx->score_wide_rays = std::atoll(wr);
    if (const char *wg = std::getenv("PCP_SCORE_WIDE_G")) ctx->score_wide_g = std::atoi(wg);
    if (const char *co = std::getenv("PCP_CELLS_ORDER_FREE")) ctx->cells_all_ordered = std::atoi(co) == 0;
    if (const char *nbk = std::getenv("PCP_NB_BLOCKS")) ctx->nb_blocks = std::atoi(nbk);
    if (const char *sp = std::getenv("PCP_SCAN_ONEPASS")) ctx->scan_onepass = std::atoi(sp) != 0;
    if (const char *ip = std::getenv("PCP_INDEX_PAIR")) ctx->index_pair = std::atoi(ip) != 0;
    if (const char *as = std::getenv("PCP_AREA_STREAM")) ctx->area_side = std::atoi(as) != 0;
    if (const char *ns = std::getenv("PCP_NB_SMALL")) ctx->nb_small = std::atoi(ns) != 0;
    if (const char *rp = std::getenv("PCP_NB_REGION_PCT"))
        ctx->nb_region_pct = std::min(100, std::max(1, std::atoi(rp)));
    if (const char *gw = std::getenv("PCP_NB_GUESS_WORDS"))
        ctx->nb_guess_max = std::max<uint64_t>(1, std::strtoull(gw, nullptr, 10));
    if (const char *ct = std::getenv("PCP_COPY_THREADS")) ctx->copy_threads = std::atoi(ct);
    if (const char *fo = std::getenv("PCP_FM_HOST_OUT")) ctx->fm_host_out = std::atoi(fo) != 0;
    if (const char *ff = std::getenv("PCP_FM_FAST")) ctx->fm_fast = std::atoi(ff);
    if (const char *bg = std::getenv("PCP_BK_GT")) ctx->bk_gt = std::atoi(bg);
    if (const char *sp = std::getenv("PCP_SCAN_PAIR")) ctx->scan_pair = std::atoi(sp) != 0;
    if (const char *fc = std::getenv("PCP_CARVE_FUSE_COPY")) ctx->carve_fuse_copy = std::atoi(fc) != 0;
    if (const char *bp = std::getenv("PCP_BK_PTS")) ctx->bk_pts = std::atoi(bp);
    if (const char *zc = std::getenv("PCP_ZC_IN")) ctx->zc_in = std::atoi(zc) != 0;
    if (const char *ck = std::getenv("PCP_COPY_KERNEL")) ctx->copy_kernel = std::atoi(ck) != 0;
    if (const char *tb = std::getenv("PCP_TERRAIN_BLOCKS")) ctx->terrain_blocks = std::atoi(tb);
    if (const char *tf = std::getenv("PCP_TERRAIN_FINE")) ctx->terrain_fine = std::atoi(tf);
    if (const char *tt = std::getenv("PCP_FINE_TILE")) ctx->fine_tile = std::atoi(tt);
    if (const char *fs = std::getenv("PCP_FINE_SKIP")) ctx->fine_skip = std::atoi(fs) == 2 ? 2 : 1;
    if (const char *fp = std::getenv("PCP_FINE_PACK")) ctx->fine_pack = std::atoi(fp) != 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        cus > 0)
        ctx->num_cus = cus;
    if (const char *ng = std::getenv("PCP_NO_GRAPHS")) ctx->use_graphs = std::atoi(ng) == 0;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return PCP_E_HIP;
    }
    *out = ctx;
    return PCP_OK;
}

void pcp_destroy(pcp_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->area_stream) (void)hipStreamSynchronize(ctx->area_stream);
    prof_resolve(ctx);
    for (hipEvent_t e : ctx->event_pool) (void)hipEventDestroy(e);
    if (ctx->area_fork_ev) (void)hipEventDestroy(ctx->area_fork_ev);
    if (ctx->area_join_ev) (void)hipEventDestroy(ctx->area_join_ev);
    if (ctx->keys_ev) (void)hipEventDestroy(ctx->keys_ev);
    comm_release(ctx);
    host_copy_release(ctx);
    for (int k = 0; k < pcp_ctx::kUpRing; ++k) {
        if (ctx->up_ev[k]) (void)hipEventDestroy(ctx->up_ev[k]);
        ctx->up_buf[k].release();
    }
    ctx->cand_host.release();
    ctx->tc_host.release();
    ctx->cv_host.release();
    ctx->terrain.release();
    ctx->aux.release();
    ctx->exc_norm.release();
    ctx->exc_near.release();
    ctx->area_nrm.release();
    ctx->nb_list.release();
    ctx->nb_meta.release();
    ctx->nb_ctl.release();
    ctx->nb_pts.release();
    ctx->nb_list_c.release();
    ctx->nb_meta_c.release();
    ctx->nb_sel.release();
    ctx->carve.release();
    ctx->carve_buf.release();
    ctx->cell_cnt.release();
    ctx->cell_cnt2.release();
    ctx->carve_gen.release();
    ctx->fan_host.release();
    ctx->res_host.release();
    ctx->fm_res_host.release();
    ctx->small_host.release();
    ctx->area_host.release();
    DevBuf *bufs[] = {&ctx->cells_xyz, &ctx->cells_nrm, &ctx->cells_n_d, &ctx->stage, &ctx->fan_tab,
                      &ctx->poses_d,   &ctx->steps_d,   &ctx->out_a, &ctx->out_b,
                      &ctx->out_c,     &ctx->out_d,     &ctx->stats_d, &ctx->f_in,
                      &ctx->f_misc,    &ctx->bk_stat};
    for (DevBuf *b : bufs) b->release();
    for (auto &b : ctx->scratch) b.release();
    for (auto &b : ctx->fbuf) b.release();
    if (ctx->fm_exec) (void)hipGraphExecDestroy(ctx->fm_exec);
    if (ctx->fm_graph) (void)hipGraphDestroy(ctx->fm_graph);
    ctx->lat_flags.release();
    ctx->scan_state.release();
    ctx->carve_ctr.release();
    ctx->exc_land.release();
    if (ctx->area_stream) (void)hipStreamDestroy(ctx->area_stream);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *pcp_last_error(const pcp_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int pcp_synchronize(pcp_ctx *ctx) {
    if (!ctx) return PCP_E_INVALID;
    area_join(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    return PCP_OK;
}

int pcp_stream_create(pcp_ctx *ctx, void **stream) {
    if (!ctx || !stream) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t s = nullptr;
    PCP_HIP(ctx, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return PCP_OK;
}

int pcp_stream_destroy(pcp_ctx *ctx, void *stream) {
    if (!ctx || !stream) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    PCP_HIP(ctx, hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return PCP_OK;
}

int pcp_host_alloc(pcp_ctx *ctx, uint64_t bytes, void **hptr) {
    if (!ctx || !hptr) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault));
    return PCP_OK;
}

int pcp_host_free(pcp_ctx *ctx, void *hptr) {
    if (!ctx) return PCP_E_INVALID;
    if (hptr) PCP_HIP(ctx, hipHostFree(hptr));
    return PCP_OK;
}

int pcp_host_register(pcp_ctx *ctx, void *hptr, uint64_t bytes) {
    if (!ctx || !hptr || !bytes) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, hipHostRegister(hptr, bytes, hipHostRegisterDefault));
    return PCP_OK;
}

int pcp_host_unregister(pcp_ctx *ctx, void *hptr) {
    if (!ctx || !hptr) return PCP_E_INVALID;
    PCP_HIP(ctx, hipHostUnregister(hptr));
    return PCP_OK;
}

int pcp_dev_alloc(pcp_ctx *ctx, uint64_t bytes, void **dptr) {
    if (!ctx || !dptr) return PCP_E_INVALID;
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    PCP_HIP(ctx, hipMalloc(dptr, bytes ? bytes : 16));
    return PCP_OK;
}

int pcp_dev_free(pcp_ctx *ctx, void *dptr) {
    if (!ctx) return PCP_E_INVALID;
    if (dptr) PCP_HIP(ctx, hipFree(dptr));
    return PCP_OK;
}

int pcp_memcpy_h2d(pcp_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return PCP_E_INVALID;
    PCP_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_memcpy_d2h(pcp_ctx *ctx, void *dst, const void *src, uint64_t bytes) {
    if (!ctx || (bytes && (!dst || !src))) return PCP_E_INVALID;
    PCP_HIP(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return PCP_OK;
}

int pcp_profile_enable(pcp_ctx *ctx, int enable) {
    if (!ctx) return PCP_E_INVALID;
    ctx->prof = enable != 0;
    return PCP_OK;
}

int pcp_profile_reset(pcp_ctx *ctx) {
    if (!ctx) return PCP_E_INVALID;
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    for (auto &s : ctx->slots) s = ProfSlot{};
    return PCP_OK;
}

int pcp_profile_get(pcp_ctx *ctx, int kid, double *total_ms, uint64_t *launches) {
    if (!ctx || kid < 0 || kid >= PCP_K_COUNT) return PCP_E_INVALID;
    PCP_HIP(ctx, hipStreamSynchronize(ctx->stream));
    prof_resolve(ctx);
    if (total_ms) *total_ms = ctx->slots[kid].total_ms;
    if (launches) *launches = ctx->slots[kid].launches;
    return PCP_OK;
}

const char *pcp_kernel_name(int kid) {
    static const char *names[PCP_K_COUNT] = {"raycast_fan", "score_cells", "zx120_cells",
                                             "pose_sum",    "cell_flags",  "candidates",
                                             "index_build", "crop",        "voxel",
                                             "transform",   "filter_merge", "excavate",
                                             "excav_setup", "voxel_redo"};
    if (kid < 0 || kid >= PCP_K_COUNT) return "unknown";
    return names[kid];
}

int pcp_step_table(double end, double *steps, uint64_t cap, uint64_t *n) {
    if (!n || (cap && !steps)) return PCP_E_INVALID;
    std::vector<double> s = step_table(end);
    *n = s.size();
    for (uint64_t i = 0; i < s.size() && i < cap; ++i) steps[i] = s[i];
    return PCP_OK;
}

}  // extern "C"
