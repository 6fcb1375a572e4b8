// pcp_multi.hip -- one process, n GPUs: the virtual-LiDAR pose search sharded over devices
// (SURVEY.md §8b `pcp_multi_create`, §8e).  Host code only (the key kernels live in
// pcp_vlidar.hip): n contexts, one RCCL communicator over them (ncclCommInitAll), poses
// partitioned contiguously (rank r takes [r*P/n, (r+1)*P/n), the first P % n ranks one more),
// the terrain index replicated, and ONE collective per query:
//   fan:            ncclAllReduce(ncclUint64, ncclMin) over P keys (blocked << 32) | pose
//   reference mode: ncclAllReduce(ncclUint64, ncclMax) over [P totals | P covered | 3 x C
//                   newest-pose flag keys]
// The reduced vector lands on every rank; rank 0's copy gives the host the reference-exact
// argmin / strict-'>' argmax (virtual_lidar.cpp:471-474) and the stale-flag colour statistics.
//
// Ranks that all share ONE device (a rehearsal on one GPU; RCCL refuses duplicate devices in
// one communicator) combine their key vectors on that device instead: same keys, same
// finalization, min / max by a kernel.  A mixed list ({0, 0, 1}) is refused: the combine
// kernel would read another device's buffers (no peer access is set up).
//
// The per-device index builds (pcp_multi_set_*) run on one host thread per device; a query
// issues every rank's pose upload before any rank's launches.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pcp_internal.hpp"

using namespace pcp;

namespace {
// one host thread per rank (rank 0 = the caller's thread): every rank's work -- index builds,
// a query's pose upload + launches -- is issued concurrently instead of rank after rank.
// Only used when the ranks sit on distinct devices (one context per device per thread).
class RankPool {
   public:
    void start(int n) {
        for (int r = 1; r < n; ++r) th_.emplace_back([this, r] { loop(r); });
    }
    ~RankPool() {
        {
            std::lock_guard<std::mutex> l(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    bool active() const { return !th_.empty(); }
    // f(r) for every rank r, concurrently; returns when all are done
    void run(const std::function<void(int)> &f) {
        {
            std::lock_guard<std::mutex> l(mu_);
            job_ = &f;
            pending_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(mu_);
        done_.wait(l, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

   private:
    void loop(int r) {
        uint64_t seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> l(mu_);
            cv_.wait(l, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const std::function<void(int)> *f = job_;
            l.unlock();
            (*f)(r);
            l.lock();
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)> *job_ = nullptr;
    uint64_t gen_ = 0;
    int pending_ = 0;
    bool stop_ = false;
};
}  // namespace

struct pcp_multi {
    int n = 0;
    RankPool pool;                      // threads of ranks 1..n-1 (distinct devices only)
    std::vector<pcp_ctx *> ctx;
    std::vector<ncclComm_t> comm;       // empty when ranks share a device
    std::vector<DevBuf> keys;           // per rank: the vector the collective reduces
    DevBuf tmp;                         // rank 0: a peer vector (shared-device combine)
    PinnedBuf host;                     // rank 0's reduced vector + per-rank units
    std::string err;
};

namespace {

int merr(pcp_multi *m, int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    m->err = buf;
    return code;
}

// a rank's call failed: its context holds the message
int from_ctx(pcp_multi *m, int r, int rc) {
    m->err = "rank " + std::to_string(r) + ": " + pcp_last_error(m->ctx[r]);
    return rc;
}

// f(r) -> status for every rank: concurrently on the rank threads when the ranks own distinct
// devices, else in rank order; the first failing rank's status (its context has the message)
int for_ranks(pcp_multi *m, const std::function<int(int)> &f) {
    std::vector<int> rc(m->n, PCP_OK);
    if (m->pool.active()) {
        m->pool.run([&](int r) { rc[r] = f(r); });
    } else {
        for (int r = 0; r < m->n; ++r)
            if ((rc[r] = f(r)) != PCP_OK) break;
    }
    for (int r = 0; r < m->n; ++r)
        if (rc[r] != PCP_OK) return from_ctx(m, r, rc[r]);
    return PCP_OK;
}

#define M_HIP(m, expr)                                                                    \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess)                                                             \
            return merr((m), PCP_E_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                        __FILE__, __LINE__);                                              \
    } while (0)

#define M_NCCL(m, expr)                                                                   \
    do {                                                                                  \
        ncclResult_t _r = (expr);                                                         \
        if (_r != ncclSuccess)                                                            \
            return merr((m), PCP_E_HIP, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r),  \
                        __FILE__, __LINE__);                                              \
    } while (0)

void shard(uint64_t total, int world, int rank, uint64_t &lo, uint64_t &cnt) {
    const uint64_t base = total / (uint64_t)world, rem = total % (uint64_t)world;
    lo = (uint64_t)rank * base + std::min<uint64_t>((uint64_t)rank, rem);
    cnt = base + ((uint64_t)rank < rem ? 1 : 0);
}

// reduce the n per-rank key vectors (count uint64 each) in place: afterwards every rank's
// buffer (RCCL) or rank 0's buffer (shared device) holds the reduction
int reduce_keys(pcp_multi *m, size_t count, bool is_max) {
    if (!m->comm.empty()) {
        M_NCCL(m, ncclGroupStart());
        for (int r = 0; r < m->n; ++r) {
            ncclResult_t rr =
                ncclAllReduce(m->keys[r].p, m->keys[r].p, count, ncclUint64,
                              is_max ? ncclMax : ncclMin, m->comm[r], m->ctx[r]->stream);
            if (rr != ncclSuccess) {
                (void)ncclGroupEnd();
                return merr(m, PCP_E_HIP, "ncclAllReduce: %s", ncclGetErrorString(rr));
            }
        }
        M_NCCL(m, ncclGroupEnd());
        return PCP_OK;
    }
    // shared device: every rank's stream done, then rank 0 folds the others in
    for (int r = 1; r < m->n; ++r) M_HIP(m, hipStreamSynchronize(m->ctx[r]->stream));
    pcp_ctx *c0 = m->ctx[0];
    M_HIP(m, hipSetDevice(c0->device));
    for (int r = 1; r < m->n; ++r) {
        launch_keys_combine(c0->stream, m->keys[0].as<unsigned long long>(),
                            m->keys[r].as<const unsigned long long>(), count, is_max);
        M_HIP(m, hipGetLastError());
    }
    return PCP_OK;
}

int ensure_keys(pcp_multi *m, size_t count) {
    for (int r = 0; r < m->n; ++r) {
        M_HIP(m, hipSetDevice(m->ctx[r]->device));
        M_HIP(m, m->keys[r].ensure(count * sizeof(unsigned long long) + 64));
    }
    return PCP_OK;
}

}  // namespace

extern "C" {

int pcp_multi_create(int n_dev, const int *devices, pcp_multi **out) {
    if (!out || n_dev <= 0 || n_dev > 64) return PCP_E_INVALID;
    *out = nullptr;
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have <= 0) return PCP_E_HIP;
    std::vector<int> dev(n_dev);
    for (int r = 0; r < n_dev; ++r) {
        dev[r] = devices ? devices[r] : r;
        if (dev[r] < 0 || dev[r] >= have) return PCP_E_INVALID;
    }
    std::vector<int> sorted = dev;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const bool one_device = sorted.front() == sorted.back();
    if (!distinct && !one_device) return PCP_E_INVALID;   // mixed: no combine across devices
    pcp_multi *m = new (std::nothrow) pcp_multi();
    if (!m) return PCP_E_NOMEM;
    m->n = n_dev;
    m->ctx.assign(n_dev, nullptr);
    m->keys.resize(n_dev);
    for (int r = 0; r < n_dev; ++r) {
        int rc = pcp_create(dev[r], &m->ctx[r]);
        if (rc) {
            pcp_multi_destroy(m);
            return rc;
        }
    }
    if (distinct) {
        m->comm.resize(n_dev);
        if (ncclCommInitAll(m->comm.data(), n_dev, dev.data()) != ncclSuccess) {
            m->comm.clear();
            pcp_multi_destroy(m);
            return PCP_E_HIP;
        }
        m->pool.start(n_dev);
    }
    *out = m;
    return PCP_OK;
}

void pcp_multi_destroy(pcp_multi *m) {
    if (!m) return;
    for (ncclComm_t c : m->comm) (void)ncclCommDestroy(c);
    for (int r = 0; r < m->n; ++r) {
        if (!m->ctx[r]) continue;
        (void)hipSetDevice(m->ctx[r]->device);
        m->keys[r].release();
        if (r == 0) m->tmp.release();
    }
    m->host.release();
    for (pcp_ctx *c : m->ctx) pcp_destroy(c);
    delete m;
}

const char *pcp_multi_last_error(const pcp_multi *m) { return m ? m->err.c_str() : "null"; }

int pcp_multi_info(const pcp_multi *m, int *n_dev, int *uses_rccl) {
    if (!m) return PCP_E_INVALID;
    if (n_dev) *n_dev = m->n;
    if (uses_rccl) *uses_rccl = m->comm.empty() ? 0 : 1;
    return PCP_OK;
}

pcp_ctx *pcp_multi_ctx(pcp_multi *m, int rank) {
    return (m && rank >= 0 && rank < m->n) ? m->ctx[rank] : nullptr;
}

// the index builds run on every device from the host buffer (each takes ~1 ms per 1M points),
// all devices at once (one host thread per device)
int pcp_multi_set_terrain(pcp_multi *m, const pcp_cloud_view *terrain) {
    if (!m) return PCP_E_INVALID;
    return for_ranks(m, [&](int r) { return pcp_set_terrain(m->ctx[r], terrain); });
}

int pcp_multi_set_aux_cloud(pcp_multi *m, const pcp_cloud_view *aux) {
    if (!m) return PCP_E_INVALID;
    return for_ranks(m, [&](int r) { return pcp_set_aux_cloud(m->ctx[r], aux); });
}

int pcp_multi_set_cells(pcp_multi *m, const double *xyz, const float *normals, uint64_t n) {
    if (!m) return PCP_E_INVALID;
    return for_ranks(m, [&](int r) { return pcp_set_cells(m->ctx[r], xyz, normals, n); });
}

int pcp_multi_raycast_fan(pcp_multi *m, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, uint32_t *blocked, uint64_t *units,
                          int64_t *best_idx) {
    if (!m) return PCP_E_INVALID;
    if (!fan || (n && (!poses5 || !blocked)))
        return merr(m, PCP_E_INVALID, "pcp_multi_raycast_fan: null argument");
    if (best_idx) *best_idx = -1;
    if (n == 0) return PCP_OK;
    if (n > 65535u * (uint64_t)m->n)
        return merr(m, PCP_E_INVALID, "pcp_multi_raycast_fan: too many poses");
    const uint32_t P = (uint32_t)n;
    if (int rc = ensure_keys(m, P)) return rc;
    std::vector<FanEnq> o(m->n);
    std::vector<uint64_t> lo(m->n), cnt(m->n);
    for (int r = 0; r < m->n; ++r) shard(n, m->n, r, lo[r], cnt[r]);
    // every rank enqueued (on its own thread) before waiting on any
    int erc = for_ranks(m, [&](int r) -> int {
        pcp_ctx *c = m->ctx[r];
        if (cnt[r])
            if (int rc = fan_enqueue(c, poses5 + 5 * lo[r], cnt[r], fan, false, false, false, o[r]))
                return rc;
        PCP_HIP(c, hipSetDevice(c->device));
        launch_fan_keys(c->stream, o[r].blocked_d, (uint32_t)lo[r], (uint32_t)cnt[r], P,
                        m->keys[r].as<unsigned long long>());
        PCP_CHECK_LAUNCH(c);
        return PCP_OK;
    });
    if (erc) return erc;
    if (int rc = reduce_keys(m, P, false)) return rc;
    // rank 0's reduced keys and every rank's units into one pinned block
    M_HIP(m, m->host.ensure((size_t)P * 16 + 64));
    unsigned long long *kh = m->host.as<unsigned long long>();
    unsigned long long *uh = kh + P;
    for (int r = 0; r < m->n; ++r) {
        pcp_ctx *c = m->ctx[r];
        M_HIP(m, hipSetDevice(c->device));
        if (r == 0)
            M_HIP(m, hipMemcpyAsync(kh, m->keys[0].p, (size_t)P * 8, hipMemcpyDeviceToHost,
                                    c->stream));
        if (cnt[r])
            M_HIP(m, hipMemcpyAsync(uh + lo[r], o[r].units_d, cnt[r] * 8, hipMemcpyDeviceToHost,
                                    c->stream));
    }
    for (int r = 0; r < m->n; ++r) {
        M_HIP(m, hipSetDevice(m->ctx[r]->device));
        M_HIP(m, hipStreamSynchronize(m->ctx[r]->stream));
        prof_resolve(m->ctx[r]);
    }
    unsigned long long kmin = ~0ull;
    for (uint32_t i = 0; i < P; ++i) {
        blocked[i] = (uint32_t)(kh[i] >> 32);
        if (units) units[i] = uh[i];
        kmin = std::min(kmin, kh[i]);
    }
    if (best_idx) *best_idx = (int64_t)(kmin & 0xffffffffull);
    return PCP_OK;
}

int pcp_multi_score_poses(pcp_multi *m, const double *poses5, uint64_t n,
                          const double zx120_pose5[5], const pcp_vl_params *p,
                          uint8_t *cell_flags, double *total_score, int32_t *covered,
                          pcp_vl_report *rep) {
    if (!m) return PCP_E_INVALID;
    for (int r = 0; r < m->n; ++r)   // (a setup still in flight on a rank: settled first)
        if (area_finish(m->ctx[r]) != PCP_OK)
            return merr(m, PCP_E_HIP, "pcp_multi_score_poses: %s", m->ctx[r]->err.c_str());
    const uint64_t C = m->ctx[0]->n_cells;
    if (!zx120_pose5 || !p || !rep || (n && !poses5) || (C && !cell_flags))
        return merr(m, PCP_E_INVALID, "pcp_multi_score_poses: null argument");
    for (int r = 1; r < m->n; ++r)
        if (m->ctx[r]->n_cells != C)
            return merr(m, PCP_E_STATE, "pcp_multi_score_poses: ranks hold different cells");
    if (n > 65535u * (uint64_t)m->n)
        return merr(m, PCP_E_INVALID, "pcp_multi_score_poses: too many poses");
    const int P = (int)n;
    const size_t count = 2 * (size_t)P + 3 * (size_t)C;
    if (int rc = ensure_keys(m, count)) return rc;
    std::vector<ScoreEnq> o(m->n);
    std::vector<uint64_t> lo(m->n), cnt(m->n);
    for (int r = 0; r < m->n; ++r) shard(n, m->n, r, lo[r], cnt[r]);
    int erc = for_ranks(m, [&](int r) -> int {
        pcp_ctx *c = m->ctx[r];
        if (int rc = score_enqueue(c, poses5 + 5 * lo[r], cnt[r], zx120_pose5, p, o[r])) return rc;
        launch_score_keys(c->stream, o[r], (int)lo[r], P, m->keys[r].as<unsigned long long>());
        PCP_CHECK_LAUNCH(c);
        return PCP_OK;
    });
    if (erc) return erc;
    if (int rc = reduce_keys(m, count, true)) return rc;
    // finalize on rank 0: the caller's flags, the reduced newest-pose keys, the zx120 bits
    pcp_ctx *c0 = m->ctx[0];
    hipStream_t st = c0->stream;
    M_HIP(m, hipSetDevice(c0->device));
    const size_t v_bytes = 2 * (size_t)P * 8, fl_off = (v_bytes + 16 + 15) & ~(size_t)15;
    const size_t st_off = (fl_off + C + 15) & ~(size_t)15;
    M_HIP(m, m->host.ensure(st_off + 64 * sizeof(int32_t) + 64));
    char *pin = m->host.as<char>();
    if (C) {
        std::memcpy(pin + fl_off, cell_flags, C);
        M_HIP(m, hipMemcpyAsync(o[0].flags_d, pin + fl_off, C, hipMemcpyHostToDevice, st));
    }
    M_HIP(m, hipMemsetAsync(o[0].stats, 0, 64 * sizeof(int32_t), st));
    launch_flags_from_keys(st, m->keys[0].as<const unsigned long long>(), o[0].zbits, (int)C, P,
                           o[0].flags_d, o[0].stats);
    M_HIP(m, hipGetLastError());
    if (P) M_HIP(m, hipMemcpyAsync(pin, m->keys[0].p, v_bytes, hipMemcpyDeviceToHost, st));
    // the zx120 total: row cnt[0] of rank 0's totals
    M_HIP(m, hipMemcpyAsync(pin + v_bytes, o[0].tot_d + cnt[0], sizeof(double),
                            hipMemcpyDeviceToHost, st));
    if (C) M_HIP(m, hipMemcpyAsync(pin + fl_off, o[0].flags_d, C, hipMemcpyDeviceToHost, st));
    M_HIP(m, hipMemcpyAsync(pin + st_off, o[0].stats, 64 * sizeof(int32_t),
                            hipMemcpyDeviceToHost, st));
    for (int r = 0; r < m->n; ++r) {
        M_HIP(m, hipSetDevice(m->ctx[r]->device));
        M_HIP(m, hipStreamSynchronize(m->ctx[r]->stream));
        prof_resolve(m->ctx[r]);
    }
    if (C) std::memcpy(cell_flags, pin + fl_off, C);
    const unsigned long long *vh = reinterpret_cast<const unsigned long long *>(pin);
    double zx_total;
    std::memcpy(&zx_total, pin + v_bytes, sizeof(double));
    double best = -INFINITY;
    int64_t best_idx = -1;
    for (int k = 0; k < P; ++k) {   // runOptimization :471-474, first maximum wins
        double t;
        std::memcpy(&t, &vh[k], sizeof(double));
        if (total_score) total_score[k] = t;
        if (covered) covered[k] = (int32_t)vh[P + k];   // (the low 32 bits: kScoreWritten dropped)
        if (t > best) {
            best = t;
            best_idx = k;
        }
    }
    fill_report(reinterpret_cast<const int32_t *>(pin + st_off), zx_total, best_idx, best, rep);
    return PCP_OK;
}

}  // extern "C"
