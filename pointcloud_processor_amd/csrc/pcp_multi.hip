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
// Ranks that share a device (a rehearsal on fewer GPUs than ranks; RCCL refuses duplicate
// devices in one communicator) combine their key vectors on that device instead: same keys,
// same finalization, min / max by a kernel.
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstring>
#include <string>
#include <vector>

#include "pcp_internal.hpp"

using namespace pcp;

struct pcp_multi {
    int n = 0;
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
    std::vector<int> sorted = dev;
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (distinct) {
        m->comm.resize(n_dev);
        if (ncclCommInitAll(m->comm.data(), n_dev, dev.data()) != ncclSuccess) {
            m->comm.clear();
            pcp_multi_destroy(m);
            return PCP_E_HIP;
        }
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

// the index builds run on every device from the host buffer (each takes ~1 ms per 1M points;
// the per-frame state is small next to a collective's setup)
int pcp_multi_set_terrain(pcp_multi *m, const pcp_cloud_view *terrain) {
    if (!m) return PCP_E_INVALID;
    for (int r = 0; r < m->n; ++r)
        if (int rc = pcp_set_terrain(m->ctx[r], terrain)) return from_ctx(m, r, rc);
    return PCP_OK;
}

int pcp_multi_set_aux_cloud(pcp_multi *m, const pcp_cloud_view *aux) {
    if (!m) return PCP_E_INVALID;
    for (int r = 0; r < m->n; ++r)
        if (int rc = pcp_set_aux_cloud(m->ctx[r], aux)) return from_ctx(m, r, rc);
    return PCP_OK;
}

int pcp_multi_set_cells(pcp_multi *m, const double *xyz, const float *normals, uint64_t n) {
    if (!m) return PCP_E_INVALID;
    for (int r = 0; r < m->n; ++r)
        if (int rc = pcp_set_cells(m->ctx[r], xyz, normals, n)) return from_ctx(m, r, rc);
    return PCP_OK;
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
    for (int r = 0; r < m->n; ++r) {   // enqueue every rank before waiting on any
        pcp_ctx *c = m->ctx[r];
        shard(n, m->n, r, lo[r], cnt[r]);
        if (cnt[r]) {
            if (int rc = fan_enqueue(c, poses5 + 5 * lo[r], cnt[r], fan, false, false, false, o[r]))
                return from_ctx(m, r, rc);
        }
        M_HIP(m, hipSetDevice(c->device));
        launch_fan_keys(c->stream, o[r].blocked_d, (uint32_t)lo[r], (uint32_t)cnt[r], P,
                        m->keys[r].as<unsigned long long>());
        M_HIP(m, hipGetLastError());
    }
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
    for (int r = 0; r < m->n; ++r) {
        pcp_ctx *c = m->ctx[r];
        shard(n, m->n, r, lo[r], cnt[r]);
        if (int rc = score_enqueue(c, poses5 + 5 * lo[r], cnt[r], zx120_pose5, p, o[r]))
            return from_ctx(m, r, rc);
        launch_score_keys(c->stream, o[r], (int)lo[r], P, m->keys[r].as<unsigned long long>());
        M_HIP(m, hipGetLastError());
    }
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
        if (covered) covered[k] = (int32_t)vh[P + k];
        if (t > best) {
            best = t;
            best_idx = k;
        }
    }
    fill_report(reinterpret_cast<const int32_t *>(pin + st_off), zx_total, best_idx, best, rep);
    return PCP_OK;
}

}  // extern "C"
