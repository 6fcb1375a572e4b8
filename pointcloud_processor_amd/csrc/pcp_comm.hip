// pcp_comm.hip -- one process per GPU: the pose-sharded fan search with libpcp's OWN RCCL
// communicator (bench.py --gpus N).  Host code only.
//
// The caller's framework (torch.distributed over gloo in bench.py) carries nothing but the
// 128-byte ncclUniqueId from rank 0 to the other ranks and the host-side barriers; every byte
// of the data path stays in this library's HIP runtime: the fan kernels, the keys
// (blocked << 32) | global pose written into this context's device vector, ONE
// ncclAllReduce(ncclUint64, ncclMin) over it on the context's stream, and the reduced vector
// back to pinned memory.  The minimum key is the first-minimum argmin of runOptimization's
// candidate loop (virtual_lidar.cpp:467-475): lowest blocked count, ties to the lowest index.
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "pcp_internal.hpp"

using namespace pcp;

namespace pcp {
void comm_release(pcp_ctx *ctx) {
    if (ctx->comm) (void)ncclCommDestroy(static_cast<ncclComm_t>(ctx->comm));
    ctx->comm = nullptr;
    ctx->comm_nranks = 0;
    ctx->comm_rank = 0;
    for (hipEvent_t &e : ctx->comm_ev) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    ctx->comm_keys.release();
    ctx->comm_host.release();
}
}  // namespace pcp

#define PCP_NCCL(ctx, expr)                                                                 \
    do {                                                                                    \
        ncclResult_t _r = (expr);                                                           \
        if (_r != ncclSuccess)                                                              \
            return set_err((ctx), PCP_E_HIP, "%s: %s (%s:%d)", #expr, ncclGetErrorString(_r), \
                           __FILE__, __LINE__);                                             \
    } while (0)

static_assert(sizeof(ncclUniqueId) == PCP_COMM_ID_BYTES, "ncclUniqueId size");

// Every rank reaches the collective, whatever happened before it.  RCCL has no timeout: a rank
// that returned early would leave the others blocked inside ncclAllReduce (ncclCommAbort frees
// only the calling rank's resources; the peers would wait until the launcher kills them).  So
// the reduced vector carries one HEALTH word at its end: a healthy rank writes the reduction's
// identity there (MIN: ~0, MAX: 0), a rank whose work before the collective failed fills its
// whole vector with the absorbing value (MIN: 0, MAX: ~0) and still runs the collective.
// Afterwards every rank sees the failure in that word and returns PCP_E_STATE; the failing
// rank returns its own error.  Only when even the poison cannot be enqueued (no vector, a
// dead stream) does the rank abort its communicator, and the launcher's kill-on-failure is
// then what releases the others.
static void comm_drop(pcp_ctx *ctx) {
    (void)ncclCommAbort(static_cast<ncclComm_t>(ctx->comm));
    ctx->comm = nullptr;
    ctx->comm_nranks = 0;
    ctx->comm_rank = 0;
}

// the failed rank's vector: count words of the absorbing value, on the context's stream
static bool comm_poison(pcp_ctx *ctx, size_t count, bool is_max) {
    if (hipSetDevice(ctx->device) != hipSuccess) return false;
    if (ctx->comm_keys.ensure(count * 8 + 64) != hipSuccess) return false;
    return hipMemsetAsync(ctx->comm_keys.p, is_max ? 0xff : 0x00, count * 8, ctx->stream) ==
           hipSuccess;
}

// the shard's fans and its keys on the context's stream, up to (not including) the collective
static int fan_allreduce_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n,
                                 const pcp_fan_params *fan, uint64_t lo, uint32_t P,
                                 double *collective_ms, const unsigned long long **units_out) {
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // [P + 1 keys (the reduced span) | this shard's n unit counts]: one landing copy afterwards
    PCP_HIP(ctx, ctx->comm_keys.ensure((size_t)(P + 1 + n) * 8 + 64));
    unsigned long long *keys = ctx->comm_keys.as<unsigned long long>();
    if (n) {
        // k_fan_reduce writes the vector itself: the shard's keys, ~0 in the other ranks' slots
        // and in the health word (slot P: no pose of any shard), the units behind it
        FanEnq o;
        o.keys = keys;
        o.keys_lo = (uint32_t)lo;
        o.keys_P = P;
        if (int rc = fan_enqueue(ctx, poses5, n, fan, false, false, false, o)) return rc;
        *units_out = o.units_d;
    } else {   // no poses here: the identity everywhere
        launch_fan_keys(st, nullptr, (uint32_t)lo, 0u, P + 1, keys);
        PCP_CHECK_LAUNCH(ctx);
    }
    if (collective_ms)
        for (hipEvent_t &e : ctx->comm_ev)
            if (!e) PCP_HIP(ctx, hipEventCreate(&e));
    if (collective_ms) PCP_HIP(ctx, hipEventRecord(ctx->comm_ev[0], st));
    return PCP_OK;
}

extern "C" {

int pcp_comm_unique_id(uint8_t id[PCP_COMM_ID_BYTES]) {
    if (!id) return PCP_E_INVALID;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return PCP_E_HIP;
    std::memcpy(id, &u, sizeof(u));
    return PCP_OK;
}

int pcp_comm_init_rank(pcp_ctx *ctx, int nranks, const uint8_t id[PCP_COMM_ID_BYTES], int rank) {
    if (!ctx) return PCP_E_INVALID;
    if (!id || nranks <= 0 || rank < 0 || rank >= nranks)
        return set_err(ctx, PCP_E_INVALID, "pcp_comm_init_rank: rank %d of %d", rank, nranks);
    if (ctx->comm) return set_err(ctx, PCP_E_STATE, "pcp_comm_init_rank: already initialised");
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t c = nullptr;
    PCP_NCCL(ctx, ncclCommInitRank(&c, nranks, u, rank));
    ctx->comm = c;
    ctx->comm_nranks = nranks;
    ctx->comm_rank = rank;
    return PCP_OK;
}

int pcp_comm_info(const pcp_ctx *ctx, int *nranks, int *rank) {
    if (!ctx) return PCP_E_INVALID;
    if (nranks) *nranks = ctx->comm ? ctx->comm_nranks : 0;
    if (rank) *rank = ctx->comm ? ctx->comm_rank : 0;
    return PCP_OK;
}

int pcp_get_runtime_info(pcp_runtime_info *info) {
    if (!info) return PCP_E_INVALID;
    std::memset(info, 0, sizeof(*info));
    int v = 0;
    if (hipRuntimeGetVersion(&v) == hipSuccess) info->hip_runtime_version = v;
    v = 0;
    if (ncclGetVersion(&v) == ncclSuccess) info->rccl_version = v;
    Dl_info d;
    hipError_t (*hip_malloc)(void **, size_t) = &hipMalloc;
    if (dladdr(reinterpret_cast<const void *>(hip_malloc), &d) && d.dli_fname)
        std::snprintf(info->hip_path, sizeof(info->hip_path), "%s", d.dli_fname);
    if (dladdr(reinterpret_cast<const void *>(&ncclAllReduce), &d) && d.dli_fname)
        std::snprintf(info->rccl_path, sizeof(info->rccl_path), "%s", d.dli_fname);
    return PCP_OK;
}

int pcp_raycast_fan_allreduce(pcp_ctx *ctx, const double *poses5, uint64_t n,
                              const pcp_fan_params *fan, uint64_t lo, uint64_t p_total,
                              uint32_t *blocked_all, uint64_t *units, int64_t *best_idx,
                              double *collective_ms) {
    if (!ctx) return PCP_E_INVALID;
    if (best_idx) *best_idx = -1;
    if (!ctx->comm)
        return set_err(ctx, PCP_E_STATE, "pcp_raycast_fan_allreduce: no communicator "
                                         "(pcp_comm_init_rank)");
    if (!fan || (n && !poses5))
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan_allreduce: null argument");
    // (every rank sees the same p_total: a bad one fails on every rank and none reduces)
    if (p_total > 65535u * 64u)
        return set_err(ctx, PCP_E_INVALID, "pcp_raycast_fan_allreduce: %llu poses",
                       (unsigned long long)p_total);
    if (p_total == 0) return PCP_OK;
    const uint32_t P = (uint32_t)p_total;
    const unsigned long long *units_d = nullptr;   // (the shard's units: k_fan_reduce also puts
                                                   // them behind the health word, landed below)
    // everything before the collective; a failure poisons this rank's vector (health word 0)
    int rc = PCP_OK;
    if (lo + n > p_total)
        rc = set_err(ctx, PCP_E_INVALID,
                     "pcp_raycast_fan_allreduce: shard [%llu, %llu) of %llu poses",
                     (unsigned long long)lo, (unsigned long long)(lo + n),
                     (unsigned long long)p_total);
    else
        rc = fan_allreduce_enqueue(ctx, poses5, n, fan, lo, P, collective_ms, &units_d);
    if (rc) {
        const std::string why = ctx->err;
        if (!comm_poison(ctx, (size_t)P + 1, false)) {
            comm_drop(ctx);
            return set_err(ctx, rc, "%s", why.c_str());
        }
        collective_ms = nullptr;
        units = nullptr;
    }
    hipStream_t st = ctx->stream;
    unsigned long long *keys = ctx->comm_keys.as<unsigned long long>();
    PCP_NCCL(ctx, ncclAllReduce(keys, keys, (size_t)P + 1, ncclUint64, ncclMin,
                                static_cast<ncclComm_t>(ctx->comm), st));   // the one collective
    if (collective_ms) PCP_HIP(ctx, hipEventRecord(ctx->comm_ev[1], st));
    // the reduced vector (+ health word) and this shard's units (behind it in the same device
    // vector) into one pinned block by ONE copy kernel
    PCP_HIP(ctx, ctx->comm_host.ensure((size_t)(P + 1 + n) * 8 + 64));
    unsigned long long *kh = ctx->comm_host.as<unsigned long long>();
    if (int rcc = copy_to_pinned_async(ctx, kh, keys, (size_t)(P + 1 + (n && units ? n : 0)) * 8, st))
        return rcc;
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
    if (rc) return rc;   // (ctx->err: this rank's own failure, set before the poison)
    if (kh[P] != ~0ull)
        return set_err(ctx, PCP_E_STATE, "pcp_raycast_fan_allreduce: a peer rank failed before "
                                         "the collective (health word poisoned)");
    if (collective_ms) {
        float ms = 0.0f;
        PCP_HIP(ctx, hipEventElapsedTime(&ms, ctx->comm_ev[0], ctx->comm_ev[1]));
        *collective_ms = ms;
    }
    unsigned long long kmin = ~0ull;
    for (uint32_t i = 0; i < P; ++i) {
        if (blocked_all) blocked_all[i] = (uint32_t)(kh[i] >> 32);
        kmin = kh[i] < kmin ? kh[i] : kmin;
    }
    if (units)
        for (uint64_t i = 0; i < n; ++i) units[i] = kh[P + 1 + i];
    for (uint32_t i = 0; i < P; ++i)   // a slot no rank wrote: the ranks' shards disagree
        if (kh[i] == ~0ull)
            return set_err(ctx, PCP_E_STATE, "pcp_raycast_fan_allreduce: pose %u has no rank "
                                             "(shards do not cover [0, p_total))", i);
    if (best_idx) *best_idx = (int64_t)(kmin & 0xffffffffull);
    return PCP_OK;
}

// runOptimization's scoring for N processes (virtual_lidar.cpp:460-519): this rank's shard
// scored as pcp_multi_score_poses scores a rank's (k_score_cells + k_row_sum, then the keys:
// k_score_keys), ONE ncclAllReduce(ncclUint64, ncclMax) over [P totals | P covered | 3 x C
// newest-pose flag keys | health], then every rank resolves the stale flags from the reduced
// keys (k_flags_from_keys) and runs the strict-'>' argmax on the host
int pcp_score_poses_allreduce(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                              const pcp_vl_params *p, uint64_t lo, uint64_t p_total,
                              uint8_t *cell_flags, double *total_all, int32_t *covered_all,
                              pcp_vl_report *rep, double *collective_ms) {
    if (!ctx) return PCP_E_INVALID;
    if (!ctx->comm)
        return set_err(ctx, PCP_E_STATE, "pcp_score_poses_allreduce: no communicator "
                                         "(pcp_comm_init_rank)");
    if (!zx || !p || !rep)   // (every rank passes the same kind of arguments)
        return set_err(ctx, PCP_E_INVALID, "pcp_score_poses_allreduce: null argument");
    if (p_total > 65535u * 64u)
        return set_err(ctx, PCP_E_INVALID, "pcp_score_poses_allreduce: %llu poses",
                       (unsigned long long)p_total);
    int rc = area_finish(ctx);   // (the cells' count sizes the vector: every rank holds the same)
    const uint64_t C = ctx->n_cells;
    const uint32_t P = (uint32_t)p_total;
    const size_t count = 2 * (size_t)P + 3 * (size_t)C + 1, hw = count - 1;
    ScoreEnq o;
    hipStream_t st = ctx->stream;
    if (!rc) {
        if ((n && !poses5) || (C && !cell_flags))
            rc = set_err(ctx, PCP_E_INVALID, "pcp_score_poses_allreduce: null argument");
        else if (lo + n > p_total || n > 65535)
            rc = set_err(ctx, PCP_E_INVALID,
                         "pcp_score_poses_allreduce: shard [%llu, %llu) of %llu poses",
                         (unsigned long long)lo, (unsigned long long)(lo + n),
                         (unsigned long long)p_total);
    }
    auto enqueue = [&]() -> int {
        PCP_HIP(ctx, hipSetDevice(ctx->device));
        PCP_HIP(ctx, ctx->comm_keys.ensure(count * 8 + 64));
        // (the caller's flags ride in the query's one upload: k_flags_from_keys updates them)
        if (int e = score_enqueue(ctx, poses5, n, zx, p, o, C ? cell_flags : nullptr)) return e;
        unsigned long long *v = ctx->comm_keys.as<unsigned long long>();
        launch_score_keys(st, o, (int)lo, (int)P, v);
        PCP_CHECK_LAUNCH(ctx);
        PCP_HIP(ctx, hipMemsetAsync(v + hw, 0, 8, st));   // health: MAX's identity
        if (collective_ms) {
            for (hipEvent_t &e : ctx->comm_ev)
                if (!e) PCP_HIP(ctx, hipEventCreate(&e));
            PCP_HIP(ctx, hipEventRecord(ctx->comm_ev[0], st));
        }
        return PCP_OK;
    };
    if (!rc) rc = enqueue();
    if (rc) {
        const std::string why = ctx->err;
        if (!comm_poison(ctx, count, true)) {
            comm_drop(ctx);
            return set_err(ctx, rc, "%s", why.c_str());
        }
        collective_ms = nullptr;
    }
    unsigned long long *v = ctx->comm_keys.as<unsigned long long>();
    PCP_NCCL(ctx, ncclAllReduce(v, v, count, ncclUint64, ncclMax,
                                static_cast<ncclComm_t>(ctx->comm), st));   // the one collective
    if (collective_ms) PCP_HIP(ctx, hipEventRecord(ctx->comm_ev[1], st));
    // pinned: [2P keys | zx120 total | health | C flags | 64 stats]
    const size_t v_bytes = 2 * (size_t)P * 8, fl_off = (v_bytes + 16 + 15) & ~(size_t)15;
    const size_t st_off = (fl_off + C + 15) & ~(size_t)15;
    PCP_HIP(ctx, ctx->comm_host.ensure(st_off + 64 * sizeof(int32_t) + 64));
    char *pin = ctx->comm_host.as<char>();
    if (rc) {   // the failed rank only completes its collective
        PCP_HIP(ctx, hipStreamSynchronize(st));
        return set_err(ctx, rc, "%s", ctx->err.c_str());
    }
    // the statistics were zeroed by k_score_cells (C > 0; else k_score_enqueue's memset), the
    // caller's flags uploaded with the poses: resolve, then ONE landing kernel for everything
    // the host reads -- the zx120 total is row n of this rank's totals (every rank evaluates it)
    launch_flags_from_keys(st, v, o.zbits, (int)C, (int)P, o.flags_d, o.stats);
    PCP_CHECK_LAUNCH(ctx);
    launch_score_land(st, v, (int)P, hw, o.tot_d + n, o.flags_d, (int)C, o.stats, pin, fl_off,
                      st_off);
    PCP_CHECK_LAUNCH(ctx);
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
    unsigned long long health;
    std::memcpy(&health, pin + v_bytes + 8, 8);
    if (health != 0)
        return set_err(ctx, PCP_E_STATE, "pcp_score_poses_allreduce: a peer rank failed before "
                                         "the collective (health word poisoned)");
    const unsigned long long *vh = reinterpret_cast<const unsigned long long *>(pin);
    for (uint32_t k = 0; k < P; ++k)   // (cell_flags untouched: the query did not complete)
        if (!(vh[P + k] & kScoreWritten))
            return set_err(ctx, PCP_E_STATE, "pcp_score_poses_allreduce: pose %u of %u was "
                                             "scored by no rank", k, P);
    if (collective_ms) {
        float ms = 0.0f;
        PCP_HIP(ctx, hipEventElapsedTime(&ms, ctx->comm_ev[0], ctx->comm_ev[1]));
        *collective_ms = ms;
    }
    if (C) std::memcpy(cell_flags, pin + fl_off, C);
    double zx_total;
    std::memcpy(&zx_total, pin + v_bytes, sizeof(double));
    double best = -INFINITY;
    int64_t best_idx = -1;
    for (uint32_t k = 0; k < P; ++k) {   // runOptimization :471-474, the first maximum wins
        double t;
        std::memcpy(&t, &vh[k], sizeof(double));
        if (total_all) total_all[k] = t;
        if (covered_all) covered_all[k] = (int32_t)vh[P + k];
        if (t > best) {
            best = t;
            best_idx = k;
        }
    }
    fill_report(reinterpret_cast<const int32_t *>(pin + st_off), zx_total, best_idx, best, rep);
    return PCP_OK;
}

}  // extern "C"
