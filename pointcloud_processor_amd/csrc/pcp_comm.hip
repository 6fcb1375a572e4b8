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

#include <cstdio>
#include <cstring>

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

// the shard's fans and its keys on the context's stream, up to (not including) the collective
static int fan_allreduce_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n,
                                 const pcp_fan_params *fan, uint64_t lo, uint32_t P,
                                 double *collective_ms, const unsigned long long **units_out) {
    PCP_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    PCP_HIP(ctx, ctx->comm_keys.ensure((size_t)P * 8 + 64));
    const uint32_t *blocked_d = nullptr;
    if (n) {
        FanEnq o;   // device results (no host landing): the keys kernel reads them
        if (int rc = fan_enqueue(ctx, poses5, n, fan, false, false, false, o)) return rc;
        blocked_d = o.blocked_d;
        *units_out = o.units_d;
    }
    unsigned long long *keys = ctx->comm_keys.as<unsigned long long>();
    launch_fan_keys(st, blocked_d, (uint32_t)lo, (uint32_t)n, P, keys);   // ~0 elsewhere
    PCP_CHECK_LAUNCH(ctx);
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
    if (lo + n > p_total || p_total > 65535u * 64u)
        return set_err(ctx, PCP_E_INVALID,
                       "pcp_raycast_fan_allreduce: shard [%llu, %llu) of %llu poses",
                       (unsigned long long)lo, (unsigned long long)(lo + n),
                       (unsigned long long)p_total);
    if (p_total == 0) return PCP_OK;   // every rank sees the same p_total: no rank reduces
    const uint32_t P = (uint32_t)p_total;
    const unsigned long long *units_d = nullptr;
    // everything before the collective: a failure here would leave the other ranks blocked in
    // ncclAllReduce with no timeout, so it aborts the communicator (their collective then fails
    // instead of hanging) and marks this context's communicator gone
    if (int rc = fan_allreduce_enqueue(ctx, poses5, n, fan, lo, P, collective_ms, &units_d)) {
        (void)ncclCommAbort(static_cast<ncclComm_t>(ctx->comm));
        ctx->comm = nullptr;
        ctx->comm_nranks = 0;
        ctx->comm_rank = 0;
        return rc;
    }
    hipStream_t st = ctx->stream;
    unsigned long long *keys = ctx->comm_keys.as<unsigned long long>();
    PCP_NCCL(ctx, ncclAllReduce(keys, keys, P, ncclUint64, ncclMin,
                                static_cast<ncclComm_t>(ctx->comm), st));   // the one collective
    if (collective_ms) PCP_HIP(ctx, hipEventRecord(ctx->comm_ev[1], st));
    // the reduced vector and this shard's units into one pinned block
    PCP_HIP(ctx, ctx->comm_host.ensure((size_t)(P + n) * 8 + 64));
    unsigned long long *kh = ctx->comm_host.as<unsigned long long>();
    PCP_HIP(ctx, hipMemcpyAsync(kh, keys, (size_t)P * 8, hipMemcpyDeviceToHost, st));
    if (n && units)
        PCP_HIP(ctx, hipMemcpyAsync(kh + P, units_d, n * 8, hipMemcpyDeviceToHost, st));
    PCP_HIP(ctx, hipStreamSynchronize(st));
    prof_resolve(ctx);
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
        for (uint64_t i = 0; i < n; ++i) units[i] = kh[P + i];
    for (uint32_t i = 0; i < P; ++i)   // a slot no rank wrote: the ranks' shards disagree
        if (kh[i] == ~0ull)
            return set_err(ctx, PCP_E_STATE, "pcp_raycast_fan_allreduce: pose %u has no rank "
                                             "(shards do not cover [0, p_total))", i);
    if (best_idx) *best_idx = (int64_t)(kmin & 0xffffffffull);
    return PCP_OK;
}

}  // extern "C"
