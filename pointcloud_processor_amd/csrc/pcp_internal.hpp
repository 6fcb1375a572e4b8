// pcp_internal.hpp -- shared host/device declarations of libpcp (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "pcp_abi.h"

namespace pcp {
struct CopyPool;

// ---------------------------------------------------------------------------------------
// reference constants (virtual_lidar.cpp:100-114)
// ---------------------------------------------------------------------------------------
constexpr double kPi = 3.14159265358979323846;
constexpr double kMinDistance = 0.5;
constexpr double kRayStep = 0.3;
constexpr double kVisRadius = 0.08;
constexpr double kRayRadius = kVisRadius * 0.7;     // radiusSearch radius at :782
constexpr double kRelaxedRadius = kVisRadius * 3.0; // :743
constexpr double kMinElevation = -85.0 * kPi / 180.0;
constexpr double kMaxElevation = 85.0 * kPi / 180.0;
constexpr double kCellMargin = 4e-3;   // conservative margin of the stencil
constexpr double kQueryMargin = 1e-3;

// ---------------------------------------------------------------------------------------
// device buffer (grow-only).  A buffer that must grow is reallocated with 25 % headroom (and at
// least 64 KiB): a hipFree synchronizes the whole device, so a per-frame chain whose sizes
// wander (C5) must converge to few reallocations instead of one per new maximum.  Every
// reallocation is counted process-wide (pcp_alloc_stats).
// ---------------------------------------------------------------------------------------
void note_realloc(size_t bytes, bool pinned);
uint64_t alloc_count(int which);   // 0 device, 1 pinned reallocations, 2 bytes allocated

constexpr size_t kHeadroomMax = 16u << 20;   // first allocations below this get +25 %

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        const bool grow = cap != 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 256 ? 256 : bytes;
        // message-sized buffers start with the headroom a growth would add: streamed clouds
        // vary by a few percent frame to frame, and each growth is a free + malloc in a frame
        if (grow || want < kHeadroomMax) want = std::max<size_t>(want + want / 4, 64u << 10);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        note_realloc(want, false);
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// pinned (page-locked) host staging buffer (grow-only, same growth rule): small per-call H2D /
// D2H transfers from it skip the runtime's pageable staging copy
struct PinnedBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        const bool grow = cap != 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 4096 ? 4096 : bytes;
        if (grow || want < kHeadroomMax) want = std::max<size_t>(want + want / 4, 64u << 10);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        note_realloc(want, true);
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// ---------------------------------------------------------------------------------------
// Uniform-grid spatial index (replaces pcl::KdTreeFLANN).  Points sorted by cell, cell
// start offsets (prefix sum, ncell+1 entries), and a dilated occupancy bitmask: bit of
// cell c = any point in the 2x2x2 block whose lower corner is c.  Cells are padded by one
// on every side so that a stencil whose lower corner falls outside [0, n-2] is provably
// empty.  See DESIGN.md "Terrain index".
// ---------------------------------------------------------------------------------------
struct GridView {               // POD passed to kernels by value
    const float4 *pts;          // x, y, z, bitcast(original index)
    const uint32_t *start;      // ncell + 1
    const uint32_t *occ2;       // dilated occupancy bits, (ncell + 31) / 32 words
    double ox, oy, oz;          // origin (lower corner of cell 0)
    double inv_c, c;
    double lo_x, lo_y, lo_z;    // origin + r_q + margin (stencil lower corner offset)
    int32_t nx, ny, nz;
    uint32_t n_pts;
    // tight bbox of the points, inflated by r_q + margin: samples outside are empty
    double bx0, bx1, by0, by1, bz0, bz1;
    // float copies for the stencil-corner and clip arithmetic: their rounding (~1e-5 m) stays
    // far inside the 1 mm query margin, so the skips remain exact (Terrain index)
    float flo_x, flo_y, flo_z, finv_c;
    float fnx1, fny1, fnz1;     // n - 1 per axis
    float fb[6];                // clip box x0, x1, y0, y1, z0, z1
    // z band of each stencil corner's 2x2x2 block (z-sorted indices only, else null): u16 =
    // lo | hi << 8, the block's lowest / highest point z as conservative steps of kZq cells
    // above the block's floor (lo 0 = unbounded below, hi 255 = unbounded above; lo > hi =
    // empty block).  fzoff = (r_q + m) / c (stencil-corner offset), fzt = (r_q + 2 mm) / c.
    const uint16_t *occz;
    float fzoff, fzt;
    // block-major copy (null unless built): the points of each stencil corner's 2x2x2 block in
    // one run, descending z -- bpts[bstart[lin] .. bstart[lin + 1]); one directory load and one
    // early exit per scan instead of 4 + 8
    const uint32_t *bstart;
    const float4 *bpts;
    // fine-window copy (null unless built, pcp_fine.hip): fine cells of c / F
    // in x, y (F = ffine); the window of fine cell W = the points within r + m (xy) of W's
    // rectangle, one run in descending z ended by a sentinel, wpts.  One record per (fine cell
    // x, y, coarse corner z), x-fastest, frx x fry x frz (frz = nz - 1): {walk start, probe
    // thresholds lo | hi << 8} for the window's points in coarse z cells iz, iz + 1 -- the
    // march's probe and the scan's directory in one load.  fus_off = fzoff / kZq: the probe's
    // sample height above the block floor in kZq steps is frac(fz) / kZq + fus_off.
    const uint2 *frec;
    const float4 *wpts;
    uint32_t frx, fry, frz;
    float fus_off, ffine;
    int32_t ftile;              // records in 4 x 4 xy tiles (1) or split (2), PCP_FINE_TILE
    // ftile 2: the record split in two arrays of 8 x 8 xy tiles -- the probe's 2-byte
    // thresholds (one 128-byte line per tile) and the 4-byte walk start, read by candidates only
    const uint16_t *fband;
    const uint32_t *fstart;     // fskip 1: walk start (28 bits) | skip (4 bits, << 28): entries
                                // of the run at or above oz + (iz + 1.5) c, skipped by a
                                // candidate whose q lies more than r below that height; fskip 2:
                                // start (25 bits) | skips at iz + 1.375 (4 bits, << 25) and
                                // iz + 1.6875 (3 bits, << 29)
    int32_t fskip;
    float fzc, fzo;             // c and oz in float (the skip test)
    int32_t wpack;              // wpts entries packed to 12 bytes (x, y, z), PCP_FINE_PACK
};
constexpr float kZq = 2.0f / 250.0f;   // z band step, cells (2 cells = 250 steps)

struct GridIndex {
    bool present = false;        // a tree exists (KdTreeFLANN::Ptr non-null)
    uint64_t n_pts = 0;
    double r_q = 0.0;            // stencil radius the cell edge was sized for
    double c = 0.0;
    int32_t nx = 0, ny = 0, nz = 0;
    double bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
    DevBuf pts, start, occ2, occz, bstart, bpts, frec, wpts;
    bool occz_ok = false;
    bool blk_ok = false;         // block-major copy built (bstart / bpts)
    bool blk_fail = false;       // copy unavailable for this index (size cap or allocation
                                 // failure): the scans keep the per-cell runs, no retry
    bool fine_ok = false;        // fine-window copy built (frec / wpts)
    bool fine_fail = false;      // fine copy past its caps / not allocated: no retry
    uint32_t frx = 0, fry = 0, frz = 0;
    int32_t wpack = 0;           // wpts as 12-byte (x, y, z) entries
    float ffine = 0.0f;
    int32_t ftile = 0;
    int32_t fskip = 1;           // walk-start skip thresholds (PCP_FINE_SKIP)
    size_t fstart_off = 0;       // ftile 2: byte offset of the start array inside frec
    bool occ2_ok = false;        // occ2 built (only indices queried by stencil_any need it)
    GridView view() const;
    void release() {
        pts.release();
        start.release();
        occ2.release();
        occz.release();
        bstart.release();
        bpts.release();
        frec.release();
        wpts.release();
        occz_ok = false;
        blk_ok = false;
        blk_fail = false;
        fine_ok = false;
        fine_fail = false;
        occ2_ok = false;
        present = false;
        n_pts = 0;
    }
};

// ---------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------
struct ProfSlot {
    double total_ms = 0.0;
    uint64_t launches = 0;
};

struct CloudBufs {                 // one cloud's filter-pipeline scratch
    DevBuf xyz, idx, keys[2], sparse, sparse_idx, hist, out;
    DevBuf skeys;                  // the fast chain: crop tiles' keys + digit-0 rows
    void release() {
        skeys.release();
        xyz.release();
        idx.release();
        for (int q = 0; q < 2; ++q) keys[q].release();
        sparse.release();
        sparse_idx.release();
        hist.release();
        out.release();
    }
};

struct PendingEvent {
    int kid;
    hipEvent_t a, b;
};

}  // namespace pcp

struct pcp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // virtual_lidar state
    pcp::GridIndex terrain;      // raycast index (r_q = 0.056)
    uint64_t terrain_cloud_n = 0;  // current terrain cloud size (stale-tree semantics)
    pcp::GridIndex aux;          // zx120 cloud index (r_q = 0.24)
    uint64_t aux_cloud_n = 0;
    uint64_t n_cells = 0;
    pcp::DevBuf cells_xyz, cells_nrm;
    pcp::DevBuf cells_n_d;           // the lattice's cell count on the device (k_lattice_compact)
    // pcp_set_excavation_area_async: the setup enqueued and not waited for; area_finish (the
    // next call that needs the cells on the host, or the tick after its own synchronisation)
    // settles the count and regrows + reruns the neighbour lists on an overflow
    bool area_pending = false;
    uint64_t cells_cap = 0;          // the lattice's points: an upper bound of n_cells
    uint32_t area_npts = 0, area_grid_a = 0, area_grid_c = 0;
    uint64_t area_total = 0;
    pcp::PinnedBuf area_host;        // the setup's landing: [cells, area list use, cell list use,
                                     // overflow, pool cursors]
    // the async setup's normals + lattice on a stream of their own (PCP_AREA_STREAM, default 1):
    // forked from ctx->stream after the indices, joined by the scoring (score_enqueue) or by
    // area_finish, so the terrain / zx120 index builds in between overlap the neighbour lists
    bool area_side = true;
    bool area_forked = false;        // side work enqueued and not yet joined into ctx->stream
    hipStream_t area_stream = nullptr;
    hipEvent_t area_fork_ev = nullptr, area_join_ev = nullptr;
    pcp::DevBuf lat_flags;           // the lattice's per-point flags (k_lattice_flags)
    // pcp_filter_merge_nodes' outputs in tc_host (pcp_filter_merge_landed), until tc_host's
    // next writer
    bool fm_land_valid = false;
    int fm_land_k = 0;
    const void *fm_land_merged = nullptr;
    std::vector<const float *> fm_land_filtered;
    pcp::PinnedBuf exc_land;
    // pcp_excavate_area_async called with null outputs: its records left in exc_land
    // (pcp_excavate_landed), until the next pcp_excavate* call
    bool exc_keep_valid = false;
    const void *exc_keep_terr = nullptr, *exc_keep_area = nullptr;
    // the carve's four counters, two sets used in turn: each call's k_gen_emit clears the set
    // the next call uses (no memset launch in front of it)
    pcp::DevBuf carve_ctr;
    int carve_ctr_sel = 0;
    bool carve_ctr_clean[2] = {false, false};         // pcp_excavate_area_async: the carve's records, read in place
                                     // by the setup + terrain index it enqueues
    // excavation area (pcp_set_excavation_area): indices for the normal radius (1.5 m) and the
    // lattice test radius (1.5 * grid_resolution), and the per-point normals
    pcp::GridIndex exc_norm, exc_near;
    pcp::DevBuf area_nrm;
    uint64_t area_n = 0;
    // the normals in the reference's summation order (PCP_NORMALS_EXACT, default 1; 0: the
    // order-free fixed-point kernels, A/B only): sorted neighbour lists, their per-query
    // {base, count}, cursors + overflow word; list entries the last call needed
    bool normals_exact = true;       // PCP_NORMALS_EXACT=0: round 3's order-free normals (A/B)
    bool score_wide = true;          // k_score_cells_wide for few-ray launches (PCP_SCORE_WIDE=0: A/B)
    int64_t score_wide_rays = -1;    // PCP_SCORE_WIDE_RAYS: rays up to which it runs (A/B; -1: default)
    int score_wide_g = 0;            // PCP_SCORE_WIDE_G: its lanes per ray, 2 / 4 / 8 / 16 (A/B; 0: default)
    bool cells_all_ordered = false;  // PCP_CELLS_ORDER_FREE=0: every cell through the lists (A/B)
    int nb_blocks = 0;               // PCP_NB_BLOCKS: k_nb_lists grid (A/B; 0 = kNbBlocks)
    bool nb_small = true;            // PCP_NB_SMALL=0: 32-bit list keys below 2^16 points too (A/B)
    int nb_region_pct = 75;          // PCP_NB_REGION_PCT: list words in the blocks' regions (rest: spill pool)
    uint64_t nb_guess_max = 64ull << 20;   // PCP_NB_GUESS_WORDS: cap of a first list buffer (words)
    pcp::DevBuf nb_list, nb_meta, nb_ctl, nb_pts;   // nb_pts: input points by index
    pcp::DevBuf nb_list_c, nb_meta_c;                // the cells' lists
    pcp::DevBuf nb_sel;                              // cells left to the ordered path
    uint64_t nb_need_c = 0;
    bool nb_ctl_zero = false;                // nb_ctl's cursors known zero (cleared by the last call)
    uint64_t nb_need = 0;
    uint64_t normals_regrown = 0;
    // excavated-terrain carve (pcp_excavate): index of the input cloud + scratch
    pcp::GridIndex carve;
    pcp::DevBuf carve_buf;
    // the index builds' per-cell counters: all zero between builds (the build's scan clears what
    // it counted), so no build zeroes them; cell_cnt_dirty marks a build that stopped between
    // its count and its scan (the next one clears the buffer first)
    pcp::DevBuf cell_cnt;
    bool cell_cnt_dirty = false;
    pcp::DevBuf cell_cnt2;           // the second grid's counters of build_index_pair
    bool cell_cnt2_dirty = false;
    bool index_pair = true;          // PCP_INDEX_PAIR=0: the area's two grids by two builds (A/B)
    // the generated lattice (surface + area records, their height queries) on the device:
    // [GenPoint surf | GenPoint area | queries (G generated + n input) | area records].  It
    // depends on the parameters and the excavation pose alone; while carve_key matches, the
    // next call neither regenerates nor uploads it
    pcp::DevBuf carve_gen;
    double carve_key[16] = {};
    bool carve_gen_ok = false;
    uint32_t carve_G = 0;
    uint64_t carve_nsurf = 0, carve_narea = 0;
    // scratch
    pcp::DevBuf stage, scratch[8];
    pcp::DevBuf fan_tab, poses_d, steps_d, out_a, out_b, out_c, out_d, stats_d;
    pcp::PinnedBuf fan_host;                 // pinned staging of poses in / counts out
    pcp::PinnedBuf res_host;                 // pinned landing of the filter chain's sizes
    pcp::PinnedBuf fm_res_host;              // pcp_filter_merge's result sizes, stored by its
                                             // kernels themselves (fixed: a graph holds it)
    pcp::PinnedBuf small_host;               // pinned landing of small size readbacks
    // pcp_raycast_fan_keys: the query's completion (a caller's stream waits on it) -- the next
    // query waits for it before it reuses the pinned pose staging
    hipEvent_t keys_ev = nullptr;
    bool keys_pending = false;
    // one process per GPU (pcp_comm_init_rank): this rank's RCCL communicator (an ncclComm_t),
    // the key vector its collective reduces and the pinned landing of the reduced vector
    void *comm = nullptr;
    int comm_nranks = 0, comm_rank = 0;
    pcp::DevBuf comm_keys;
    pcp::PinnedBuf comm_host;
    hipEvent_t comm_ev[2] = {};
    // pinned upload ring (upload_async): host bytes copied here, then a stream-ordered DMA
    static constexpr int kUpRing = 4;
    pcp::PinnedBuf up_buf[kUpRing];
    hipEvent_t up_ev[kUpRing] = {};
    bool up_used[kUpRing] = {};
    int up_next = 0;
    int pin_held = -1;                       // ring slot held by pin_stage until pin_release
    bool copy_kernel = true;                 // pinned -> device uploads by a copy kernel on the
                                             // stream (PCP_COPY_KERNEL; 0: DMA)
    bool zc_in = true;                       // message-sized inputs read in place from pinned
                                             // memory (PCP_ZC_IN; 0: DMA'd first)
    pcp::PinnedBuf tc_host;                  // transform_concat / carve: records stored by the
                                             // kernels straight into pinned memory
    pcp::PinnedBuf cand_host;                // generate_candidates: poses + count in one readback
    // host copies of message-sized buffers split over helper threads (pcp_hostcopy.hip,
    // PCP_COPY_THREADS, default 3; 0: plain memcpy)
    int copy_threads = 3;
    // exclusive_scan_u32's one-pass form (PCP_SCAN_ONEPASS, default 1): the tiles' status words
    // (value | epoch, flag) and the ticket that orders the tiles; epoch = the call's number
    bool scan_onepass = true;
    pcp::DevBuf scan_state;
    uint32_t scan_epoch = 0, scan_ticket = 0;
    pcp::CopyPool *copy_pool = nullptr;
    pcp::PinnedBuf cv_host;                  // pcp_crop_voxel's fast chain: centroids + result
                                             // sizes stored by the kernels (one round trip)
    int32_t fan_naz = -1, fan_nel = -1;      // cached fan direction tables
    double fan_elmin = 0.0, fan_elmax = 0.0;
    double steps_end = -1e300;               // cached step table
    int steps_K = 0;
    int num_cus = 256;                       // multiprocessors of the device
    int fan_batch = 0;                       // fan kernel variant (PCP_FAN_BATCH), A/B only
    int fan_npw = 8;                         // poses per wave of the fan kernel (PCP_FAN_NPW)
    bool fan_host_out = true;                // k_fan_reduce stores into the pinned landing
                                             // block, no D2H copy (PCP_FAN_HOST_OUT)
    int fm_fast = 2;                         // pcp_filter_merge's voxel chain (PCP_FM_FAST): 2 the
                                             // bucket chain, 1 the LSD fast chain, 0 the general one
    pcp::DevBuf bk_stat;                     // the bucket chain's per-bucket words
    int bk_gt = 0;                           // crop tiles per k_bk_group group (PCP_BK_GT; 0: one
                                             // round of blocks)
    bool carve_fuse_copy = true;             // the composed carve's records copied by its
                                             // index's extraction (PCP_CARVE_FUSE_COPY)
    bool scan_pair = true;                   // a grid pair's two one-tile scans in one launch
                                             // (PCP_SCAN_PAIR)
    int bk_pts = 512;                        // bucket chain: input points per bucket at least
                                             // (PCP_BK_PTS; 0: buckets from the voxel count only)
    bool fm_host_out = true;                 // pcp_filter_merge's result sizes stored by its
                                             // kernels into pinned memory (PCP_FM_HOST_OUT)
    int terrain_blocks = 1;                  // block-major terrain copy (PCP_TERRAIN_BLOCKS)
    int fine_pack = 1;                       // fine-window entries as 12 bytes (PCP_FINE_PACK)
    int fine_skip = 2;                       // split records' skip thresholds: 1 or 2
    int fine_tile = 2;                       // fine records: 0 x-fastest, 1 4 x 4 tiles, 2 split
                                             // in 8 x 8 tiles (PCP_FINE_TILE)
    int terrain_fine = 2;                    // fine-window layout of that copy, cells of c / F
                                             // (PCP_TERRAIN_FINE = F; 0: the 2x2x2 blocks)
    int terrain_queries = 0;                 // queries since the last pcp_set_terrain
    // filter/merge scratch
    pcp::DevBuf f_in, f_misc;
    std::vector<pcp::CloudBufs> fbuf;        // per-cloud scratch of the filter pipeline
    // captured filter_merge pipeline (device-resident inputs), replayed while its key matches
    hipGraph_t fm_graph = nullptr;
    hipGraphExec_t fm_exec = nullptr;
    std::vector<uint8_t> fm_key;
    bool capturing = false;
    bool use_graphs = true;
    // profiling
    bool prof = false;
    pcp::ProfSlot slots[PCP_K_COUNT];
    std::vector<pcp::PendingEvent> pending;
    std::vector<hipEvent_t> event_pool;
};

namespace pcp {

// error helpers --------------------------------------------------------------------------
int set_err(pcp_ctx *ctx, int code, const char *fmt, ...);
int hip_fail(pcp_ctx *ctx, hipError_t e, const char *what, const char *file, int line);

#define PCP_HIP(ctx, expr)                                                       \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) return ::pcp::hip_fail((ctx), _e, #expr, __FILE__, __LINE__); \
    } while (0)

#define PCP_CHECK_LAUNCH(ctx) PCP_HIP(ctx, hipGetLastError())

// profiling: bracket launches on ctx->stream
struct ProfScope {
    pcp_ctx *ctx;
    int kid;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(pcp_ctx *c, int k, hipStream_t s = nullptr);
    ~ProfScope();
};
void prof_resolve(pcp_ctx *ctx);   // after a stream sync
void prof_count(pcp_ctx *ctx, int kid);   // one event of kid (launches + 1, no time), always

// profiling of ONE kernel through the events hipExtLaunchKernelGGL records around its own
// execution: unlike stream-ordered events on an idle queue, the interval excludes the host's
// submission gap before the launch (pass .a / .b to the launch; null when not profiling)
struct KernelTimer {
    pcp_ctx *ctx;
    int kid;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(pcp_ctx *c, int k);
    ~KernelTimer();
};

// index ----------------------------------------------------------------------------------
// zsort: points of each cell in descending z (needed by scan_stencil's early exit: the
// terrain and aux indices); the other indices' queries are order-free
// occ: build the dilated occupancy bits (stencil_any: the aux index; the fan's A/B variant 2)
// raw_io (nullable): *raw_io non-null = the cloud's bytes already device-readable there (a
// previous build's, or a caller's staging); on return *raw_io = where the bytes were read.  A
// message-sized cloud is read in place from the pinned ring (pin_stage): without raw_io the
// slot is released behind the extraction; with raw_io the caller releases it (pin_release)
// after its own last reader.  Larger clouds are DMA'd into ctx->stage.  raw_copy (nullable,
// with raw_io: *raw_io then pinned, device-readable memory): the records are also copied there
// -- by the extraction itself where it can (16-byte multiples) -- and *raw_io = raw_copy on
// return, so the caller's later kernels read device memory (the composed carve)
int build_index(pcp_ctx *ctx, GridIndex &g, const pcp_cloud_view &v, double r_q,
                bool zsort = true, bool occ = true, const unsigned char **raw_io = nullptr,
                unsigned char *raw_copy = nullptr);
// two order-free indices (no z order, no occupancy bits) of one message-sized cloud from one
// pass over its raw records, plus the caller's per-point preparation (prep_pts: (x, y, z, 0) by
// input index; prep_nrm: NaN normals of the non-finite points; both nullable).  *paired false
// (nothing done): the cloud is empty, has no finite point or is past the host-bbox size -- build
// them with build_index.  raw_io as build_index's
int build_index_pair(pcp_ctx *ctx, GridIndex &ga, double ra, GridIndex &gb, double rb,
                     const pcp_cloud_view &v, const unsigned char **raw_io, float4 *prep_pts,
                     float *prep_nrm, bool *paired);
// the block-major copy of a z-sorted index (GridView.bstart / bpts); no-op when built
int build_blocks(pcp_ctx *ctx, GridIndex &g);
// the fine-window copy of a z-sorted index (GridView.frec / wpts); no-op when built.  Marks
// fine_fail (no retry) past its size caps or on an allocation failure.
int build_fine(pcp_ctx *ctx, GridIndex &g);
// before a terrain query: build the terrain's block copy per PCP_TERRAIN_BLOCKS (0 never,
// 1 at the second query after pcp_set_terrain -- a terrain that is queried once, as in the
// per-frame chain, does not pay for it --, 2 at the first)
int terrain_blocks_before_query(pcp_ctx *ctx);

// scan: exclusive prefix sum of n uint32 values into out (n + 1 entries, out[n] = total).
// tmp must hold scan_tmp_bytes(n).
size_t scan_tmp_bytes(uint64_t n);
// out2 (optional, may alias in): a second copy of out[0 .. n), e.g. a scatter's cursors; with
// zero2 it is cleared instead (out2 = in: counters left zero for their next use)
// preset16 (nullable): n halfwords set to 0x00FF by the same pass (the sparse z bands' preset)
int exclusive_scan_u32(pcp_ctx *ctx, const uint32_t *in, uint32_t *out, uint64_t n, void *tmp,
                       uint32_t *out2 = nullptr, bool zero2 = false, uint16_t *preset16 = nullptr);
// two such scans (tmp sized for the larger); two one-tile ones are a single launch
int exclusive_scan_u32_pair(pcp_ctx *ctx, const uint32_t *in_a, uint32_t *out_a, uint64_t n_a,
                            uint32_t *out2_a, const uint32_t *in_b, uint32_t *out_b, uint64_t n_b,
                            uint32_t *out2_b, void *tmp, bool zero2);

// fan query up to the per-pose sums, enqueued on ctx->stream (pcp_vlidar.hip): device results
// in flight on return, the caller synchronizes.  n > 0.
struct FanEnq {
    // input (pcp_raycast_fan_allreduce): k_fan_reduce also writes the one-collective vector --
    // keys[keys_lo + p] = (blocked << 32) | (keys_lo + p), ~0 in the other slots [0, keys_P]
    // (the health word at keys_P included), the units behind it at keys[keys_P + 1 + p]
    unsigned long long *keys = nullptr;
    uint32_t keys_lo = 0, keys_P = 0;
    // outputs
    uint32_t *blocked_d = nullptr;
    unsigned long long *units_d = nullptr;
    int16_t *fh_d = nullptr;
    uint32_t rays = 0;
    size_t stats_bytes = 0;
    unsigned long long *stats_d = nullptr;
};
// burst > 0: the plain kernel `burst` times back-to-back between two events, the average
// launch time to *burst_ms (pcp_raycast_fan_burst).  host_out: k_fan_reduce stores the
// per-pose {units u64[n], blocked u32[n]} straight into the pinned landing block
// (ctx->fan_host past the staged poses) instead of device memory; o.*_d stay null.
int fan_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n, const pcp_fan_params *fan,
                bool want_fh, bool stats, bool stamps, FanEnq &o, int burst = 0,
                double *burst_ms = nullptr, bool host_out = false);

// runOptimization's scoring up to the per-pose sums, enqueued on ctx->stream (pcp_vlidar.hip)
struct ScoreEnq {
    int P = 0, C = 0;
    double *comb = nullptr;        // [P][C] mobile scores
    double *score_z = nullptr;     // [C] zx120 scores
    uint8_t *mbits = nullptr;      // [P][C] result bits of the poses
    uint8_t *zbits = nullptr;      // [C] result bits of the zx120 evaluation
    uint8_t *flags_d = nullptr;    // [C] cell flag bytes (caller fills)
    double *tot_d = nullptr;       // [P + 1] totals, row P = zx120
    int32_t *cov_d = nullptr;      // [P + 1]
    int32_t *stats = nullptr;      // 64 colour-statistics slots (device: atomics)
    int32_t *stats_host = nullptr; // zc: where the last flag block copies the finished stats
    bool zc = false;               // flags / totals / covered live in the pinned block itself
    const uint32_t *P_dev = nullptr;   // the device's pose count (rows P = capacity)
    const uint32_t *C_dev = nullptr;   // the device's cell count (C = the lattice's capacity:
                                       // a pcp_set_excavation_area_async still in flight)
    const double *poses_k = nullptr;   // the poses / zx120 pose k_score_cells read
    const double *zx_k = nullptr;
    // the query's block (poses_d on the device, res_host pinned, same offsets): poses at 0,
    // cell flags at fl_off, totals + covered (tc_bytes) ending at most at st_off, stats at
    // st_off, blk_bytes in all
    size_t tc_bytes = 0, st_off = 0, fl_off = 0, blk_bytes = 0;
};
// cell_flags (C bytes) travel with the poses when given (pcp_score_poses); k_score_cells zeroes
// the statistics
// fuse_tail: the row sums are left to the caller's k_sum_flags launch (pcp_score_poses)
// zc: the kernels read the poses and flags from the pinned block and store the flags, totals,
// covered counts and (via the last flag block) the statistics back into it -- no copies (only
// with fuse_tail and cells present)
// P_dev / poses_dev: the poses are on the device already (generated in the same stream), n =
// the rows' capacity and *P_dev their count (pcp_generate_and_score)
int score_enqueue(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx[5],
                  const pcp_vl_params *p, ScoreEnq &o, const uint8_t *cell_flags = nullptr,
                  bool fuse_tail = false, bool zc = false, const uint32_t *P_dev = nullptr,
                  const double *poses_dev = nullptr);
// key kernels of the pose-sharded search (pcp_vlidar.hip; used by pcp_multi.hip)
// identity: the value of the other ranks' slots (~0 for ncclUint64 MIN, INT64_MAX for a signed
// int64 MIN as torch.distributed reduces it)
void launch_fan_keys(hipStream_t st, const uint32_t *blocked_d, uint32_t lo, uint32_t cnt,
                     uint32_t P, unsigned long long *keys, unsigned long long identity = ~0ull);
// the covered key's mark of a pose some rank scored (k_score_keys; the low 32 bits: the count)
constexpr unsigned long long kScoreWritten = 1ull << 32;
void launch_score_keys(hipStream_t st, const ScoreEnq &o, int lo, int P, unsigned long long *v);
void launch_flags_from_keys(hipStream_t st, const unsigned long long *v, const uint8_t *zbits,
                            int C, int P, uint8_t *flags, int32_t *stats);
void launch_keys_combine(hipStream_t st, unsigned long long *a, const unsigned long long *b,
                         size_t n, bool is_max);
// pcp_score_poses_allreduce's landing: reduced keys, zx120 total, health, flags, stats -> pinned
void launch_score_land(hipStream_t st, const unsigned long long *v, int P, size_t hw,
                       const double *zx_total, const uint8_t *flags, int C, const int32_t *stats,
                       void *pin, size_t fl_off, size_t st_off);
// a device buffer into pinned host memory by a copy kernel (k_copy_pinned; a DMA when the copy
// kernel is off or the pointers are not 16-byte aligned)
int copy_to_pinned_async(pcp_ctx *ctx, void *dst_pinned, const void *src_d, size_t bytes,
                         hipStream_t st);
// the colour-statistics slots (k_cell_flags order) -> pcp_vl_report
void fill_report(const int32_t *st_h, double zx_total, int64_t best_idx, double best,
                 pcp_vl_report *rep);

// pcp_set_excavation_area_async's settlement (pcp_excav.hip): waits for the stream, regrows and
// reruns the neighbour lists on an overflow, sets ctx->n_cells; a no-op with nothing pending
// (stream_synced: the caller has just synchronised ctx->stream after the join)
int area_finish(pcp_ctx *ctx, bool stream_synced = false);
// after a stream synchronisation that followed the pending setup: did its lists overflow?  (the
// count in ctx->area_host is then valid, the cells' normals are not)
bool area_overflowed(const pcp_ctx *ctx);
// the async setup's side stream joined into ctx->stream (a stream wait, no host wait); a no-op
// when nothing is forked
void area_join(pcp_ctx *ctx);
// the area setup over records already device-readable (raw_pre: pcp_excavate_area_async's
// pinned landing; nullptr: staged from area->data as pcp_set_excavation_area does)
int area_setup_from(pcp_ctx *ctx, const pcp_cloud_view *area, double grid_resolution,
                    int32_t vertical_layers, double grid_bbox[6], uint64_t *n_cells, bool defer,
                    const unsigned char *raw_pre);
// pcp_set_terrain over records already device-readable (raw_pre), or staged (nullptr)
int set_terrain_from(pcp_ctx *ctx, const pcp_cloud_view *terrain, const unsigned char *raw_pre);

// the context's RCCL communicator and its buffers (pcp_comm.hip), at pcp_destroy
void comm_release(pcp_ctx *ctx);
// memcpy for host buffers, split over the context's helper threads from 256 KiB on
// (pcp_hostcopy.hip); host_copy_release stops the helpers (pcp_destroy)
void host_copy(pcp_ctx *ctx, void *dst, const void *src, size_t bytes);
void host_copy_release(pcp_ctx *ctx);

// validate a cloud view
int check_view(pcp_ctx *ctx, const pcp_cloud_view *v, const char *what);

// a small (<= 4 KB) device -> host readback through pinned memory; synchronizes the stream
// (a pageable destination costs a staging copy per call)
int read_small(pcp_ctx *ctx, void *dst, const void *src_d, size_t bytes, hipStream_t st);

// host -> device copy of a caller's (pageable) buffer that does NOT wait for the stream: a
// pageable hipMemcpyAsync returns only once the stream has drained up to it (an implicit
// synchronisation in the middle of a chain).  Up to kUploadPinnedMax bytes are copied on the
// host into a slot of a pinned ring and DMA'd stream-ordered (the slot is reused only after
// its previous DMA completed); larger buffers take the pageable path.  The caller may reuse
// src_h on return either way.
constexpr size_t kUploadPinnedMax = 16u << 20;
int upload_async(pcp_ctx *ctx, void *dst_d, const void *src_h, size_t bytes, hipStream_t st);
// pinned host -> device by a copy kernel on st (no copy-engine hand-off); unaligned pointers
// take hipMemcpyAsync
int copy_pinned_async(pcp_ctx *ctx, void *dst_d, const void *src_pinned, size_t bytes,
                      hipStream_t st);
// several host pieces into one pinned slot at their byte offsets, then ONE DMA of `bytes`
// (the gaps between pieces are don't-care bytes on the device)
struct HostPiece {
    size_t off;
    const void *src;
    size_t bytes;
};
int upload_pieces(pcp_ctx *ctx, void *dst_d, const HostPiece *pc, int k, size_t bytes,
                  hipStream_t st);
// zero-copy staging of message-sized inputs (<= kPinDirectMax bytes): the pieces are copied on
// the host into a slot of the pinned ring and the kernels read them there, over the host link
// -- no DMA, so no copy-engine hand-off in front of the first kernel.  *dev = the slot (a
// device-readable host pointer).  The slot stays held until pin_release records, on st, the
// point after the last kernel that reads it (a call that stages twice without releasing
// drains the stream first).
constexpr size_t kPinDirectMax = 4u << 20;
int pin_stage(pcp_ctx *ctx, const HostPiece *pc, int k, size_t bytes, const void **dev);
void pin_release(pcp_ctx *ctx, hipStream_t st);

// the smallest float d with fl(d * d) >= r2: a point with dz = qz - pz >= d fails FLANN's
// float test (its sum is >= fl(dz^2) >= r2), and so does every lower point of a z-descending
// run -- the walks' early exit as one compare
float exit_dist(float r2);

// fan tables (shared definition with the oracle's orc_fan_tables)
void fan_tables(int32_t n_az, int32_t n_el, double el_min, double el_max, double *ca,
                double *sa, double *ce, double *se);
std::vector<double> step_table(double end);

}  // namespace pcp
