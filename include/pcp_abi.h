/*
 * pcp_abi.h -- C ABI of libpcp: the MI355X-native hot path of
 * YamaguchiAtsushi/pointcloud_processor (crop/voxel -> SE(3)+concat -> virtual-LiDAR
 * ray-trace pose search), re-designed for gfx950.
 *
 * The reference has no plugin/operator/FFI API: its only stable interface is the ROS2
 * surface.  Each entry point below replaces one algorithm member function
 * of a reference node (cited file:line); a node shell keeps the topics/params/QoS and calls
 * these with the PointCloud2 buffers it already holds.  See INTEGRATION.md.
 *
 * Conventions
 *  - every function returns int status (PCP_OK = 0, < 0 on error) and never throws;
 *    the message is available from pcp_last_error(ctx).
 *  - a pcp_ctx owns one HIP device, one HIP stream and all device buffers.  It is NOT
 *    thread-safe (the reference runs callbacks on a single-threaded executor).
 *  - unless a `flags` argument says otherwise, pointers are HOST pointers owned by the
 *    caller; calls are synchronous (results are in host memory on return).
 *  - empty inputs are not errors: they return PCP_OK with zero outputs / best_idx = -1.
 *  - PCP_E_CAPACITY: an output buffer was too small; the *n_out argument holds the size
 *    that was needed and nothing else was written.
 */
#ifndef PCP_ABI_H
#define PCP_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCP_ABI_VERSION 2   /* 2: pcp_index_info.scan_layout */

enum pcp_status {
    PCP_OK = 0,
    PCP_E_INVALID = -1,   /* bad argument (null pointer, misaligned field, bad size) */
    PCP_E_HIP = -2,       /* HIP runtime / device error */
    PCP_E_CAPACITY = -3,  /* output capacity too small (*n_out = required) */
    PCP_E_STATE = -4,     /* missing prerequisite (e.g. pcp_set_cells not called) */
    PCP_E_NOMEM = -5      /* device or host allocation failed */
};

typedef struct pcp_ctx pcp_ctx;

/* A PointCloud2-like array-of-structs buffer: `n` points of `point_step` bytes each with
 * FLOAT32 x/y/z at byte offsets off_x/off_y/off_z (sensor_msgs::PointField).  Offsets and
 * point_step must be multiples of 4.  This is exactly what pcl::fromROSMsg reads. */
typedef struct pcp_cloud_view {
    const void *data;
    uint64_t n;
    uint32_t point_step;
    uint32_t off_x, off_y, off_z;
} pcp_cloud_view;

/* ---- context ----------------------------------------------------------------------- */
int pcp_abi_version(void);
int pcp_device_count(int *n);
int pcp_create(int device, pcp_ctx **out);
void pcp_destroy(pcp_ctx *ctx);
const char *pcp_last_error(const pcp_ctx *ctx);
int pcp_synchronize(pcp_ctx *ctx);

/* a second HIP stream of libpcp's own runtime on the context's device (e.g. the wait_stream of
 * pcp_raycast_fan_keys); the caller destroys it before the context */
int pcp_stream_create(pcp_ctx *ctx, void **stream);
int pcp_stream_destroy(pcp_ctx *ctx, void *stream);

/* device buffers owned by the caller (for inputs resident in HBM, e.g. benchmarks) */
int pcp_dev_alloc(pcp_ctx *ctx, uint64_t bytes, void **dptr);
int pcp_dev_free(pcp_ctx *ctx, void *dptr);
int pcp_memcpy_h2d(pcp_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int pcp_memcpy_d2h(pcp_ctx *ctx, void *dst, const void *src, uint64_t bytes);
/* Pinned (page-locked) host memory for PointCloud2 data blobs: the node shell deserializes
 * into / publishes from these, so every H2D/D2H of the calls above runs as direct DMA instead
 * of the runtime's pageable staging.  pcp_host_register pins an existing buffer in place
 * (unregister before freeing it). */
int pcp_host_alloc(pcp_ctx *ctx, uint64_t bytes, void **hptr);
int pcp_host_free(pcp_ctx *ctx, void *hptr);
int pcp_host_register(pcp_ctx *ctx, void *hptr, uint64_t bytes);
int pcp_host_unregister(pcp_ctx *ctx, void *hptr);

/* process-wide counts of scratch (re)allocations by the library: device buffers, pinned
 * staging buffers, bytes allocated.  Each device reallocation frees the old buffer (a device
 * synchronization), so a streaming caller checks these settle after its first frames. */
int pcp_alloc_stats(uint64_t *device_reallocs, uint64_t *pinned_reallocs, uint64_t *bytes);

/* ---- in-library kernel timing (HIP events on the ctx stream) ------------------------ */
enum pcp_kernel_id {
    PCP_K_RAYCAST_FAN = 0,   /* fan ray-march (BASELINE configs[1], the headline)   */
    PCP_K_SCORE_CELLS,       /* mobile pose x cell ray-march + score                 */
    PCP_K_ZX120_CELLS,       /* pose-invariant zx120 cell evaluation                 */
    PCP_K_POSE_SUM,          /* ordered per-pose score sums                          */
    PCP_K_CELL_FLAGS,        /* stale-flag resolve + colour statistics              */
    PCP_K_CANDIDATES,        /* candidate lattice + ground height                    */
    PCP_K_INDEX_BUILD,       /* all kernels of a spatial index build                 */
    PCP_K_CROP,              /* crop-box stream compaction                           */
    PCP_K_VOXEL,             /* voxel keying + sort + centroid                       */
    PCP_K_TRANSFORM,         /* SE(3) + RGB + concat                                  */
    PCP_K_FILTER_MERGE,      /* whole crop->voxel->transform pipeline (graph replay)   */
    PCP_K_EXCAVATE,          /* excavated-terrain carve: heights + pit test + compaction */
    PCP_K_EXCAV_SETUP,       /* excavation-area normals + cell grid                    */
    PCP_K_VOXEL_REDO,        /* bucket-chain frames redone by the LSD chain (a bucket past
                              * its LDS capacity); launches = frames redone             */
    PCP_K_COUNT
};
int pcp_profile_enable(pcp_ctx *ctx, int enable);
int pcp_profile_reset(pcp_ctx *ctx);
int pcp_profile_get(pcp_ctx *ctx, int kernel_id, double *total_ms, uint64_t *launches);
const char *pcp_kernel_name(int kernel_id);

/* ---- pointcloud_filter (SimplifiedScanMatcher) --------------------------------------- */
/* cropFrontArea, pointcloud_filter.cpp:87-120 (predicate :111-113).  Order-preserving
 * strict box  box[0] < x < box[1], box[2] < y < box[3], box[4] < z < box[5]  with the
 * float coordinate compared to the double bound.  kept_idx (nullable): input indices of
 * the kept points, ascending.  out_xyz16 (nullable): kept points as PointXYZ (16-B
 * stride: x,y,z,1.0f). */
int pcp_crop_box(pcp_ctx *ctx, const pcp_cloud_view *in, const double box[6],
                 uint32_t *kept_idx, float *out_xyz16, uint64_t cap, uint64_t *n_kept);

/* downsampleCloud -> pcl::VoxelGrid<PointXYZ>, pointcloud_filter.cpp:122-139.
 * out_xyz16: centroids (PointXYZ, 16-B stride) in ascending voxel index.
 * voxel_idx / voxel_count (nullable): PCL's linear voxel index and points per voxel.
 * *passthrough = 1 when PCL's int32 index-overflow guard fires (output = input). */
int pcp_voxel_grid(pcp_ctx *ctx, const pcp_cloud_view *in, float leaf, float *out_xyz16,
                   uint32_t *voxel_idx, uint32_t *voxel_count, uint64_t cap, uint64_t *n_out,
                   int32_t *passthrough);

/* processCloudSimple, pointcloud_filter.cpp:64-85: crop then voxel (leaf <= 0: crop only)
 * fused on the device.  Output PointXYZ 16-B stride (the toROSMsg layout). */
int pcp_crop_voxel(pcp_ctx *ctx, const pcp_cloud_view *in, const double box[6], float leaf,
                   float *out_xyz16, uint64_t cap, uint64_t *n_out, uint64_t *n_cropped);

/* ---- pointcloud_merger (GnssGicpMatcher cloud part) ------------------------------------ */
typedef struct pcp_rigid {
    double t[3];   /* geometry_msgs Transform.translation */
    double q[4];   /* rotation x, y, z, w */
} pcp_rigid;

/* processPointClouds + processRobotCloud, pointcloud_merger.cpp:308-394: for each cloud i
 * in order, tf2::doTransform (float32 Eigen Translation3f*Quaternionf, :370) and tag colour
 * rgb[3i..3i+2] (:376-387), concatenated (robot first, then zx120, :316-325).
 * out_xyzrgb32: PointXYZRGB memory image, 32-B stride (x,y,z,1.0f,rgba,pad). */
int pcp_transform_concat(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds,
                         const pcp_rigid *tf, const uint8_t *rgb, void *out_xyzrgb32,
                         uint64_t cap, uint64_t *n_out);

/* Full device pipeline (BASELINE configs[2]): per cloud crop -> voxel(leaf) -> transform +
 * colour, concatenated.  boxes: 6 doubles per cloud.  flags: PCP_MEM_DEVICE_IN (cloud data
 * pointers are device pointers) / PCP_MEM_DEVICE_OUT (out is a device pointer).
 * n_per_cloud (nullable, k entries): points each cloud contributed. */
#define PCP_MEM_DEVICE_IN 1u
#define PCP_MEM_DEVICE_OUT 2u
int pcp_filter_merge(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds, const double *boxes,
                     float leaf, const pcp_rigid *tf, const uint8_t *rgb, void *out_xyzrgb32,
                     uint64_t cap, uint64_t *n_out, uint64_t *n_per_cloud, uint32_t flags);
/* The launch file's filter node (both sensors) and merger node composed in one process (a
 * component container; the C5 chain): per cloud i crop -> voxel(leaf), its centroids in its own
 * frame into filtered[i] (host, clouds[i].n PointXYZ 16-B records at most: the node's
 * /filtered_points message) AND all clouds transformed + coloured + concatenated into `out`
 * (host, PointXYZRGB 32-B, cap records: pcp_filter_merge's output), ONE synchronisation.  Host
 * memory in and out (message-sized clouds are read in place from pinned staging).  `out` and
 * each filtered[i] may be NULL (not copied: read them with pcp_filter_merge_landed).
 * n_per_cloud / n_cropped (nullable, k entries): centroids and cropped points of each cloud. */
int pcp_filter_merge_nodes(pcp_ctx *ctx, int k, const pcp_cloud_view *clouds,
                           const double *boxes, float leaf, const pcp_rigid *tf,
                           const uint8_t *rgb, void *out, uint64_t cap, uint64_t *n_out,
                           uint64_t *n_per_cloud, float *const *filtered, uint64_t *n_cropped);
/* Where the last pcp_filter_merge_nodes call's outputs landed: the context's pinned memory,
 * host-readable (the same bytes `out` / `filtered[i]` receive; a caller that reads them here may
 * pass out = NULL, filtered[i] = NULL to that call) -- merged: *n_out PointXYZRGB records,
 * filtered[i]: n_per_cloud[i] PointXYZ records.  A view over `merged` given to
 * pcp_excavate_area_async is read in place by the device (no staging copy).  Valid until the
 * context's next pcp_filter_merge*, pcp_transform_concat or pcp_excavate call; PCP_E_STATE when
 * there is none, or k differs from that call's. */
int pcp_filter_merge_landed(pcp_ctx *ctx, int k, const void **merged, const float **filtered);

/* ---- virtual_lidar (SimplifiedDualLidarOptimizer) -------------------------------------- */
typedef struct pcp_vl_params {      /* virtual_lidar.cpp:66-71 */
    double grid_resolution;         /* 0.1  */
    double sensor_height;           /* 1.1  */
    double search_radius;           /* 3.0  */
    double max_distance;            /* 15.0 */
    int32_t num_candidates;         /* 100  */
    int32_t vertical_layers;        /* 10   */
} pcp_vl_params;

/* GridCell flag bits (virtual_lidar.cpp:20-44) as kept by the caller between ticks */
#define PCP_F_RANGE_Z 1u
#define PCP_F_FOV_Z 2u
#define PCP_F_VIS_Z 4u
#define PCP_F_RANGE_M 8u
#define PCP_F_FOV_M 16u
#define PCP_F_VIS_M 32u

typedef struct pcp_vl_report {
    int64_t best_idx;            /* -1: no candidates */
    double best_score;           /* -inf when no candidates (:464) */
    double zx120_total_score;    /* evaluateZX120Only (:360-452) */
    int32_t zx120_range_ok, zx120_fov_ok, zx120_visible_ok;
    int32_t total_cells;
    int32_t zx120_green, zx120_red, zx120_blue, zx120_yellow;
    int32_t green, red, blue, yellow;   /* dual configuration (:480-519) */
} pcp_vl_report;

/* terrainCallback (:180-192): replaces KdTreeFLANN::setInputCloud(terrain).  n == 0 keeps
 * the previous index for ray casts (the reference keeps the stale tree) while ground
 * heights see the empty cloud (:601). */
int pcp_set_terrain(pcp_ctx *ctx, const pcp_cloud_view *terrain);
/* zx120PointsCallback (:194-207): index of /zx120/filtered_points for the relaxed check. */
int pcp_set_aux_cloud(pcp_ctx *ctx, const pcp_cloud_view *aux);
/* the valid cells of generateExcavationGrid3D (:236-287): centres (x,y,z double) and
 * surface normals (float, computeCellSurfaceNormal :301-340), in grid order. */
int pcp_set_cells(pcp_ctx *ctx, const double *xyz, const float *normals, uint64_t n);

/* excavationAreaCallback (virtual_lidar.cpp:164-178) on the GPU: replaces the excavation
 * KdTreeFLANN, computeTerrainNormals (:209-234: pcl::NormalEstimation, radius 1.5, viewpoint
 * (0,0,0), then flipped to normal_z >= 0) and generateExcavationGrid3D (:236-287, with
 * isPointNearExcavation :289-299 at radius 1.5 * grid_resolution and computeCellSurfaceNormal
 * :301-340).  The valid cells, in the reference's loop order, with their surface normals become
 * the context's scoring cells (as pcp_set_cells).  An empty area returns PCP_OK and keeps the
 * previous cells (:168).  grid_bbox (nullable out): grid_min_x, grid_max_x, grid_min_y,
 * grid_max_y, excavation_min_z, excavation_max_z after the margin; n_cells (nullable out).
 * `area` is host memory (the PointCloud2 data blob). */
int pcp_set_excavation_area(pcp_ctx *ctx, const pcp_cloud_view *area, double grid_resolution,
                            int32_t vertical_layers, double grid_bbox[6], uint64_t *n_cells);
/* The same setup, enqueued on the context's stream and NOT waited for (a composed chain: the
 * terrain and zx120 indices and the tick are enqueued behind it while it runs).  grid_bbox as
 * above (host arithmetic, exact at return); cells_cap: the lattice's points, an upper bound of
 * the cell count.  The count is settled -- and the neighbour lists regrown and rerun, should
 * they have overflowed -- by the next call that needs it: pcp_generate_and_score does so after
 * its own synchronisation (ONE wait for both; its cell_flags must then hold cells_cap bytes,
 * are taken as fresh GridCells -- all clear, :259 -- and come back for the settled count), every
 * other call that reads the cells (pcp_score_poses, pcp_get_cells, pcp_set_cells, the multi
 * calls, another setup) before it starts.  Results are identical to pcp_set_excavation_area's. */
int pcp_set_excavation_area_async(pcp_ctx *ctx, const pcp_cloud_view *area,
                                  double grid_resolution, int32_t vertical_layers,
                                  double grid_bbox[6], uint64_t *cells_cap);
/* the context's scoring cells (settles a pending setup: may wait for the stream) */
int pcp_cells_count(pcp_ctx *ctx, uint64_t *n_cells);
/* ---- excavated_surface_generator.cpp (ExcavationTerrainGenerator) ------------------------ */
typedef struct pcp_excavation_params {   /* excavated_surface_generator.cpp:29-51 */
    double depth;                 /* excavation.depth 1.0 */
    double slope_angle_deg;       /* excavation.slope_angle 75.0 */
    double offset_x, offset_y;    /* excavation.offset_x/_y 4.0, 1.0 (zx120 base frame) */
    double point_density;         /* excavation.point_density 0.05 */
    double terrain_search_radius; /* excavation.terrain_search_radius 0.5 */
    int32_t l_shape_enabled;      /* excavation.l_shape_enabled 1 */
    double arm1_length, arm1_width, arm2_length, arm2_width;   /* 2.0 1.2 2.0 1.2 */
    double width, length;         /* rectangle mode 1.2, 1.8 */
} pcp_excavation_params;

/* matchedCloudCallback (:259-326) with excavation enabled and the zx120 TF present
 * (zx120_base = map -> zx120/base_link).  in: /matched_point_cloud, host memory (x/y/z float
 * fields; the rgb float at byte 16 when point_step >= 20, else 0).  Outputs are PointXYZRGB
 * records (32 B: x, y, z, 1, rgb, 0, 0, 0) in host buffers:
 *   terrain_out: /excavated_terrain = the input points processExcavation keeps (:451-485,
 *                input order) then generateExcavatedSurface's bottom and wall points (:487-584)
 *   area_out:    /excavation_area = generateExcavationArea (:350-455)
 * Every getTerrainHeight (:183-226) runs on the GPU against one index of the input (the
 * reference rebuilds a KD-tree per call, once per input point).  pose_out (nullable): the
 * excavation centre x, y, its terrain height, yaw (publishExcavationMarkers).  *_cap in
 * records; PCP_E_CAPACITY with *n_* set when short.  A missing TF is the caller's branch
 * (:276-279: the input is republished unchanged). */
int pcp_excavate(pcp_ctx *ctx, const pcp_cloud_view *in, const pcp_excavation_params *p,
                 const pcp_rigid *zx120_base, void *terrain_out, uint64_t terrain_cap,
                 uint64_t *n_terrain, void *area_out, uint64_t area_cap, uint64_t *n_area,
                 double pose_out[4]);
/* The carve node and virtual_lidar's two callbacks for its messages composed in one process
 * (the C5 chain): pcp_excavate, then pcp_set_excavation_area_async over /excavation_area
 * (skipped when empty: :168) and pcp_set_terrain over /excavated_terrain, fed from the carve's
 * records where they land (device-readable pinned memory, no staging copy or upload), the host
 * copies into terrain_out / area_out made after the setup and the index build are enqueued.
 * Arguments and results as those three calls'; grid_bbox / cells_cap as
 * pcp_set_excavation_area_async's (settled the same way).  Waits once (the carve's counts).
 * terrain_out = area_out = NULL: nothing is copied (the caps are not checked); the records stay
 * where they landed, read with pcp_excavate_landed -- a composed caller enqueues its next
 * consumers (the zx120 index) first and builds its messages from there. */
int pcp_excavate_area_async(pcp_ctx *ctx, const pcp_cloud_view *in,
                            const pcp_excavation_params *p, const pcp_rigid *zx120_base,
                            void *terrain_out, uint64_t terrain_cap, uint64_t *n_terrain,
                            void *area_out, uint64_t area_cap, uint64_t *n_area,
                            double pose_out[4], double grid_resolution, int32_t vertical_layers,
                            double grid_bbox[6], uint64_t *cells_cap);
/* Where the last pcp_excavate_area_async call made with null outputs left its records: the
 * context's pinned memory, host-readable -- terrain: *n_terrain, area: *n_area PointXYZRGB
 * records of that call (the bytes terrain_out / area_out would have received).  Valid until the
 * context's next pcp_excavate* call; PCP_E_STATE when there is none. */
int pcp_excavate_landed(pcp_ctx *ctx, const void **terrain, const void **area);

/* ---- calc_drivable_area.cpp (the occupancy-grid node) -------------------------------------- */
typedef struct pcp_drivable_params {   /* calc_drivable_area.cpp:20-26 */
    double grid_resolution;            /* 1.0 */
    double map_width, map_height;      /* 100, 100 */
    double max_gradient;               /* 0.3 */
    int32_t min_points_per_cell;       /* 10 */
    double start_clear_radius;         /* 3.0 */
} pcp_drivable_params;

/* robotCloudCallback (:67-226): the robot's filtered cloud (host memory, sensor frame) through
 * tf2::doTransform(cloud_to_map) (Eigen float), binned into the grid centred on (robot_x,
 * robot_y) (map -> four_wheel_robot/base_link); start_x/y = the first robot position (the
 * node's state).  grid (dims[1] rows of dims[0] int8, row-major over y): 0 free, 100 obstacle,
 * -1 unknown -- nav_msgs/OccupancyGrid.data; origin = the grid's lower-left corner.  An empty
 * cloud publishes nothing (:107-111): PCP_OK, grid untouched. */
int pcp_drivable_area(pcp_ctx *ctx, const pcp_cloud_view *cloud, const pcp_rigid *cloud_to_map,
                      double robot_x, double robot_y, double start_x, double start_y,
                      const pcp_drivable_params *p, int8_t *grid, uint64_t cap, int32_t dims[2],
                      double origin[2]);

/* upper bounds of pcp_excavate's record counts for an n-point input (host arithmetic only) */
int pcp_excavate_bounds(const pcp_excavation_params *p, uint64_t n_in, uint64_t *terrain_cap,
                        uint64_t *area_cap);

/* the context's scoring cells: xyz (n x 3 double) and normals (n x 3 float), either nullable;
 * *n_cells = count (PCP_E_CAPACITY when it exceeds cap). */
int pcp_get_cells(pcp_ctx *ctx, double *xyz, float *normals, uint64_t cap, uint64_t *n_cells);
/* terrain_normals_ of the last pcp_set_excavation_area, in input order (n x 3 float, NaN
 * where fewer than 3 neighbours or a non-finite point). */
int pcp_get_area_normals(pcp_ctx *ctx, float *normals, uint64_t cap, uint64_t *n);

/* generateCandidatePositions + getGroundHeight (:550-625).  grid_bbox = {grid_min_x,
 * grid_max_x, grid_min_y, grid_max_y, excavation_min_z, excavation_max_z} after the
 * margin (:251-254).  zx120_pose5 = {x,y,z,pitch,yaw} from getZX120Position (:342-358).
 * poses5 out: x,y,z,pitch,yaw per candidate, in the reference's lattice order. */
int pcp_generate_candidates(pcp_ctx *ctx, const double grid_bbox[6], const pcp_vl_params *p,
                            const double zx120_pose5[5], double *poses5, uint64_t cap,
                            uint64_t *n_out);

/* runOptimization's scoring (:460-519): evaluateZX120Only, evaluatePosition per candidate
 * (:627-654), strict-'>' argmax (:471-474) and the colour statistics from the stale
 * GridCell flags (:487-501).  cell_flags: in/out, one byte per cell (PCP_F_*), the state
 * the caller's GridCells hold.  total_score/covered (nullable): per candidate. */
int pcp_score_poses(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx120_pose5[5],
                    const pcp_vl_params *p, uint8_t *cell_flags, double *total_score,
                    int32_t *covered, pcp_vl_report *rep);

/* Diagnostics of the reference's own ray march (the roofline of k_score_cells, bench.py
 * reference_mode; never used for results).  pcp_score_poses_stats: the query's visibility rays
 * (the same rows, cells and march as pcp_score_poses) counted by a twin of the kernel --
 * stats[0] z-band probes (2-byte records), stats[1] candidates' walk starts (4 bytes),
 * stats[2] point records tested (12 bytes), stats[3] directory loads (0 with the fine-window
 * copy).  pcp_score_poses_burst: the query's production k_score_cells launch `reps` times
 * back-to-back between two stream events; *ms_per_launch = the interval / reps.  Neither
 * touches the caller's GridCell flags. */
/* evaluateCellScore's value for every (pose, cell) of the query (k_score_cells' rows, before
 * evaluatePosition's std::max): score_mobile [n][n_cells], score_zx120 [n_cells] (host).  The
 * per-cell parity bar (tests); the caller's GridCell flags are not touched. */
int pcp_score_matrix(pcp_ctx *ctx, const double *poses5, uint64_t n, const double zx120_pose5[5],
                     const pcp_vl_params *p, double *score_mobile, double *score_zx120);
int pcp_score_poses_stats(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const double zx120_pose5[5], const pcp_vl_params *p, uint64_t stats[4]);
int pcp_score_poses_burst(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const double zx120_pose5[5], const pcp_vl_params *p, int reps,
                          double *ms_per_launch);

/* runOptimization's device part in one call (:455-519): pcp_generate_candidates then
 * pcp_score_poses on those candidates, identical results, one synchronisation -- the scoring
 * reads the candidates and their count where the generation left them on the device (the
 * reference's generateCandidatePositions + candidate loop).  poses5 (cap poses) receives the
 * candidates, *n_out their count; the rest as pcp_score_poses.  Lattices past 65,535 points
 * run as the two calls. */
int pcp_generate_and_score(pcp_ctx *ctx, const double grid_bbox[6], const pcp_vl_params *p,
                           const double zx120_pose5[5], double *poses5, uint64_t cap,
                           uint64_t *n_out, uint8_t *cell_flags, double *total_score,
                           int32_t *covered, pcp_vl_report *rep);

/* Dense ray fan (BASELINE configs[1]): per pose, n_az x n_el rays, ray (i, j) with local
 * direction (cos e_j cos a_i, cos e_j sin a_i, sin e_j), a_i = 2*pi*i/n_az,
 * e_j = el_min + (el_max-el_min)*(j+0.5)/n_el, rotated by the pose yaw, marched with
 * checkVisibilityWithRaycasting's rule (:765-797) to end = max_distance - 0.08.
 * blocked[p]: rays that hit terrain (occlusion score); units[p] (nullable): sample
 * queries the reference would execute; first_hit (nullable, [p][j][i] int16): sample
 * index of the first blocked sample or -1 (depth = pcp_step_table[k]);
 * best_idx (nullable): argmin blocked, ties -> lowest index. */
typedef struct pcp_fan_params {
    int32_t n_az, n_el;
    double el_min, el_max;     /* radians */
    double max_distance;
} pcp_fan_params;
int pcp_raycast_fan(pcp_ctx *ctx, const double *poses5, uint64_t n, const pcp_fan_params *fan,
                    uint32_t *blocked, uint64_t *units, int16_t *first_hit, int64_t *best_idx);

/* Diagnostic build of the same march (not for timing): stats[0] = samples probed after the
 * exact clip, stats[1] = samples whose 2x2x2 stencil survives the z-band probe and is scanned,
 * stats[2] = point records loaded (12 B each), stats[3] = block directory entries loaded.
 * Used to state the roofline's requested bytes. */
int pcp_raycast_fan_stats(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, uint64_t stats[4]);

/* Kernel timing for the roofline: the production fan kernel of this query, `reps` launches
 * back-to-back between two stream events (after the query's own setup); *ms_per_launch = the
 * interval / reps.  The queue does not idle inside the interval, so the figure agrees with a
 * rocprofv3 kernel trace (a synchronous query's own events also hold the queue wake-up). */
int pcp_raycast_fan_burst(pcp_ctx *ctx, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, int reps, double *ms_per_launch);

/* Diagnostic build with s_memtime stamps (shader clock) per wave: stamps[(p*W + w)*4 + i],
 * W = ceil(n_az*n_el/64), i = 0 start, 1 after direction setup, 2 after the march, 3 end.
 * For locating where wave lifetime goes; never used for timing. */
int pcp_raycast_fan_stamps(pcp_ctx *ctx, const double *poses5, uint64_t n,
                           const pcp_fan_params *fan, uint64_t *stamps);

/* One rank's shard of a pose-sharded fan query whose collective the CALLER runs (one process
 * per GPU: bench.py --gpus N over torch.distributed / RCCL).  The fans of poses5[0 .. n) --
 * global poses [lo, lo + n) of p_total -- are cast as pcp_raycast_fan does, and their keys
 * (blocked << 32) | global pose index are written into the caller's DEVICE buffer
 * keys_dev[p_total] (int64; INT64_MAX in the other ranks' slots), so one all-reduce(MIN) over
 * int64 gives every rank the blocked count of every pose and the argmin (ties: lowest index;
 * virtual_lidar.cpp:467-475).  units_dev (device, nullable, n entries): ray-hit tests per pose.
 * wait_stream (a hipStream_t of the same device, created through the SAME HIP runtime that
 * libpcp links -- not a handle from a framework that bundles its own, such as a PyTorch
 * wheel; nullable): that stream is made to wait for the keys (hipStreamWaitEvent) and the call
 * returns without a host synchronisation; NULL: the call returns once the keys are written.
 * No host copy of the results is made. */
int pcp_raycast_fan_keys(pcp_ctx *ctx, const double *poses5, uint64_t n,
                         const pcp_fan_params *fan, uint64_t lo, uint64_t p_total,
                         int64_t *keys_dev, uint64_t *units_dev, void *wait_stream);

/* ---- one process per GPU: libpcp's own RCCL communicator (bench.py --gpus N) ------------ */
/* The caller's framework only carries the 128-byte id from rank 0 to the others (and its own
 * host-side barriers); the collective runs in this library's HIP runtime on the context's
 * stream, so no stream or device pointer ever crosses into another runtime (a PyTorch wheel
 * bundles its own).  pcp_comm_unique_id: rank 0, before the others' pcp_comm_init_rank
 * (ncclGetUniqueId); pcp_comm_init_rank: ncclCommInitRank on the context's device, collective
 * over all ranks (each rank's context on a distinct device).  The communicator lives until
 * pcp_destroy. */
#define PCP_COMM_ID_BYTES 128
int pcp_comm_unique_id(uint8_t id[PCP_COMM_ID_BYTES]);
int pcp_comm_init_rank(pcp_ctx *ctx, int nranks, const uint8_t id[PCP_COMM_ID_BYTES], int rank);
int pcp_comm_info(const pcp_ctx *ctx, int *nranks, int *rank);   /* 0 ranks: none */
/* Which HIP runtime and RCCL this process's libpcp actually runs on (a PyTorch wheel ships both
 * under the same SONAMEs; whichever was loaded first serves every later NEEDED entry): the
 * versions the libraries report (hipRuntimeGetVersion, ncclGetVersion) and the files they were
 * loaded from (dladdr of hipMalloc / ncclAllReduce).  Paths are NUL-terminated, truncated to
 * cap bytes.  No device call: safe without a GPU. */
typedef struct pcp_runtime_info {
    int32_t hip_runtime_version;   /* HIP_VERSION encoding: major * 10^7 + minor * 10^5 + patch */
    int32_t rccl_version;          /* NCCL_VERSION_CODE encoding: major * 10^4 + minor * 100 + patch */
    char hip_path[512];
    char rccl_path[512];
} pcp_runtime_info;
int pcp_get_runtime_info(pcp_runtime_info *info);
/* One rank's shard of a pose-sharded fan query, collective included (every rank calls it with
 * the same p_total and fan): the fans of poses5[0 .. n) -- global poses [lo, lo + n) -- cast as
 * pcp_raycast_fan does, their keys (blocked << 32) | global pose written into the context's
 * device vector of p_total uint64 (UINT64_MAX elsewhere), ONE ncclAllReduce(ncclUint64,
 * ncclMin) over it on the context's stream, the reduced vector copied back once.
 * blocked_all (host, p_total entries, nullable): every pose's blocked count on every rank;
 * units (host, n entries, nullable): this shard's ray-hit tests per pose; best_idx: the argmin
 * (ties: lowest index; virtual_lidar.cpp:467-475); collective_ms (nullable): the all-reduce's
 * time between two events on the stream.  PCP_E_STATE without a communicator, or when a pose
 * of [0, p_total) was written by no rank.  Replaces the pose loop of runOptimization
 * (virtual_lidar.cpp:467-475) for N processes. */
int pcp_raycast_fan_allreduce(pcp_ctx *ctx, const double *poses5, uint64_t n,
                              const pcp_fan_params *fan, uint64_t lo, uint64_t p_total,
                              uint32_t *blocked_all, uint64_t *units, int64_t *best_idx,
                              double *collective_ms);

/* runOptimization's scoring for one rank of N processes (virtual_lidar.cpp:460-519; every
 * rank calls it with the same p_total, zx120 pose, parameters and cells): this rank's poses5[0 ..
 * n) -- global poses [lo, lo + n) of p_total -- scored as pcp_score_poses scores them, then ONE
 * ncclAllReduce(ncclUint64, ncclMax) on the context's stream over [p_total totals (IEEE bits:
 * totals are >= +0) | p_total covered counts | 3 x n_cells newest-pose flag keys | 1 health
 * word] (the vector pcp_multi_score_poses reduces), then on every rank: the stale GridCell flags
 * resolved from the newest pose overall (:480-519, cell_flags in/out as pcp_score_poses), the
 * strict-'>' argmax over all totals (:471-474) and the colour statistics into *rep.
 * total_all / covered_all (host, p_total entries, nullable): every pose's total and covered
 * count.  collective_ms (nullable): the all-reduce between two events on the stream.
 * A rank whose work before the collective fails still runs it with a poisoned health word: it
 * returns its own error, every other rank PCP_E_STATE (nobody is left blocked in RCCL).
 * PCP_E_STATE too when a pose of [0, p_total) was scored by no rank (cell_flags untouched).
 * Results are identical to pcp_score_poses over all p_total poses on one context. */
int pcp_score_poses_allreduce(pcp_ctx *ctx, const double *poses5, uint64_t n,
                              const double zx120_pose5[5], const pcp_vl_params *p, uint64_t lo,
                              uint64_t p_total, uint8_t *cell_flags, double *total_all,
                              int32_t *covered_all, pcp_vl_report *rep, double *collective_ms);

/* ---- one process, n GPUs: the pose search sharded over devices ------ */
/* pcp_multi_create(n_dev, devices, &m): one context per device (devices NULL: 0 .. n_dev-1)
 * and ONE RCCL communicator over them (ncclCommInitAll).  Poses are partitioned contiguously
 * (rank r takes [r*P/n, (r+1)*P/n), the first P % n ranks one more, the split of
 * runOptimization's candidate loop, virtual_lidar.cpp:467-475); the terrain, zx120 cloud and
 * cells are replicated; each query runs ONE collective:
 *   pcp_multi_raycast_fan  ncclAllReduce(ncclUint64, ncclMin) over P keys (blocked << 32) | p
 *                          -> blocked counts of every pose and the argmin (ties: lowest p)
 *   pcp_multi_score_poses  ncclAllReduce(ncclUint64, ncclMax) over [P totals (IEEE bits of
 *                          values >= +0) | P covered | 3 x n_cells newest-pose flag keys]
 *                          -> the reference's strict-'>' argmax (:471-474) and the stale-flag
 *                          colour statistics (:480-519), as pcp_score_poses.
 * Results are identical to one context over all poses.  The devices must be either all
 * distinct (RCCL) or all the same device (a rehearsal on one GPU: no communicator, the key
 * vectors are combined on that device by a kernel, pcp_multi_info reports uses_rccl = 0); a
 * mixed list such as {0, 0, 1} is refused with PCP_E_INVALID.  The per-device index builds
 * of pcp_multi_set_* run on one host thread per device.  Not thread-safe, like pcp_ctx. */
typedef struct pcp_multi pcp_multi;
int pcp_multi_create(int n_dev, const int *devices, pcp_multi **out);
void pcp_multi_destroy(pcp_multi *m);
const char *pcp_multi_last_error(const pcp_multi *m);
int pcp_multi_info(const pcp_multi *m, int *n_dev, int *uses_rccl);
pcp_ctx *pcp_multi_ctx(pcp_multi *m, int rank);   /* a rank's context (per-rank calls) */
int pcp_multi_set_terrain(pcp_multi *m, const pcp_cloud_view *terrain);
int pcp_multi_set_aux_cloud(pcp_multi *m, const pcp_cloud_view *aux);
int pcp_multi_set_cells(pcp_multi *m, const double *xyz, const float *normals, uint64_t n);
int pcp_multi_raycast_fan(pcp_multi *m, const double *poses5, uint64_t n,
                          const pcp_fan_params *fan, uint32_t *blocked, uint64_t *units,
                          int64_t *best_idx);
int pcp_multi_score_poses(pcp_multi *m, const double *poses5, uint64_t n,
                          const double zx120_pose5[5], const pcp_vl_params *p,
                          uint8_t *cell_flags, double *total_score, int32_t *covered,
                          pcp_vl_report *rep);

/* The march's sample distances: s_0 = 0.5, s_{k+1} = s_k + 0.3 (repeated double addition,
 * :765-796) while s_k < end.  Returns the count in *n (writes min(cap, n) values). */
int pcp_step_table(double end, double *steps, uint64_t cap, uint64_t *n);

/* Test infrastructure: the library's device exclusive scan (the index builds' prefix sums)
 * over a host array; out: n + 1 entries (out[n] = the total).  Scans of 2-64 tiles of 2,048
 * run as one look-back pass (PCP_SCAN_ONEPASS, default 1), others as three launches. */
int pcp_debug_exclusive_scan(pcp_ctx *ctx, const uint32_t *in, uint64_t n, uint32_t *out);

/* diagnostics of the terrain index (cell edge, dims, points) */
typedef struct pcp_index_info {
    uint64_t n_points;
    double cell;
    int32_t nx, ny, nz;
    double bmin[3], bmax[3];
    /* the layout the terrain scans walk: 0 per-cell runs, 1 2x2x2 block copy, 2 fine-window
       copy (the copies are built at the second query after pcp_set_terrain) */
    int32_t scan_layout;
    /* fine-window record layout (scan_layout 2): 0 x-fastest 8-byte records, 1 4 x 4 tiles of
       them, 2 split records -- 2-byte probe thresholds + 4-byte walk starts, 8 x 8 tiles (this
       field sits in what was the struct's tail padding: the size is unchanged) */
    int32_t fine_tile;
} pcp_index_info;
int pcp_terrain_info(pcp_ctx *ctx, pcp_index_info *info);

#ifdef __cplusplus
}
#endif
#endif /* PCP_ABI_H */
