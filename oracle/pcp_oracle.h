/*
 * pcp_oracle.h -- CPU restatement of YamaguchiAtsushi/pointcloud_processor's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the timed CPU
 * baseline -- never as the product path.  The product is libpcp.so (HIP, gfx950).
 *
 * PARITY UNPINNED: the reference cannot be built here (it needs rclcpp, PCL, FLANN,
 * Eigen, tf2 and GeographicLib; none are installed and there is no network) and it
 * ships no tests, fixtures or golden vectors.  This restatement
 * follows the reference sources line by line (cited per function) and restates the
 * third-party arithmetic (PCL 1.12.1 KdTreeFLANN/VoxelGrid, FLANN 1.9.1 L2_Simple,
 * Eigen 3.4 Quaternionf/Affine3f as used by tf2_sensor_msgs::doTransform) from their
 * published algorithms.  Independent cross-checks (numpy brute force, scipy cKDTree)
 * live in tests/test_oracle.py.
 *
 * All arithmetic is compiled with -ffp-contract=off (no FMA), matching a generic
 * x86-64 build of the reference (SSE2 only, no contraction).
 */
#ifndef PCP_ORACLE_H
#define PCP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* thread count for the OpenMP-parallel fan raycast (CPU baseline). 1 = faithful
 * single-threaded executor of the reference (virtual_lidar.cpp:965-970). */
void orc_set_threads(int n);
int orc_get_threads(void);

/* ---- pointcloud_filter.cpp ---------------------------------------------------- */
/* cropFrontArea (pointcloud_filter.cpp:106-116): strict box, float coord vs double
 * bound, order-preserving. box = {xlo,xhi,ylo,yhi,zlo,zhi}. Returns kept count. */
int64_t orc_crop_box(const float *pts, int64_t n, int64_t stride_floats,
                     const double box[6], uint32_t *kept_idx);

/* downsampleCloud -> pcl::VoxelGrid<PointXYZ>::applyFilter (pointcloud_filter.cpp:122-139).
 * Output in ascending voxel index. *passthrough=1 when PCL's int32 overflow guard fires
 * (output = input copied, idx/count untouched). Returns n_out. */
int64_t orc_voxel_grid(const float *pts, int64_t n, int64_t stride_floats, float leaf,
                       float *out_xyz /*3*n*/, uint32_t *out_idx /*n*/,
                       uint32_t *out_count /*n*/, int *passthrough);

/* ---- pointcloud_merger.cpp ------------------------------------------------------ */
/* processRobotCloud (pointcloud_merger.cpp:354-394): tf2::doTransform (Eigen float
 * Translation3f * Quaternionf) + PointXYZRGB colour tag.  out8 = 8 floats per point
 * (PointXYZRGB memory image: x,y,z,1.0f, rgba(u32), 0,0,0). q = {x,y,z,w}. */
void orc_transform_rgb(const float *pts, int64_t n, int64_t stride_floats,
                       const double t[3], const double q[4],
                       uint8_t r, uint8_t g, uint8_t b, float *out8);

/* the whole C3 frame on `threads` OpenMP threads (pcp_oracle_mt.c; bench.py's MT CPU
 * baseline): per cloud crop -> VoxelGrid(leaf > 0) -> transform + colour, concatenated in
 * cloud order into out8 (PointXYZRGB records); the bytes of the sequential composition.
 * t3q4: per cloud t[3] then q[4] (x, y, z, w).  Returns the record count, -1 on overflow of
 * cap or leaf <= 0. */
int64_t orc_filter_frame_mt(int k, const float *const *pts, const int64_t *n,
                            const int64_t *stride, const double *boxes, float leaf,
                            const double *t3q4, const uint8_t *rgb, float *out8, int64_t cap,
                            int64_t *n_per, int threads);

#define VL_MIN_DISTANCE 0.5
#define VL_ZX120_OFFSET_X 0.4
#define VL_RAY_STEP_SIZE 0.3
#define VL_VISIBILITY_RADIUS 0.08

/* ---- virtual_lidar.cpp ------------------------------------------------------------ */
typedef struct orc_cloud orc_cloud;   /* exact radius-search structure (uniform grid) */
typedef struct orc_kdtree orc_kdtree; /* restated KdTreeFLANN (pcp_flann.c) */
orc_cloud *orc_cloud_build(const float *pts, int64_t n, int64_t stride_floats);
void orc_cloud_free(orc_cloud *c);
/* KdTreeFLANN::radiusSearch(q, radius) > 0  (FLANN L2_Simple, dist < float(r*r)) */
int orc_cloud_any_within(const orc_cloud *c, float qx, float qy, float qz, double radius);
/* the number of points with L2_Simple distance < float(r*r) (exact: every candidate cell) */
int64_t orc_cloud_count_within(const orc_cloud *c, float qx, float qy, float qz, double radius);

/* ---- pcp_flann.c: FLANN 1.9.1 KDTreeSingleIndex as PCL 1.12.1 KdTreeFLANN configures it
 * (the second, independent checker of the radius predicate; see pcp_flann.c) -------------- */
orc_kdtree *orc_kd_build(const float *pts, int64_t n, int64_t stride_floats, int leaf_max);
void orc_kd_free(orc_kdtree *t);
int64_t orc_kd_size(const orc_kdtree *t);
const float *orc_kd_point(const orc_kdtree *t, int64_t cloud_idx);
/* FLANN mode: every radius query of the oracle on c (ray march, relaxed check, ground
 * height) goes through kd instead of the grid scan; NULL restores the grid */
void orc_cloud_use_kdtree(orc_cloud *c, const orc_kdtree *kd);
/* radiusSearch with r2 = float(r*r) already formed; idx (nullable) gets up to cap neighbours'
 * indices in the caller's cloud (tree order, unsorted) */
int64_t orc_kd_radius(const orc_kdtree *t, float qx, float qy, float qz, float r2,
                      int64_t *idx, int64_t cap);
int64_t orc_kd_radius_search(const orc_kdtree *t, float qx, float qy, float qz, double radius);
void orc_kd_check_queries(const orc_kdtree *t, const orc_cloud *g, const float *q, int64_t nq,
                          double radius, uint64_t stats[4]);
void orc_kd_raycast_fan(const orc_kdtree *t, const orc_cloud *g, const double *poses5, int64_t P,
                        int32_t n_az, int32_t n_el, double el_min, double el_max,
                        double max_distance, int16_t *first_hit, uint32_t *blocked,
                        uint64_t *units, uint64_t stats[4]);
/* getGroundHeight (virtual_lidar.cpp:600-625) */
double orc_ground_height(const orc_cloud *terrain, double x, double y);

/* params (virtual_lidar.cpp:66-71) */
typedef struct orc_vl_params {
    double grid_resolution, sensor_height, search_radius, max_distance;
    int32_t num_candidates, vertical_layers;
} orc_vl_params;

/* generateCandidatePositions (virtual_lidar.cpp:550-598). bbox = {grid_min_x, grid_max_x,
 * grid_min_y, grid_max_y, excavation_min_z, excavation_max_z} (margin already applied,
 * :251-254). zx120 = {x,y,z,pitch,yaw}. Writes poses5 (x,y,z,pitch,yaw), returns count. */
int64_t orc_generate_candidates(const orc_cloud *terrain, int terrain_empty,
                                const double bbox[6], const orc_vl_params *p,
                                const double zx120[5], double *poses5, int64_t cap);

/* Cell flag bits (GridCell, virtual_lidar.cpp:20-44) */
enum {
    ORC_F_RANGE_Z = 1, ORC_F_FOV_Z = 2, ORC_F_VIS_Z = 4,
    ORC_F_RANGE_M = 8, ORC_F_FOV_M = 16, ORC_F_VIS_M = 32
};

typedef struct orc_vl_report {
    int64_t best_idx;          /* -1 when there are no candidates */
    double best_score;         /* -inf when there are no candidates (:464) */
    double zx120_total_score;  /* evaluateZX120Only (:360-452) */
    int32_t zx120_range_ok, zx120_fov_ok, zx120_visible_ok;
    int32_t total_cells;
    int32_t zx120_green, zx120_red, zx120_blue, zx120_yellow;
    int32_t green, red, blue, yellow;   /* dual stats (:480-519) */
} orc_vl_report;

/* runOptimization body after generateCandidatePositions (virtual_lidar.cpp:460-519):
 * evaluateZX120Only, then for each candidate evaluatePosition (zx120 + mobile per cell,
 * :627-654), strict-> argmax, colour statistics from the stale flags.
 * terrain may be NULL (no terrain KD-tree -> visible), aux may be NULL/empty.
 * cell_flags is in/out GridCell state. total_score/covered: per candidate. */
void orc_score_poses(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                     const double *cells_xyz, const float *cells_nrm, int64_t n_cells,
                     const double *poses5, int64_t n_poses, const double zx120[5],
                     const orc_vl_params *p, uint8_t *cell_flags,
                     double *total_score, int32_t *covered, orc_vl_report *rep);
/* per-pose totals/covered only (no flags), OpenMP over poses: the CPU baseline's MT leg */
void orc_score_totals(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                      const double *cells_xyz, const float *cells_nrm, int64_t n_cells,
                      const double *poses5, int64_t n_poses, const double zx120[5],
                      const orc_vl_params *p, double *total_score, int32_t *covered);

/* evaluateCellScore per (pose, cell) and for the zx120 pose (the per-cell parity bar):
 * sm [n_poses][n_cells] = score_mobile, sz [n_cells] = score_zx120 */
void orc_score_matrix(const orc_cloud *terrain, const orc_cloud *aux, int64_t aux_n,
                      const double *cells_xyz, const float *cells_nrm, int64_t n_cells,
                      const double *poses5, int64_t n_poses, const double zx120[5],
                      const orc_vl_params *p, double *sm, double *sz);

/* Dense azimuth x elevation fan (BASELINE configs[1]): per pose, ray
 * (az_i, el_j) with local dir (cos el cos a_i, cos el sin a_i, sin el), a_i = 2*pi*i/n_az,
 * el_j = el_min + (el_max-el_min)*(j+0.5)/n_el, rotated by the pose yaw; marched with
 * checkVisibilityWithRaycasting's rule (virtual_lidar.cpp:765-797) to end = max_distance
 * - VISIBILITY_RADIUS.  first_hit[p][j][i] = sample index of the first blocked sample or -1.
 * blocked[p] = rays with a hit; units[p] = sample queries the reference would execute. */
void orc_raycast_fan(const orc_cloud *terrain, const double *poses5, int64_t n_poses,
                     int32_t n_az, int32_t n_el, double el_min, double el_max,
                     double max_distance, int16_t *first_hit /*nullable*/,
                     uint32_t *blocked, uint64_t *units);

/* The ray-local direction tables of the fan (shared definition with libpcp). */
void orc_fan_tables(int32_t n_az, int32_t n_el, double el_min, double el_max,
                    double *ca, double *sa, double *ce, double *se);

/* ---- excavation-area setup (pcp_oracle_setup.c) ------------------------------------------
 * computeTerrainNormals (virtual_lidar.cpp:209-234): pcl::NormalEstimation, radius 1.5,
 * viewpoint (0,0,0), then flipped to normal_z >= 0; < 3 neighbours -> NaN.  normals3: n x 3. */
void orc_area_normals(const float *pts, int64_t n, int64_t stride_floats, double radius,
                      float *normals3);

/* generateExcavationGrid3D (:236-287) with isPointNearExcavation (radius 1.5 * resolution)
 * and computeCellSurfaceNormal (:301-340) from area_normals3 (NULL: default (0,0,1)).
 * Cells in the reference's loop order (rows i over y, columns j over x, layers k).  Returns
 * the number of valid cells (writes at most cap); grid_bbox = x0, x1, y0, y1, z0, z1 after
 * the margin; dims = grid_height, grid_width, layers. */
int64_t orc_excavation_grid(const float *pts, int64_t n, int64_t stride_floats,
                            double grid_resolution, int32_t vertical_layers,
                            const float *area_normals3, double *cells_xyz, float *cells_nrm,
                            int64_t cap, double grid_bbox[6], int32_t dims[3]);

/* ---- excavated_surface_generator.cpp (pcp_oracle_setup.c) -------------------------------- */
typedef struct orc_exc_params {
    double depth, slope_angle_deg, offset_x, offset_y, point_density, terrain_search_radius;
    int32_t l_shape_enabled;
    double arm1_length, arm1_width, arm2_length, arm2_width, width, length;
} orc_exc_params;

/* getTerrainHeight (:183-226) over the cloud (FLANN radius search from (x, y, 0), 2-D filter,
 * mean z in result order; else the nearest point's z; else 0) */
double orc_terrain_height(const float *pts, int64_t n, int64_t stride_floats, double x, double y,
                          double radius);

/* matchedCloudCallback with the TF present (:259-326): zx120 base transform t, q (x,y,z,w).
 * keep[i] = 1 for the input points processExcavation keeps (:451-485); surf = the points
 * generateExcavatedSurface appends (:487-584), area = generateExcavationArea's cloud
 * (:350-455), both as (x, y, z, rgb-float) rows; pose_out = centre x, y, terrain z, yaw. */
void orc_excavate(const float *pts, int64_t n, int64_t stride_floats, const orc_exc_params *p,
                  const double t[3], const double q[4], uint8_t *keep, float *surf,
                  int64_t cap_surf, int64_t *n_surf, float *area, int64_t cap_area,
                  int64_t *n_area, double pose_out[4]);

/* calc_drivable_area.cpp robotCloudCallback (:67-226): grid gh rows x gw int8 (0 / 100 / -1),
 * dims = gw, gh; origin = robot - map/2.  t, q: cloud frame -> map (x, y, z, w). */
void orc_drivable_area(const float *pts, int64_t n, int64_t stride_floats, const double t[3],
                       const double q[4], double robot_x, double robot_y, double start_x,
                       double start_y, double res, double map_w, double map_h,
                       double max_gradient, int32_t min_points, double clear_r, int8_t *grid,
                       int32_t dims[2], double origin[2]);

#ifdef __cplusplus
}
#endif
#endif
