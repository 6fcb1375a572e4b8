// pcp_nodes.hpp -- C++ host side above the C ABI: the algorithm part of the reference's three
// ROS2 nodes, with the reference's class and method names, parameter names/defaults and
// log-and-skip error behaviour.  No ROS dependency: an rclcpp shell owns one of these per node
// and forwards its callbacks.  Every compute call goes to libpcp (HIP).
#pragma once

#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "pcp_abi.h"

namespace pcp {

// ---- sensor_msgs::msg::PointCloud2 (the fields the nodes read/write) -------------------------
struct PointField {
    enum : uint8_t { INT8 = 1, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 };
    std::string name;
    uint32_t offset = 0;
    uint8_t datatype = FLOAT32;
    uint32_t count = 1;
};

struct PointCloud2 {
    std::string frame_id;
    double stamp = 0.0;
    uint32_t height = 1, width = 0;
    std::vector<PointField> fields;
    bool is_bigendian = false;
    uint32_t point_step = 0, row_step = 0;
    std::vector<uint8_t> data;
    bool is_dense = true;
    size_t size() const { return (size_t)width * height; }
    bool empty() const { return size() == 0; }
};

// pcl::toROSMsg layouts
PointCloud2 make_xyz_cloud(const float *xyz16, size_t n, const std::string &frame);  // PointXYZ
PointCloud2 make_xyzrgb_cloud(const void *rec32, size_t n, const std::string &frame);
// the pcl::fromROSMsg field lookup: FLOAT32 x/y/z by name
bool cloud_view(const PointCloud2 &m, pcp_cloud_view &v, std::string *why = nullptr);

struct Transform {   // geometry_msgs::msg::Transform
    double t[3] = {0, 0, 0};
    double q[4] = {0, 0, 0, 1};   // x, y, z, w
};

// one HIP device context shared by the node cores of a process
class Device {
   public:
    explicit Device(int device = 0);
    ~Device();
    Device(const Device &) = delete;
    Device &operator=(const Device &) = delete;
    pcp_ctx *ctx() const { return ctx_; }
    const char *error() const { return pcp_last_error(ctx_); }

   private:
    friend class MultiDevice;
    struct Borrow {};
    Device(pcp_ctx *ctx, Borrow) : ctx_(ctx), owned_(false) {}   // a MultiDevice rank's context
    pcp_ctx *ctx_ = nullptr;
    bool owned_ = true;
};

// n GPUs in this process (pcp_multi: one context per device + one RCCL communicator).  The
// virtual-LiDAR node shards its candidate poses over them; rank 0's context serves every
// other call (candidate generation, the excavation-area setup, the other nodes).
class MultiDevice {
   public:
    explicit MultiDevice(const std::vector<int> &devices);
    ~MultiDevice();
    MultiDevice(const MultiDevice &) = delete;
    MultiDevice &operator=(const MultiDevice &) = delete;
    pcp_multi *get() const { return m_; }
    int size() const { return n_; }
    bool usesRccl() const { return rccl_; }
    Device &rank0() { return *r0_; }
    const char *error() const { return pcp_multi_last_error(m_); }

   private:
    pcp_multi *m_ = nullptr;
    int n_ = 0;
    bool rccl_ = false;
    std::unique_ptr<Device> r0_;
};

// ---- pointcloud_filter.cpp (SimplifiedScanMatcher) -----------------------------------------
class SimplifiedScanMatcher {
   public:
    struct Params {   // pointcloud_filter.cpp:30-39
        double robot_front_range = 15.0, robot_side_range = 10.0, robot_height_range = 10.0;
        double backhoe_front_range = 15.0, backhoe_side_range = 10.0, backhoe_height_range = 10.0;
        double voxel_leaf_size = 0.2;
    };
    explicit SimplifiedScanMatcher(Device &dev) : dev_(dev) {}
    SimplifiedScanMatcher(Device &dev, const Params &p) : dev_(dev), p_(p) {}
    Params &params() { return p_; }
    const Params &params() const { return p_; }
    // callbacks (:52-62): the returned message is what the node publishes
    PointCloud2 robotCloudCallback(const PointCloud2 &msg) { return processCloudSimple(msg, "robot"); }
    PointCloud2 backhoeCloudCallback(const PointCloud2 &msg) { return processCloudSimple(msg, "backhoe"); }
    // fromROSMsg -> cropFrontArea -> downsampleCloud -> toROSMsg, header kept (:64-85)
    PointCloud2 processCloudSimple(const PointCloud2 &in, const std::string &vehicle_type);
    size_t lastCroppedSize() const { return last_cropped_; }
    const std::string &lastError() const { return err_; }

   private:
    Device &dev_;
    Params p_;
    size_t last_cropped_ = 0;
    std::vector<float> out_;   // result landing, reused (grown, never re-zeroed per message)
    std::string err_;
};

// ---- pointcloud_merger.cpp (GnssGicpMatcher, cloud part) ------------------------------------
class GnssGicpMatcher {
   public:
    explicit GnssGicpMatcher(Device &dev) : dev_(dev) {}
    void robotCloudCallback(const PointCloud2 &msg) { robot_ = msg; have_robot_ = true; }      // :176-178
    void backhoeCloudCallback(const PointCloud2 &msg) { backhoe_ = msg; have_backhoe_ = true; } // :180-182
    struct Output {
        PointCloud2 merged, robot_colored, backhoe_colored;   // /matched_point_cloud, ...
    };
    // processPointClouds (:308-352).  The caller did the TF lookups map <- */velodyne_link
    // (:362-366); nullptr = the lookup threw, and that robot is skipped (:389-393).
    Output processPointClouds(bool origin_set, const Transform *robot_tf, const Transform *zx120_tf);
    const std::string &lastError() const { return err_; }

   private:
    Device &dev_;
    PointCloud2 robot_, backhoe_;
    bool have_robot_ = false, have_backhoe_ = false;
    std::vector<uint8_t> out_;   // result landing, reused
    std::string err_;
};

// ---- the filter node (both sensors) + the merger node, composed in one process ----------------
// (a component container / the C5 chain): per frame ONE call, pcp_filter_merge_nodes -- both
// /filtered_points messages exactly as SimplifiedScanMatcher publishes them and the merged cloud
// exactly as GnssGicpMatcher::processPointClouds publishes it, with one synchronisation instead
// of three.  Transforms: nullptr = the TF lookup threw, that robot is skipped in the merge (its
// filtered message is still produced), as the two nodes do.
class ComposedFilterMerge {
   public:
    explicit ComposedFilterMerge(Device &dev) : dev_(dev) {}
    ComposedFilterMerge(Device &dev, const SimplifiedScanMatcher::Params &p) : dev_(dev), p_(p) {}
    struct Output {
        PointCloud2 robot_filtered, backhoe_filtered;   // the filter node's two messages
        GnssGicpMatcher::Output merge;                  // the merger node's outputs
        // merge.merged's bytes where libpcp landed them (pcp_filter_merge_landed; n = 0 when
        // none): valid until the context's next filter / merge / carve call -- a carve composed
        // behind this call reads them in place (SimplifiedDualLidarOptimizer::carveCallbacks)
        pcp_cloud_view merged_landed{};
        // frame(..., defer_messages = true): the messages' data not copied yet -- merge.merged
        // carries its header (width, fields) only, the rest are empty -- until messages(o)
        bool deferred = false;
        struct Pending {
            const float *filtered[2] = {nullptr, nullptr};
            const uint8_t *merged = nullptr;
            uint64_t per[2] = {0, 0}, keep_off = 0, keep_n = 0;
            bool tf[2] = {false, false}, origin_set = false;
        } pending;
    };
    // defer_messages: the launches and the one synchronisation only; the five messages are
    // copied out of the landing by messages(o) -- e.g. after a composed carve has read the
    // merged cloud in place (SimplifiedDualLidarOptimizer::carveCallbacks), so the copies run
    // while the device builds the grid.  Valid until the context's next filter / merge call
    Output frame(const PointCloud2 &robot, const PointCloud2 &backhoe, bool origin_set,
                 const Transform *robot_tf, const Transform *zx120_tf, bool defer_messages = false);
    void messages(Output &o) const;
    const std::string &lastError() const { return err_; }

   private:
    Device &dev_;
    SimplifiedScanMatcher::Params p_;
    std::string err_;
};

// ---- excavated_surface_generator.cpp (ExcavationTerrainGenerator) --------------------------
class ExcavationTerrainGenerator {
   public:
    struct Params : pcp_excavation_params {   // :29-51 defaults, excavation.enabled
        bool enabled = true;
        Params() : pcp_excavation_params{1.0, 75.0, 4.0, 1.0, 0.05, 0.5, 1, 2.0, 1.2, 2.0, 1.2,
                                         1.2, 1.8} {}
    };
    struct Output {
        PointCloud2 excavated_terrain;   // /excavated_terrain (frame map)
        PointCloud2 excavation_area;     // /excavation_area (frame map); empty: not published
        bool area_published = false;
        double center[3] = {0, 0, 0}, yaw = 0;   // publishExcavationMarkers pose
    };
    explicit ExcavationTerrainGenerator(Device &dev) : dev_(dev) {}
    ExcavationTerrainGenerator(Device &dev, const Params &p) : dev_(dev), p_(p) {}
    Params &params() { return p_; }
    const Params &params() const { return p_; }
    // matchedCloudCallback (:259-326); zx120_base = TF map -> zx120/base_link, nullptr = the
    // lookup threw: the input is republished unchanged (as when disabled, :260-263, :276-279)
    Output matchedCloudCallback(const PointCloud2 &msg, const Transform *zx120_base);
    const std::string &lastError() const { return err_; }

   private:
    friend class SimplifiedDualLidarOptimizer;   // carveCallbacks: the composed chain
    Device &dev_;
    Params p_;
    // result landings sized by pcp_excavate_bounds (MBs: the generated-point capacities), reused
    // so no message pays for zero-filling them
    std::vector<uint8_t> terr_, area_;
    std::string err_;
};

// ---- calc_drivable_area.cpp (its class is also named SimplifiedScanMatcher upstream) --------
struct OccupancyGrid {   // nav_msgs::msg::OccupancyGrid (the fields the node fills)
    std::string frame_id = "map";
    double resolution = 0;
    uint32_t width = 0, height = 0;
    double origin_x = 0, origin_y = 0;   // orientation w = 1
    std::vector<int8_t> data;            // 0 free, 100 obstacle, -1 unknown
};

class DrivableAreaMapper {
   public:
    explicit DrivableAreaMapper(Device &dev) : dev_(dev) { p_ = pcp_drivable_params{1.0, 100.0, 100.0, 0.3, 10, 3.0}; }
    DrivableAreaMapper(Device &dev, const pcp_drivable_params &p) : dev_(dev), p_(p) {}
    // robotCloudCallback (:67-226): cloud_to_map = the TF of the cloud's frame (nullptr: not
    // available, skipped :76-96), robot_base = map -> four_wheel_robot/base_link (nullptr:
    // skipped :114-126).  Returns false when nothing is published (also an empty cloud).
    bool robotCloudCallback(const PointCloud2 &msg, const Transform *cloud_to_map,
                            const Transform *robot_base, OccupancyGrid &out);
    bool startSet() const { return start_set_; }
    const std::string &lastError() const { return err_; }

   private:
    Device &dev_;
    pcp_drivable_params p_;
    bool start_set_ = false;   // start_position_initialized_
    double start_x_ = 0, start_y_ = 0;
    std::string err_;
};

// ---- virtual_lidar.cpp (SimplifiedDualLidarOptimizer) --------------------------------------
class SimplifiedDualLidarOptimizer {
   public:
    struct Params {   // virtual_lidar.cpp:66-71
        double grid_resolution = 0.1, sensor_height = 1.1, search_radius = 3.0,
               max_distance = 15.0;
        int num_candidates = 100, vertical_layers = 10;
    };
    struct LidarPosition {   // :46-51
        double x = 0, y = 0, z = 10, pitch = -M_PI / 2, yaw = 0, total_score = 0;
    };
    struct Result {
        bool ran = false;                  // false: early return of :455
        LidarPosition best;                // /optimal_mobile_lidar_position
        double best_score = -INFINITY;
        LidarPosition zx120;
        std::vector<LidarPosition> candidates;   // with total_score (publishCandidatePositions)
        pcp_vl_report report{};
        std::string log;                   // the RCLCPP_INFO tables (:419-451, :522-543)
    };
    explicit SimplifiedDualLidarOptimizer(Device &dev) : dev_(dev) {}
    SimplifiedDualLidarOptimizer(Device &dev, const Params &p) : dev_(dev), p_(p) {}
    // the candidate loop sharded over the devices of md (one collective per tick)
    explicit SimplifiedDualLidarOptimizer(MultiDevice &md) : dev_(md.rank0()), multi_(md.get()) {}
    SimplifiedDualLidarOptimizer(MultiDevice &md, const Params &p)
        : dev_(md.rank0()), multi_(md.get()), p_(p) {}
    Params &params() { return p_; }
    const Params &params() const { return p_; }
    // excavationAreaCallback (:164-178): GPU normals + 3-D cell grid from /excavation_area;
    // an empty cloud keeps the previous grid (:168).  true: generateExcavationGrid3D ran to its
    // end (:284-286) -- the shell then logs the grid size and publishes the grid markers
    bool excavationAreaCallback(const PointCloud2 &msg);
    void terrainCallback(const PointCloud2 &msg);       // :180-192
    void zx120PointsCallback(const PointCloud2 &msg);   // :194-207
    // cells computed elsewhere (tests, replays): the valid cells of generateExcavationGrid3D
    // (:236-287) with computeCellSurfaceNormal; grid_bbox = grid_min_x, grid_max_x,
    // grid_min_y, grid_max_y, excavation_min_z/max_z
    void setExcavationGrid(const std::vector<double> &xyz, const std::vector<float> &normals,
                           const double grid_bbox[6]);
    // runOptimization (:454-548); zx120_base = TF map -> zx120/base_link, nullptr = missing
    Result runOptimization(const Transform *zx120_base);
    const std::vector<uint8_t> &cellFlags() const { return flags_; }
    // settles a pending deferred grid first (may wait for the device)
    size_t lastCells();
    // composed chain (intra-process nodes, e.g. the C5 replay): excavationAreaCallback enqueues
    // the grid setup and returns without waiting (pcp_set_excavation_area_async); the next
    // runOptimization waits once for both.  Off by default: a ROS shell publishes the grid
    // markers from the area callback, which needs the cells there
    void setDeferredGrid(bool on) { defer_grid_ = on && !multi_; }
    // composed chain: gen's matchedCloudCallback, then this node's excavationAreaCallback (when
    // the area is published) and terrainCallback for gen's two messages, in one call
    // (pcp_excavate_area_async: the carve's records feed the deferred grid setup and the terrain
    // index where they land, no re-upload).  Same messages, same state as the three calls; with
    // the grid not deferred (or sharded, or the carve disabled / its TF missing) it makes them.
    // Errors: gen.lastError() for the carve, lastError() for the two callbacks
    // landed (nullable): merged's bytes in the context's pinned landing
    // (ComposedFilterMerge::Output::merged_landed), read in place instead of the message --
    // which may then be its header only (a deferred ComposedFilterMerge frame) as long as the
    // composed path applies (grid deferred, one device, carve enabled, TF present).
    // zx120 (nullable): this node's zx120PointsCallback for that message as well, made after
    // the carve's consumers are enqueued and before gen's two messages are built from the
    // carve's landed records (pcp_excavate_landed): the zx120 index builds while the host copies
    ExcavationTerrainGenerator::Output carveCallbacks(ExcavationTerrainGenerator &gen,
                                                      const PointCloud2 &merged,
                                                      const Transform *zx120_base,
                                                      const pcp_cloud_view *landed = nullptr,
                                                      const PointCloud2 *zx120 = nullptr);
    const std::string &lastError() const { return err_; }

   private:
    Device &dev_;
    pcp_multi *multi_ = nullptr;   // non-null: poses sharded over its devices
    Params p_;
    bool terrain_cloud_ = false;   // terrain_cloud_ non-null (a message arrived)
    size_t zx120_size_ = 0;        // zx120_cloud_->size() (:433-434)
    size_t n_cells_ = 0;           // deferred: the lattice's capacity until settled
    bool defer_grid_ = false;
    bool grid_pending_ = false;    // a deferred setup whose count is not settled yet
    double bbox_[6] = {0, 0, 0, 0, 0, 0};
    std::vector<uint8_t> flags_;   // GridCell flag state across ticks
    std::string err_;
};

// runOptimization's two RCLCPP_INFO tables (virtual_lidar.cpp:419-451, :522-543) from a report:
// host arithmetic only (the percentages in the reference's expression order, line by line)
std::string optimization_log(const SimplifiedDualLidarOptimizer::LidarPosition &zx120,
                             const SimplifiedDualLidarOptimizer::LidarPosition &best,
                             double best_score, const pcp_vl_report &q, size_t zx120_size);

}  // namespace pcp
