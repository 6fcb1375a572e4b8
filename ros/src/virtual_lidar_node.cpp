// virtual_lidar: the rclcpp shell of virtual_lidar.cpp (SimplifiedDualLidarOptimizer) -- node
// name, parameters, topics, the 3 s optimisation timer and the three outputs of :62-97,
// :454-548, :802-962.  Normals, the 3-D cell grid, candidate generation, the ray-fan
// occlusion scoring and the argmax run in libpcp; this file only moves messages.
//
// PCP_DEVICES="0,1,2,3" shards the candidate poses over those GPUs (pcp_multi: one RCCL
// all-reduce of the per-pose score keys per tick); unset, one GPU (PCP_DEVICE, default 0).
#include "pcp_ros.hpp"

#include <algorithm>
#include <sstream>

#include <geometry_msgs/msg/point_stamped.hpp>
#include <visualization_msgs/msg/marker_array.hpp>

using namespace std::chrono_literals;
using Marker = visualization_msgs::msg::Marker;

namespace {
std::vector<int> devices_from_env() {
    std::vector<int> d;
    if (const char *s = std::getenv("PCP_DEVICES")) {
        std::stringstream ss(s);
        std::string tok;
        while (std::getline(ss, tok, ','))
            if (!tok.empty()) d.push_back(std::atoi(tok.c_str()));
    }
    return d;
}
}  // namespace

class SimplifiedDualLidarOptimizerNode : public rclcpp::Node {
   public:
    SimplifiedDualLidarOptimizerNode() : Node("simplified_dual_lidar_optimizer") {
        const std::vector<int> devs = devices_from_env();
        if (devs.size() > 1) {
            multi_ = std::make_unique<pcp::MultiDevice>(devs);
            core_ = std::make_unique<pcp::SimplifiedDualLidarOptimizer>(*multi_);
            dev_ = &multi_->rank0();
            RCLCPP_INFO(get_logger(), "Scoring sharded over %d GPUs (%s)", multi_->size(),
                        multi_->usesRccl() ? "RCCL all-reduce"
                                           : "one device: on-device key combine");
        } else {
            dev_ = &pcp_ros::device();
            core_ = std::make_unique<pcp::SimplifiedDualLidarOptimizer>(*dev_);
        }
        tf_buffer_ = std::make_shared<tf2_ros::Buffer>(get_clock());
        tf_listener_ = std::make_shared<tf2_ros::TransformListener>(*tf_buffer_);
        declare_parameter("grid_resolution", 0.1);
        declare_parameter("sensor_height", 1.1);
        declare_parameter("search_radius", 3.0);
        declare_parameter("max_distance", 15.0);
        declare_parameter("num_candidates", 100);
        declare_parameter("vertical_layers", 10);
        updateParameters();

        excavation_area_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/excavation_area", 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) {
                // generateExcavationGrid3D logs the grid and republishes the grid markers, from
                // the fresh cells' flags, every time it runs (:284-286)
                if (core_->excavationAreaCallback(pcp_ros::from_ros(*m))) {
                    RCLCPP_INFO(get_logger(),
                                "Generated 3D grid: %d valid cells across %d vertical layers",
                                (int)core_->lastCells(), core_->params().vertical_layers);
                    publishGridVisualization();
                } else {
                    report("Failed to process excavation area");
                }
            });
        terrain_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/excavated_terrain", 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) {
                core_->terrainCallback(pcp_ros::from_ros(*m));
                terrain_cloud_ = true;
                report("Failed to build terrain KD-tree");
            });
        zx120_points_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/zx120/filtered_points", 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) {
                core_->zx120PointsCallback(pcp_ros::from_ros(*m));
                if (!report("Failed to build ZX120 KD-tree") && m->width * m->height > 0)
                    RCLCPP_INFO(get_logger(), "ZX120 point cloud updated: %u points",
                                m->width * m->height);
            });
        optimal_position_pub_ =
            create_publisher<geometry_msgs::msg::PointStamped>("/optimal_mobile_lidar_position", 10);
        candidate_positions_pub_ = create_publisher<visualization_msgs::msg::MarkerArray>(
            "/mobile_lidar_candidate_positions", 10);
        grid_visualization_pub_ = create_publisher<visualization_msgs::msg::MarkerArray>(
            "/excavation_grid_visualization", 10);
        optimization_timer_ = create_wall_timer(3s, [this] { runOptimization(); });
    }

   private:
    bool report(const char *what) {
        if (core_->lastError().empty()) return false;
        RCLCPP_ERROR(get_logger(), "%s: %s", what, core_->lastError().c_str());
        return true;
    }

    void updateParameters() {   // :155-162
        auto &p = core_->params();
        p.grid_resolution = get_parameter("grid_resolution").as_double();
        p.sensor_height = get_parameter("sensor_height").as_double();
        p.search_radius = get_parameter("search_radius").as_double();
        p.max_distance = get_parameter("max_distance").as_double();
        p.num_candidates = (int)get_parameter("num_candidates").as_int();
        p.vertical_layers = (int)get_parameter("vertical_layers").as_int();
    }

    void runOptimization() {
        // :455 -- the early return comes before updateParameters (:457), so a parameter change
        // reaches the next excavation grid only once a tick has run
        pcp::Transform zx120;
        if (core_->lastCells() == 0 || !terrain_cloud_ ||
            !pcp_ros::lookup(*tf_buffer_, "map", "zx120/base_link", 0.1, zx120, nullptr))
            return;
        updateParameters();
        const pcp::SimplifiedDualLidarOptimizer::Result r = core_->runOptimization(&zx120);
        if (report("Optimization failed") || !r.ran) return;
        std::istringstream log(r.log);   // the two RCLCPP_INFO tables, line by line
        for (std::string line; std::getline(log, line);) RCLCPP_INFO(get_logger(), "%s", line.c_str());
        const auto stamp = now();
        publishOptimalPosition(r, stamp);
        publishCandidatePositions(r, stamp);
        publishGridVisualization();
    }

    void publishOptimalPosition(const pcp::SimplifiedDualLidarOptimizer::Result &r,
                                const rclcpp::Time &stamp) {   // :802-811
        geometry_msgs::msg::PointStamped m;
        m.header.stamp = stamp;
        m.header.frame_id = "map";
        m.point.x = r.best.x;
        m.point.y = r.best.y;
        m.point.z = r.best.z;
        optimal_position_pub_->publish(m);
    }

    static Marker marker(const rclcpp::Time &stamp, const char *ns, int id, int type, double x,
                         double y, double z, double sx, double sy, double sz, float cr, float cg,
                         float cb, float ca, double lifetime_s) {
        Marker m;
        m.header.stamp = stamp;
        m.header.frame_id = "map";
        m.ns = ns;
        m.id = id;
        m.type = type;
        m.action = Marker::ADD;
        m.pose.position.x = x;
        m.pose.position.y = y;
        m.pose.position.z = z;
        m.pose.orientation.w = 1.0;
        m.scale.x = sx;
        m.scale.y = sy;
        m.scale.z = sz;
        m.color.r = cr;
        m.color.g = cg;
        m.color.b = cb;
        m.color.a = ca;
        m.lifetime = rclcpp::Duration::from_seconds(lifetime_s);
        return m;
    }

    void publishCandidatePositions(const pcp::SimplifiedDualLidarOptimizer::Result &r,
                                   const rclcpp::Time &stamp) {   // :813-906
        visualization_msgs::msg::MarkerArray arr;
        Marker clear;
        clear.action = Marker::DELETEALL;
        arr.markers.push_back(clear);
        arr.markers.push_back(marker(stamp, "zx120_lidar", 0, Marker::CUBE, r.zx120.x, r.zx120.y,
                                     r.zx120.z, 0.5, 0.5, 0.5, 0, 1, 1, 1, 10.0));
        for (size_t i = 0; i < r.candidates.size(); ++i) {
            const auto &c = r.candidates[i];
            arr.markers.push_back(marker(stamp, "mobile_lidar_candidates", (int)i, Marker::SPHERE,
                                         c.x, c.y, c.z, 0.3, 0.3, 0.3, 1, 1, 0, 0.7f, 8.0));
        }
        arr.markers.push_back(marker(stamp, "optimal_mobile_lidar", 0, Marker::CYLINDER, r.best.x,
                                     r.best.y, r.best.z, 1.0, 1.0, 2.0, 0, 0, 1, 0.9f, 10.0));
        candidate_positions_pub_->publish(arr);
    }

    void publishGridVisualization() {   // :908-962 (each marker stamped now(), :920)
        const rclcpp::Time stamp = now();
        uint64_t n = 0;
        pcp_get_cells(dev_->ctx(), nullptr, nullptr, 0, &n);
        std::vector<double> xyz(3 * n);
        if (n && pcp_get_cells(dev_->ctx(), xyz.data(), nullptr, n, &n) != PCP_OK) return;
        const std::vector<uint8_t> &f = core_->cellFlags();
        const double s = core_->params().grid_resolution * 0.6;
        visualization_msgs::msg::MarkerArray arr;
        Marker clear;
        clear.action = Marker::DELETEALL;
        arr.markers.push_back(clear);
        for (uint64_t i = 0; i < n && i < f.size(); ++i) {
            const uint8_t b = f[i];
            float cr = 0, cg = 1, cb = 0;                                      // green
            if (!(b & (PCP_F_RANGE_Z | PCP_F_RANGE_M))) cr = 0, cg = 0, cb = 1;   // blue
            else if (!(b & (PCP_F_FOV_Z | PCP_F_FOV_M))) cr = 1, cg = 1, cb = 0;  // yellow
            else if (!(b & (PCP_F_VIS_Z | PCP_F_VIS_M))) cr = 1, cg = 0, cb = 0;  // red
            arr.markers.push_back(marker(stamp, "excavation_grid_3d", (int)i, Marker::CUBE,
                                         xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], s, s, s, cr,
                                         cg, cb, 0.5f, 15.0));
        }
        grid_visualization_pub_->publish(arr);
    }

    std::unique_ptr<pcp::MultiDevice> multi_;
    pcp::Device *dev_ = nullptr;
    std::unique_ptr<pcp::SimplifiedDualLidarOptimizer> core_;
    bool terrain_cloud_ = false;
    std::shared_ptr<tf2_ros::Buffer> tf_buffer_;
    std::shared_ptr<tf2_ros::TransformListener> tf_listener_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr excavation_area_sub_,
        terrain_sub_, zx120_points_sub_;
    rclcpp::Publisher<geometry_msgs::msg::PointStamped>::SharedPtr optimal_position_pub_;
    rclcpp::Publisher<visualization_msgs::msg::MarkerArray>::SharedPtr candidate_positions_pub_,
        grid_visualization_pub_;
    rclcpp::TimerBase::SharedPtr optimization_timer_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<SimplifiedDualLidarOptimizerNode>());
    rclcpp::shutdown();
    return 0;
}
