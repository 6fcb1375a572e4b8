// calc_drivable_area: the rclcpp shell of calc_drivable_area.cpp (its class is also called
// SimplifiedScanMatcher upstream) -- node name, parameters (read once, :21-37), topics, TF
// lookups and log lines of :18-138, :169-231.  doTransform, binning, gradients and the start
// clearing run in libpcp (pcp_drivable_area via pcp::DrivableAreaMapper).
#include "pcp_ros.hpp"

#include <nav_msgs/msg/occupancy_grid.hpp>

class DrivableAreaNode : public rclcpp::Node {
   public:
    DrivableAreaNode() : Node("simplified_scan_matcher") {
        declare_parameter("grid_resolution", 1.0);
        declare_parameter("map_width", 100.0);
        declare_parameter("map_height", 100.0);
        declare_parameter("max_gradient", 0.3);
        declare_parameter("min_points_per_cell", 10);
        declare_parameter("start_clear_radius", 3.0);
        pcp_drivable_params p;
        p.grid_resolution = get_parameter("grid_resolution").as_double();
        p.map_width = get_parameter("map_width").as_double();
        p.map_height = get_parameter("map_height").as_double();
        p.max_gradient = get_parameter("max_gradient").as_double();
        p.min_points_per_cell = (int32_t)get_parameter("min_points_per_cell").as_int();
        p.start_clear_radius = get_parameter("start_clear_radius").as_double();
        core_ = std::make_unique<pcp::DrivableAreaMapper>(pcp_ros::device(), p);

        tf_buffer_ = std::make_shared<tf2_ros::Buffer>(get_clock());
        tf_listener_ = std::make_shared<tf2_ros::TransformListener>(*tf_buffer_);
        robot_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/four_wheel_robot/filtered_points", 1,
            [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { robotCloudCallback(*m); });
        occupancy_grid_pub_ = create_publisher<nav_msgs::msg::OccupancyGrid>("/occupancy_grid", 10);
        RCLCPP_INFO(get_logger(), "Occupancy Grid Map Generator initialized");
        RCLCPP_INFO(get_logger(), "Grid size: %d x %d, Resolution: %.2f m",
                    (int)(p.map_width / p.grid_resolution), (int)(p.map_height / p.grid_resolution),
                    p.grid_resolution);
        RCLCPP_INFO(get_logger(), "Start clear radius: %.2f m", p.start_clear_radius);
    }

   private:
    void robotCloudCallback(const sensor_msgs::msg::PointCloud2 &msg) {
        pcp::Transform cloud_to_map, robot;
        std::string why;
        // canTransform + lookupTransform with 0.5 s (:77-101)
        if (!pcp_ros::lookup(*tf_buffer_, "map", msg.header.frame_id, 0.5, cloud_to_map, &why)) {
            RCLCPP_WARN_THROTTLE(get_logger(), *get_clock(), 1000,
                                 "Transform from %s to %s not available yet",
                                 msg.header.frame_id.c_str(), "map");
            return;
        }
        if (msg.width * msg.height == 0) {
            RCLCPP_WARN(get_logger(), "Received empty point cloud");
            return;
        }
        if (!pcp_ros::lookup(*tf_buffer_, "map", "four_wheel_robot/base_link", 0.1, robot, &why)) {
            RCLCPP_WARN_THROTTLE(get_logger(), *get_clock(), 1000, "Could not get robot transform: %s",
                                 why.c_str());
            return;
        }
        const bool had_start = core_->startSet();
        pcp::OccupancyGrid g;
        if (!core_->robotCloudCallback(pcp_ros::from_ros(msg), &cloud_to_map, &robot, g)) {
            if (!core_->lastError().empty())
                RCLCPP_ERROR(get_logger(), "%s", core_->lastError().c_str());
            return;
        }
        if (!had_start)
            RCLCPP_INFO(get_logger(), "Start position set at (%.2f, %.2f)", robot.t[0], robot.t[1]);
        nav_msgs::msg::OccupancyGrid m;   // :169-178
        m.header.stamp = now();
        m.header.frame_id = g.frame_id;
        m.info.resolution = (float)g.resolution;
        m.info.width = g.width;
        m.info.height = g.height;
        m.info.origin.position.x = g.origin_x;
        m.info.origin.position.y = g.origin_y;
        m.info.origin.position.z = 0.0;
        m.info.origin.orientation.w = 1.0;
        m.data = std::move(g.data);
        occupancy_grid_pub_->publish(m);
        RCLCPP_DEBUG(get_logger(), "Published occupancy grid at (%.2f, %.2f) with %u points",
                     robot.t[0], robot.t[1], msg.width * msg.height);
    }

    std::unique_ptr<pcp::DrivableAreaMapper> core_;
    std::shared_ptr<tf2_ros::Buffer> tf_buffer_;
    std::shared_ptr<tf2_ros::TransformListener> tf_listener_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr robot_cloud_sub_;
    rclcpp::Publisher<nav_msgs::msg::OccupancyGrid>::SharedPtr occupancy_grid_pub_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<DrivableAreaNode>());
    rclcpp::shutdown();
    return 0;
}
