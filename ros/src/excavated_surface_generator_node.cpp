// excavated_surface_generator: the rclcpp shell of excavated_surface_generator.cpp
// (ExcavationTerrainGenerator) -- node name, excavation.* parameters, the 1 s parameter timer,
// topics and the marker array of :21-136 and :263-325, :586-629.  getTerrainHeight,
// processExcavation, generateExcavatedSurface and generateExcavationArea run in libpcp
// (pcp_excavate); the markers are host-side arithmetic on the centre/yaw it returns.
#include "pcp_ros.hpp"

#include <cmath>
#include <visualization_msgs/msg/marker_array.hpp>

using namespace std::chrono_literals;

class ExcavationTerrainGeneratorNode : public rclcpp::Node {
   public:
    ExcavationTerrainGeneratorNode()
        : Node("excavation_terrain_generator"), core_(pcp_ros::device()) {
        const pcp::ExcavationTerrainGenerator::Params d;   // :28-47 defaults
        declare_parameter("excavation.depth", d.depth);
        declare_parameter("excavation.slope_angle", d.slope_angle_deg);
        declare_parameter("excavation.offset_x", d.offset_x);
        declare_parameter("excavation.offset_y", d.offset_y);
        declare_parameter("excavation.point_density", d.point_density);
        declare_parameter("excavation.enabled", d.enabled);
        declare_parameter("excavation.terrain_search_radius", d.terrain_search_radius);
        declare_parameter("excavation.l_shape_enabled", d.l_shape_enabled != 0);
        declare_parameter("excavation.arm1_length", d.arm1_length);
        declare_parameter("excavation.arm1_width", d.arm1_width);
        declare_parameter("excavation.arm2_length", d.arm2_length);
        declare_parameter("excavation.arm2_width", d.arm2_width);
        declare_parameter("excavation.width", d.width);
        declare_parameter("excavation.length", d.length);
        updateParameters();

        tf_buffer_ = std::make_shared<tf2_ros::Buffer>(get_clock());
        tf_listener_ = std::make_shared<tf2_ros::TransformListener>(*tf_buffer_);
        matched_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/matched_point_cloud", 10,
            [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { matchedCloudCallback(m); });
        excavated_terrain_pub_ =
            create_publisher<sensor_msgs::msg::PointCloud2>("/excavated_terrain", 10);
        excavation_area_pub_ = create_publisher<sensor_msgs::msg::PointCloud2>("/excavation_area", 10);
        excavation_marker_pub_ =
            create_publisher<visualization_msgs::msg::MarkerArray>("/excavation_markers", 10);
        param_timer_ = create_wall_timer(1s, [this] { updateParameters(); });

        const auto &p = core_.params();
        RCLCPP_INFO(get_logger(), "Excavation Terrain Generator initialized");
        if (p.l_shape_enabled)
            RCLCPP_INFO(get_logger(),
                        "L-Shape Mode - Arm1: %.2fm x %.2fm, Arm2: %.2fm x %.2fm, Depth: %.2fm",
                        p.arm1_length, p.arm1_width, p.arm2_length, p.arm2_width, p.depth);
        else
            RCLCPP_INFO(get_logger(), "Rectangle Mode - Length: %.2fm, Width: %.2fm, Depth: %.2fm",
                        p.length, p.width, p.depth);
    }

   private:
    void updateParameters() {   // :118-136
        auto &p = core_.params();
        p.depth = get_parameter("excavation.depth").as_double();
        p.slope_angle_deg = get_parameter("excavation.slope_angle").as_double();
        p.offset_x = get_parameter("excavation.offset_x").as_double();
        p.offset_y = get_parameter("excavation.offset_y").as_double();
        p.point_density = get_parameter("excavation.point_density").as_double();
        p.enabled = get_parameter("excavation.enabled").as_bool();
        p.terrain_search_radius = get_parameter("excavation.terrain_search_radius").as_double();
        p.l_shape_enabled = get_parameter("excavation.l_shape_enabled").as_bool() ? 1 : 0;
        p.arm1_length = get_parameter("excavation.arm1_length").as_double();
        p.arm1_width = get_parameter("excavation.arm1_width").as_double();
        p.arm2_length = get_parameter("excavation.arm2_length").as_double();
        p.arm2_width = get_parameter("excavation.arm2_width").as_double();
        p.width = get_parameter("excavation.width").as_double();
        p.length = get_parameter("excavation.length").as_double();
    }

    void matchedCloudCallback(const sensor_msgs::msg::PointCloud2::SharedPtr &msg) {
        pcp::Transform zx120;
        bool have = false;
        if (core_.params().enabled) {
            std::string why;
            have = pcp_ros::lookup(*tf_buffer_, "map", "zx120/base_link", 0.1, zx120, &why);
            if (!have)
                RCLCPP_WARN_THROTTLE(get_logger(), *get_clock(), 1000,
                                     "Could not get zx120 transform: %s", why.c_str());
        }
        if (!have) {   // disabled or no TF: the input goes out unchanged (:264-266, :277)
            excavated_terrain_pub_->publish(*msg);
            return;
        }
        pcp::ExcavationTerrainGenerator::Output o =
            core_.matchedCloudCallback(pcp_ros::from_ros(*msg), &zx120);
        if (!o.area_published) {   // the library refused the cloud: logged, input republished
            RCLCPP_ERROR(get_logger(), "%s", core_.lastError().c_str());
            excavated_terrain_pub_->publish(*msg);
            return;
        }
        // header = msg->header, frame_id = "map" (:314-322)
        excavated_terrain_pub_->publish(pcp_ros::to_ros(std::move(o.excavated_terrain), msg->header.stamp));
        excavation_area_pub_->publish(pcp_ros::to_ros(std::move(o.excavation_area), msg->header.stamp));
        publishExcavationMarkers(o.center, o.yaw, msg->header.stamp);
    }

    // getExcavationBoxes (:138-181): centre (x, y) in the excavation frame, extent along x, y
    struct Box { double cx, cy, lx, ly; };
    std::vector<Box> boxes() const {
        const auto &p = core_.params();
        if (!p.l_shape_enabled) return {{0.0, 0.0, p.length, p.width}};
        return {{0.0, -p.arm1_length / 2.0, p.arm1_width, p.arm1_length},
                {p.arm2_length / 2.0, -p.arm1_length + p.arm2_width / 2.0, p.arm2_length,
                 p.arm2_width}};
    }

    void publishExcavationMarkers(const double c[3], double yaw,
                                  const builtin_interfaces::msg::Time &stamp) {   // :586-629
        const double depth = core_.params().depth;
        visualization_msgs::msg::MarkerArray arr;
        int id = 0;
        for (const Box &b : boxes()) {
            visualization_msgs::msg::Marker m;
            m.header.frame_id = "map";
            m.header.stamp = stamp;
            m.ns = "excavation";
            m.id = id++;
            m.type = visualization_msgs::msg::Marker::CUBE;
            m.action = visualization_msgs::msg::Marker::ADD;
            m.pose.position.x = c[0] + b.cx * std::cos(yaw) - b.cy * std::sin(yaw);
            m.pose.position.y = c[1] + b.cx * std::sin(yaw) + b.cy * std::cos(yaw);
            m.pose.position.z = c[2] - depth / 2;
            m.pose.orientation.z = std::sin(yaw / 2);   // setRPY(0, 0, yaw)
            m.pose.orientation.w = std::cos(yaw / 2);
            m.scale.x = b.lx;
            m.scale.y = b.ly;
            m.scale.z = depth;
            m.color.r = 0.5f;
            m.color.g = 0.25f;
            m.color.b = 0.0f;
            m.color.a = 0.3f;
            m.lifetime = rclcpp::Duration::from_seconds(0.5);
            arr.markers.push_back(m);
        }
        excavation_marker_pub_->publish(arr);
    }

    pcp::ExcavationTerrainGenerator core_;
    std::shared_ptr<tf2_ros::Buffer> tf_buffer_;
    std::shared_ptr<tf2_ros::TransformListener> tf_listener_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr matched_cloud_sub_;
    rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr excavated_terrain_pub_,
        excavation_area_pub_;
    rclcpp::Publisher<visualization_msgs::msg::MarkerArray>::SharedPtr excavation_marker_pub_;
    rclcpp::TimerBase::SharedPtr param_timer_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<ExcavationTerrainGeneratorNode>());
    rclcpp::shutdown();
    return 0;
}
