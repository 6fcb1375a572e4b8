// pointcloud_merger: the rclcpp shell of pointcloud_merger.cpp (GnssGicpMatcher) -- node name,
// cloud topics, QoS depth 10, the 100 ms timer and the three XYZRGB outputs of :20-70 and
// :308-394.  doTransform + colouring + concatenation run in libpcp (pcp_transform_concat).
//
// The GNSS half of the reference node (NavSatFix -> LocalCartesian -> TF broadcast, :84-305)
// is outside the accelerated path: this shell only takes the origin_set_ edge
// from the first valid fix (:112, :150) and reads map <- */velodyne_link from TF, whoever
// broadcasts it (the reference's GNSS code, a localiser, a bag).
#include "pcp_ros.hpp"

#include <geometry_msgs/msg/quaternion_stamped.hpp>
#include <sensor_msgs/msg/nav_sat_fix.hpp>

using namespace std::chrono_literals;

class GnssGicpMatcherNode : public rclcpp::Node {
   public:
    GnssGicpMatcherNode() : Node("gnss_gicp_matcher"), core_(pcp_ros::device()) {
        tf_buffer_ = std::make_unique<tf2_ros::Buffer>(get_clock());
        tf_listener_ = std::make_shared<tf2_ros::TransformListener>(*tf_buffer_);
        auto on_fix = [this](sensor_msgs::msg::NavSatFix::SharedPtr m) {
            if (!origin_set_ && m->status.status >= 0) {
                origin_set_ = true;
                RCLCPP_INFO(get_logger(), "Origin set from first GNSS fix: lat=%.8f, lon=%.8f",
                            m->latitude, m->longitude);
            }
        };
        robot_gnss_sub_ = create_subscription<sensor_msgs::msg::NavSatFix>(
            "/four_wheel_robot/gnss_compass_front/fix", 10, on_fix);
        backhoe_gnss_sub_ = create_subscription<sensor_msgs::msg::NavSatFix>(
            "/zx120/gnss_compass_front/fix", 10, on_fix);
        robot_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/four_wheel_robot/filtered_points", 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) {
                core_.robotCloudCallback(pcp_ros::from_ros(*m));
                got_[0] = true;
            });
        backhoe_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/zx120/filtered_points", 10, [this](sensor_msgs::msg::PointCloud2::SharedPtr m) {
                core_.backhoeCloudCallback(pcp_ros::from_ros(*m));
                got_[1] = true;
            });
        matched_cloud_pub_ = create_publisher<sensor_msgs::msg::PointCloud2>("/matched_point_cloud", 10);
        robot_colored_cloud_pub_ =
            create_publisher<sensor_msgs::msg::PointCloud2>("/robot_colored_point_cloud", 10);
        backhoe_colored_cloud_pub_ =
            create_publisher<sensor_msgs::msg::PointCloud2>("/backhoe_colored_point_cloud", 10);
        timer_ = create_wall_timer(100ms, [this] { processPointClouds(); });
        RCLCPP_INFO(get_logger(), "GNSS GICP Matcher node initialized");
    }

   private:
    void processPointClouds() {
        if (!origin_set_) return;   // :309
        pcp::Transform tf[2];
        const char *names[2] = {"four_wheel_robot", "zx120"};
        bool ok[2];
        for (int i = 0; i < 2; ++i) {
            ok[i] = false;
            if (!got_[i]) continue;   // no cloud yet: no lookup either (:316, :322)
            std::string why;
            ok[i] = pcp_ros::lookup(*tf_buffer_, "map", std::string(names[i]) + "/velodyne_link",
                                    0.1, tf[i], &why);
            if (!ok[i])
                RCLCPP_WARN_THROTTLE(get_logger(), *get_clock(), 1000,
                                     "Could not transform point cloud for %s: %s", names[i],
                                     why.c_str());
        }
        pcp::GnssGicpMatcher::Output o =
            core_.processPointClouds(true, ok[0] ? &tf[0] : nullptr, ok[1] ? &tf[1] : nullptr);
        if (!core_.lastError().empty()) {
            RCLCPP_ERROR(get_logger(), "%s", core_.lastError().c_str());
            return;
        }
        const auto stamp = now();
        pcp_ros::publish_nonempty(matched_cloud_pub_, std::move(o.merged), stamp);
        pcp_ros::publish_nonempty(robot_colored_cloud_pub_, std::move(o.robot_colored), stamp);
        pcp_ros::publish_nonempty(backhoe_colored_cloud_pub_, std::move(o.backhoe_colored), stamp);
    }

    pcp::GnssGicpMatcher core_;
    bool origin_set_ = false;
    bool got_[2] = {false, false};   // robot_cloud_data_ / backhoe_cloud_data_ non-null
    std::unique_ptr<tf2_ros::Buffer> tf_buffer_;
    std::shared_ptr<tf2_ros::TransformListener> tf_listener_;
    rclcpp::Subscription<sensor_msgs::msg::NavSatFix>::SharedPtr robot_gnss_sub_, backhoe_gnss_sub_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr robot_cloud_sub_,
        backhoe_cloud_sub_;
    rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr matched_cloud_pub_,
        robot_colored_cloud_pub_, backhoe_colored_cloud_pub_;
    rclcpp::TimerBase::SharedPtr timer_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    rclcpp::spin(std::make_shared<GnssGicpMatcherNode>());
    rclcpp::shutdown();
    return 0;
}
