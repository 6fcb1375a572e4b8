// pointcloud_filter: the rclcpp shell of pointcloud_filter.cpp (SimplifiedScanMatcher) --
// node name, topics, QoS depth 1, parameters and log lines of :11-62; cropFrontArea +
// VoxelGrid run in libpcp (pcp::SimplifiedScanMatcher -> pcp_crop_voxel).
#include "pcp_ros.hpp"

class SimplifiedScanMatcherNode : public rclcpp::Node {
   public:
    SimplifiedScanMatcherNode() : Node("simplified_scan_matcher"), core_(pcp_ros::device()) {
        robot_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/four_wheel_robot/velodyne_points", 1,
            [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { onCloud(*m, true); });
        backhoe_cloud_sub_ = create_subscription<sensor_msgs::msg::PointCloud2>(
            "/zx120/velodyne_points", 1,
            [this](sensor_msgs::msg::PointCloud2::SharedPtr m) { onCloud(*m, false); });
        robot_filtered_pub_ =
            create_publisher<sensor_msgs::msg::PointCloud2>("/four_wheel_robot/filtered_points", 1);
        backhoe_filtered_pub_ =
            create_publisher<sensor_msgs::msg::PointCloud2>("/zx120/filtered_points", 1);
        declare_parameter("robot_front_range", 15.0);
        declare_parameter("robot_side_range", 10.0);
        declare_parameter("robot_height_range", 10.0);
        declare_parameter("backhoe_front_range", 15.0);
        declare_parameter("backhoe_side_range", 10.0);
        declare_parameter("backhoe_height_range", 10.0);
        declare_parameter("voxel_leaf_size", 0.2);
        RCLCPP_INFO(get_logger(), "Simplified Scan Matcher initialized");
        RCLCPP_INFO(get_logger(), "Function: Front area cropping and downsampling only");
    }

   private:
    void onCloud(const sensor_msgs::msg::PointCloud2 &msg, bool robot) {
        // parameters are read at every message, as processCloudSimple does (:94-101, :132)
        auto &p = core_.params();
        p.robot_front_range = get_parameter("robot_front_range").as_double();
        p.robot_side_range = get_parameter("robot_side_range").as_double();
        p.robot_height_range = get_parameter("robot_height_range").as_double();
        p.backhoe_front_range = get_parameter("backhoe_front_range").as_double();
        p.backhoe_side_range = get_parameter("backhoe_side_range").as_double();
        p.backhoe_height_range = get_parameter("backhoe_height_range").as_double();
        p.voxel_leaf_size = get_parameter("voxel_leaf_size").as_double();
        const pcp::PointCloud2 in = pcp_ros::from_ros(msg);
        pcp::PointCloud2 out =
            robot ? core_.robotCloudCallback(in) : core_.backhoeCloudCallback(in);
        if (!core_.lastError().empty()) {
            RCLCPP_ERROR(get_logger(), "%s", core_.lastError().c_str());
            return;
        }
        RCLCPP_DEBUG(get_logger(), "%s cloud: %zu -> %zu -> %zu points",
                     robot ? "robot" : "backhoe", in.size(), core_.lastCroppedSize(), out.size());
        // output_msg->header = input_msg->header (:79)
        (robot ? robot_filtered_pub_ : backhoe_filtered_pub_)
            ->publish(pcp_ros::to_ros(std::move(out), msg.header.stamp));
    }

    pcp::SimplifiedScanMatcher core_;
    rclcpp::Subscription<sensor_msgs::msg::PointCloud2>::SharedPtr robot_cloud_sub_,
        backhoe_cloud_sub_;
    rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr robot_filtered_pub_,
        backhoe_filtered_pub_;
};

int main(int argc, char **argv) {
    rclcpp::init(argc, argv);
    auto node = std::make_shared<SimplifiedScanMatcherNode>();
    rclcpp::spin(node);
    rclcpp::shutdown();
    return 0;
}
