// shell_driver.cpp -- runs the virtual_lidar rclcpp shell (ros/src/virtual_lidar_node.cpp) on
// the in-process bus of the ROS stand-in (ros_stub_all.hpp).  Test infrastructure only.
//
//   shell_driver <area.bin> <terrain.bin> <zx120.bin>
//
// Each .bin holds PointXYZRGB records (32 B: x, y, z float32 at 0/4/8).  The driver plays the
// reference's message sequence on the node's own callbacks and prints one JSON object per
// step with what each output topic has published so far and the last grid MarkerArray:
//   area, empty area, area again, terrain + zx120 + TF + one 3 s timer tick.
// Linked against mock_pcp.cpp (CPU suite) or the real libpcp_nodes.so + libpcp.so (GPU).
#define main virtual_lidar_node_main
#include "virtual_lidar_node.cpp"
#undef main

#include <fstream>
#include <iostream>
#include <iterator>

namespace {

sensor_msgs::msg::PointCloud2 load_cloud(const char *path, const std::string &frame) {
    std::ifstream f(path, std::ios::binary);
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    sensor_msgs::msg::PointCloud2 m;
    m.header.frame_id = frame;
    m.height = 1;
    m.width = (uint32_t)(bytes.size() / 32);
    using PF = sensor_msgs::msg::PointField;
    m.fields = {{"x", 0, PF::FLOAT32, 1}, {"y", 4, PF::FLOAT32, 1}, {"z", 8, PF::FLOAT32, 1},
                {"rgb", 16, PF::FLOAT32, 1}};
    m.point_step = 32;
    m.row_step = 32 * m.width;
    bytes.resize((size_t)m.width * 32);
    m.data = std::move(bytes);
    m.is_dense = true;
    return m;
}

size_t count_of(const std::string &topic) {
    using visualization_msgs::msg::MarkerArray;
    if (topic == "/optimal_mobile_lidar_position") {
        const auto *p = ros_stub::publisher<geometry_msgs::msg::PointStamped>(topic);
        return p ? p->count() : 0;
    }
    const auto *p = ros_stub::publisher<MarkerArray>(topic);
    return p ? p->count() : 0;
}

void report_step(const char *step) {
    using visualization_msgs::msg::Marker;
    using visualization_msgs::msg::MarkerArray;
    std::cout << "{\"step\": \"" << step << "\"";
    for (const char *t : {"/excavation_grid_visualization", "/mobile_lidar_candidate_positions",
                          "/optimal_mobile_lidar_position"})
        std::cout << ", \"" << t << "\": " << count_of(t);
    const auto *g = ros_stub::publisher<MarkerArray>("/excavation_grid_visualization");
    if (g && g->count()) {
        const MarkerArray &a = g->last();
        int blue = 0, yellow = 0, red = 0, green = 0, cubes = 0, bad = 0;
        for (size_t i = 0; i < a.markers.size(); ++i) {
            const Marker &m = a.markers[i];
            if (i == 0) {   // the DELETEALL marker first (:911-913)
                if (m.action != Marker::DELETEALL) ++bad;
                continue;
            }
            if (m.type != Marker::CUBE || m.ns != "excavation_grid_3d" || m.id != (int)i - 1 ||
                m.header.frame_id != "map" || m.color.a != 0.5f)
                ++bad;
            ++cubes;
            if (m.color.b == 1.0f) ++blue;
            else if (m.color.r == 1.0f && m.color.g == 1.0f) ++yellow;
            else if (m.color.r == 1.0f) ++red;
            else if (m.color.g == 1.0f) ++green;
        }
        std::cout << ", \"grid\": {\"cubes\": " << cubes << ", \"blue\": " << blue
                  << ", \"yellow\": " << yellow << ", \"red\": " << red << ", \"green\": " << green
                  << ", \"malformed\": " << bad << ", \"scale\": "
                  << (a.markers.size() > 1 ? a.markers[1].scale.x : 0.0) << ", \"first_xyz\": [";
        if (a.markers.size() > 1)
            std::cout << a.markers[1].pose.position.x << ", " << a.markers[1].pose.position.y
                      << ", " << a.markers[1].pose.position.z;
        std::cout << "]}";
    }
    std::cout << "}" << std::endl;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::cerr << "usage: shell_driver area.bin terrain.bin zx120.bin\n";
        return 2;
    }
    rclcpp::init(argc, argv);
    auto node = std::make_shared<SimplifiedDualLidarOptimizerNode>();
    const sensor_msgs::msg::PointCloud2 area = load_cloud(argv[1], "map");
    sensor_msgs::msg::PointCloud2 empty = area;
    empty.width = 0;
    empty.row_step = 0;
    empty.data.clear();

    ros_stub::deliver("/excavation_area", area);
    report_step("area");
    ros_stub::deliver("/excavation_area", empty);   // :168: nothing regenerated or published
    report_step("empty_area");
    ros_stub::deliver("/excavation_area", area);
    report_step("area_again");

    ros_stub::deliver("/excavated_terrain", load_cloud(argv[2], "map"));
    ros_stub::deliver("/zx120/filtered_points", load_cloud(argv[3], "map"));
    const double t[3] = {0.0, 0.0, 0.0}, q[4] = {0.0, 0.0, 0.0, 1.0};
    ros_stub::set_transform("map", "zx120/base_link", t, q);
    ros_stub::bus().clock_ns += 3000000000LL;
    ros_stub::fire_timers();   // one optimisation tick (:80)
    report_step("tick");

    for (const std::string &line : ros_stub::bus().log) std::cerr << line << "\n";
    rclcpp::shutdown();
    return 0;
}
