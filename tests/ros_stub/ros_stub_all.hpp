// Type-level stand-in for the slice of the ROS 2 Humble API the node shells in ros/src use
// (rclcpp, message structs, tf2_ros).  Test infrastructure only: tests/test_ros_shells.py
// compiles the shells against it (g++ -fsyntax-only) so a renamed core method or a wrong
// message field is caught without a ROS install.  Nothing here runs or ships.
#pragma once

#include <chrono>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace builtin_interfaces::msg {
struct Time { int32_t sec = 0; uint32_t nanosec = 0; };
}  // namespace builtin_interfaces::msg

namespace std_msgs::msg {
struct Header { builtin_interfaces::msg::Time stamp; std::string frame_id; };
}  // namespace std_msgs::msg

namespace sensor_msgs::msg {
struct PointField { std::string name; uint32_t offset = 0; uint8_t datatype = 0; uint32_t count = 0; };
struct PointCloud2 {
    using SharedPtr = std::shared_ptr<PointCloud2>;
    std_msgs::msg::Header header;
    uint32_t height = 0, width = 0;
    std::vector<PointField> fields;
    bool is_bigendian = false;
    uint32_t point_step = 0, row_step = 0;
    std::vector<uint8_t> data;
    bool is_dense = false;
};
struct NavSatStatus { int8_t status = 0; };
struct NavSatFix {
    using SharedPtr = std::shared_ptr<NavSatFix>;
    std_msgs::msg::Header header;
    NavSatStatus status;
    double latitude = 0, longitude = 0, altitude = 0;
};
}  // namespace sensor_msgs::msg

namespace geometry_msgs::msg {
struct Vector3 { double x = 0, y = 0, z = 0; };
struct Point { double x = 0, y = 0, z = 0; };
struct Quaternion { double x = 0, y = 0, z = 0, w = 1; };
struct Pose { Point position; Quaternion orientation; };
struct Transform { Vector3 translation; Quaternion rotation; };
struct TransformStamped { std_msgs::msg::Header header; std::string child_frame_id; Transform transform; };
struct PointStamped { std_msgs::msg::Header header; Point point; };
struct QuaternionStamped { std_msgs::msg::Header header; Quaternion quaternion; };
}  // namespace geometry_msgs::msg

namespace nav_msgs::msg {
struct MapMetaData {
    float resolution = 0;
    uint32_t width = 0, height = 0;
    geometry_msgs::msg::Pose origin;
};
struct OccupancyGrid { std_msgs::msg::Header header; MapMetaData info; std::vector<int8_t> data; };
}  // namespace nav_msgs::msg

namespace rclcpp {
class Time {
   public:
    operator builtin_interfaces::msg::Time() const { return {}; }
};
class Duration {
   public:
    static builtin_interfaces::msg::Time from_seconds(double) { return {}; }
};
class Clock {};
struct Logger {};
class ParameterValue {
   public:
    double as_double() const { return 0; }
    bool as_bool() const { return false; }
    int64_t as_int() const { return 0; }
};
template <class M>
class Subscription {
   public:
    using SharedPtr = std::shared_ptr<Subscription>;
};
template <class M>
class Publisher {
   public:
    using SharedPtr = std::shared_ptr<Publisher>;
    void publish(const M &) {}
};
class TimerBase {
   public:
    using SharedPtr = std::shared_ptr<TimerBase>;
};
class Node : public std::enable_shared_from_this<Node> {
   public:
    explicit Node(const std::string &) {}
    virtual ~Node() = default;
    template <class M, class F>
    typename Subscription<M>::SharedPtr create_subscription(const std::string &, int, F &&f) {
        (void)[&] { f(std::make_shared<M>()); };
        return nullptr;
    }
    template <class M>
    typename Publisher<M>::SharedPtr create_publisher(const std::string &, int) { return nullptr; }
    template <class Rep, class Period, class F>
    TimerBase::SharedPtr create_wall_timer(std::chrono::duration<Rep, Period>, F &&f) {
        (void)[&] { f(); };
        return nullptr;
    }
    template <class T>
    void declare_parameter(const std::string &, const T &) {}
    ParameterValue get_parameter(const std::string &) const { return {}; }
    Logger get_logger() const { return {}; }
    std::shared_ptr<Clock> get_clock() const { return std::make_shared<Clock>(); }
    Time now() const { return {}; }
};
inline void init(int, char **) {}
inline void shutdown() {}
inline void spin(const std::shared_ptr<Node> &) {}
}  // namespace rclcpp

#define PCP_STUB_LOG(...) ((void)sizeof(printf(__VA_ARGS__)))
#include <cstdio>
#define RCLCPP_INFO(logger, ...) ((void)(logger), PCP_STUB_LOG(__VA_ARGS__))
#define RCLCPP_WARN(logger, ...) ((void)(logger), PCP_STUB_LOG(__VA_ARGS__))
#define RCLCPP_ERROR(logger, ...) ((void)(logger), PCP_STUB_LOG(__VA_ARGS__))
#define RCLCPP_DEBUG(logger, ...) ((void)(logger), PCP_STUB_LOG(__VA_ARGS__))
#define RCLCPP_WARN_THROTTLE(logger, clock, ms, ...) \
    ((void)(logger), (void)(clock), (void)(ms), PCP_STUB_LOG(__VA_ARGS__))

namespace visualization_msgs::msg {
struct ColorRGBA { float r = 0, g = 0, b = 0, a = 0; };
struct Marker {
    enum : int32_t { CUBE = 1, SPHERE = 2, CYLINDER = 3 };
    enum : int32_t { ADD = 0, DELETEALL = 3 };
    std_msgs::msg::Header header;
    std::string ns;
    int32_t id = 0, type = 0, action = 0;
    geometry_msgs::msg::Pose pose;
    geometry_msgs::msg::Vector3 scale;
    ColorRGBA color;
    builtin_interfaces::msg::Time lifetime;
};
struct MarkerArray { std::vector<Marker> markers; };
}  // namespace visualization_msgs::msg

namespace tf2 {
struct TimePoint {};
inline const TimePoint TimePointZero{};
struct Duration {};
inline Duration durationFromSec(double) { return {}; }
class TransformException : public std::runtime_error {
   public:
    using std::runtime_error::runtime_error;
};
}  // namespace tf2

namespace tf2_ros {
class Buffer {
   public:
    explicit Buffer(std::shared_ptr<rclcpp::Clock>) {}
    geometry_msgs::msg::TransformStamped lookupTransform(const std::string &, const std::string &,
                                                         const tf2::TimePoint &,
                                                         const tf2::Duration &) const {
        throw tf2::TransformException("stub");
    }
};
class TransformListener {
   public:
    explicit TransformListener(Buffer &) {}
};
}  // namespace tf2_ros
