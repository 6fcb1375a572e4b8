// Stand-in for the slice of the ROS 2 Humble API the node shells in ros/src use (rclcpp,
// message structs, tf2_ros).  Test infrastructure only, nothing here ships:
//  * tests/test_ros_shells.py compiles and links every shell against it, so a renamed core
//    method, a wrong message field or a bad log format fails without a ROS install;
//  * it is also a minimal in-process bus: subscriptions, publishers, wall timers, parameters
//    and a static TF table are real, so a driver (tests/ros_stub/shell_driver.cpp) can deliver
//    messages to a shell's callbacks, fire its timers and count what each topic published.
#pragma once

#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <typeinfo>
#include <utility>
#include <vector>

namespace builtin_interfaces::msg {
struct Time { int32_t sec = 0; uint32_t nanosec = 0; };
}  // namespace builtin_interfaces::msg

namespace std_msgs::msg {
struct Header { builtin_interfaces::msg::Time stamp; std::string frame_id; };
}  // namespace std_msgs::msg

namespace sensor_msgs::msg {
struct PointField {
    enum : uint8_t { INT8 = 1, UINT8, INT16, UINT16, INT32, UINT32, FLOAT32, FLOAT64 };
    std::string name; uint32_t offset = 0; uint8_t datatype = 0; uint32_t count = 0;
};
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

// ---- the in-process bus behind the stand-in (what a driver inspects) ------------------------
namespace ros_stub {
struct Bus {
    // topic -> deliverers (one per subscription), each checking the message type it was given
    std::map<std::string, std::vector<std::pair<const std::type_info *, std::function<void(const void *)>>>> subs;
    std::map<std::string, std::shared_ptr<void>> pubs;    // topic -> rclcpp::Publisher<M>
    std::map<std::string, const std::type_info *> pub_types;
    std::vector<std::function<void()>> timers;
    std::map<std::pair<std::string, std::string>, geometry_msgs::msg::TransformStamped> tf;
    std::vector<std::string> log;                          // "LEVEL text", in call order
    int64_t clock_ns = 0;                                  // now(): advanced by the driver
};
inline Bus &bus() {
    static Bus b;
    return b;
}
inline void logf(const char *lvl, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
inline void logf(const char *lvl, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    bus().log.push_back(std::string(lvl) + " " + buf);
}
}  // namespace ros_stub

namespace rclcpp {
class Time {
   public:
    Time() = default;
    explicit Time(int64_t ns) : ns_(ns) {}
    operator builtin_interfaces::msg::Time() const {
        return {(int32_t)(ns_ / 1000000000), (uint32_t)(ns_ % 1000000000)};
    }
    int64_t nanoseconds() const { return ns_; }

   private:
    int64_t ns_ = 0;
};
class Duration {
   public:
    static builtin_interfaces::msg::Time from_seconds(double s) {
        return {(int32_t)s, (uint32_t)((s - (int32_t)s) * 1e9)};
    }
};
class Clock {};
struct Logger {};
class ParameterValue {
   public:
    enum Kind { NONE, DOUBLE, INT, BOOL };
    ParameterValue() = default;
    explicit ParameterValue(double v) : k_(DOUBLE), d_(v) {}
    explicit ParameterValue(int64_t v) : k_(INT), i_(v) {}
    explicit ParameterValue(bool v) : k_(BOOL), b_(v) {}
    // rclcpp throws InvalidParameterTypeException on a type mismatch; so does the stand-in
    double as_double() const { return k_ == DOUBLE ? d_ : throw std::runtime_error("not a double"); }
    int64_t as_int() const { return k_ == INT ? i_ : throw std::runtime_error("not an integer"); }
    bool as_bool() const { return k_ == BOOL ? b_ : throw std::runtime_error("not a bool"); }

   private:
    Kind k_ = NONE;
    double d_ = 0;
    int64_t i_ = 0;
    bool b_ = false;
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
    explicit Publisher(std::string topic) : topic_(std::move(topic)) {}
    void publish(const M &m) {
        ++count_;
        last_ = m;
    }
    size_t count() const { return count_; }
    const M &last() const { return last_; }
    const std::string &topic() const { return topic_; }

   private:
    std::string topic_;
    size_t count_ = 0;
    M last_{};
};
class TimerBase {
   public:
    using SharedPtr = std::shared_ptr<TimerBase>;
};
class Node : public std::enable_shared_from_this<Node> {
   public:
    explicit Node(const std::string &name) : name_(name) {}
    virtual ~Node() = default;
    template <class M, class F>
    typename Subscription<M>::SharedPtr create_subscription(const std::string &topic, int, F &&f) {
        std::function<void(std::shared_ptr<M>)> cb(std::forward<F>(f));
        ros_stub::bus().subs[topic].push_back(
            {&typeid(M), [cb](const void *p) { cb(std::make_shared<M>(*static_cast<const M *>(p))); }});
        return std::make_shared<Subscription<M>>();
    }
    template <class M>
    typename Publisher<M>::SharedPtr create_publisher(const std::string &topic, int) {
        auto p = std::make_shared<Publisher<M>>(topic);
        ros_stub::bus().pubs[topic] = p;
        ros_stub::bus().pub_types[topic] = &typeid(M);
        return p;
    }
    template <class Rep, class Period, class F>
    TimerBase::SharedPtr create_wall_timer(std::chrono::duration<Rep, Period>, F &&f) {
        ros_stub::bus().timers.push_back(std::function<void()>(std::forward<F>(f)));
        return std::make_shared<TimerBase>();
    }
    void declare_parameter(const std::string &n, double v) { params_[n] = ParameterValue(v); }
    void declare_parameter(const std::string &n, int v) { params_[n] = ParameterValue((int64_t)v); }
    void declare_parameter(const std::string &n, int64_t v) { params_[n] = ParameterValue(v); }
    void declare_parameter(const std::string &n, bool v) { params_[n] = ParameterValue(v); }
    ParameterValue get_parameter(const std::string &n) const {
        auto it = params_.find(n);
        if (it == params_.end()) throw std::runtime_error("parameter not declared: " + n);
        return it->second;
    }
    Logger get_logger() const { return {}; }
    std::shared_ptr<Clock> get_clock() const { return std::make_shared<Clock>(); }
    Time now() const { return Time(ros_stub::bus().clock_ns); }
    const std::string &get_name() const { return name_; }

   private:
    std::string name_;
    std::map<std::string, ParameterValue> params_;
};
inline void init(int, char **) {}
inline void shutdown() {}
inline void spin(const std::shared_ptr<Node> &) {}
}  // namespace rclcpp

#define RCLCPP_INFO(logger, ...) ((void)(logger), ros_stub::logf("INFO", __VA_ARGS__))
#define RCLCPP_WARN(logger, ...) ((void)(logger), ros_stub::logf("WARN", __VA_ARGS__))
#define RCLCPP_ERROR(logger, ...) ((void)(logger), ros_stub::logf("ERROR", __VA_ARGS__))
#define RCLCPP_DEBUG(logger, ...) ((void)(logger), ros_stub::logf("DEBUG", __VA_ARGS__))
#define RCLCPP_WARN_THROTTLE(logger, clock, ms, ...) \
    ((void)(logger), (void)(clock), (void)(ms), ros_stub::logf("WARN", __VA_ARGS__))

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
    // the static table of the bus (ros_stub::set_transform); absent -> throws as tf2 does
    geometry_msgs::msg::TransformStamped lookupTransform(const std::string &target,
                                                         const std::string &source,
                                                         const tf2::TimePoint &,
                                                         const tf2::Duration &) const {
        auto it = ros_stub::bus().tf.find({target, source});
        if (it == ros_stub::bus().tf.end())
            throw tf2::TransformException("\"" + source + "\" passed to lookupTransform argument "
                                          "source_frame does not exist.");
        return it->second;
    }
};
class TransformListener {
   public:
    explicit TransformListener(Buffer &) {}
};
}  // namespace tf2_ros

// ---- driver side ----------------------------------------------------------------------------
namespace ros_stub {
// hand a message to every subscription of the topic (as the executor would, in order)
template <class M>
size_t deliver(const std::string &topic, const M &m) {
    auto it = bus().subs.find(topic);
    if (it == bus().subs.end()) return 0;
    size_t n = 0;
    for (auto &s : it->second) {
        if (*s.first != typeid(M)) throw std::runtime_error("wrong message type for " + topic);
        s.second(&m);
        ++n;
    }
    return n;
}
template <class M>
const rclcpp::Publisher<M> *publisher(const std::string &topic) {
    auto it = bus().pubs.find(topic);
    if (it == bus().pubs.end()) return nullptr;
    if (*bus().pub_types[topic] != typeid(M)) throw std::runtime_error("wrong type for " + topic);
    return static_cast<const rclcpp::Publisher<M> *>(it->second.get());
}
inline void fire_timers() {
    for (auto &t : bus().timers) t();
}
inline void set_transform(const std::string &target, const std::string &source, const double t[3],
                          const double q[4]) {
    geometry_msgs::msg::TransformStamped s;
    s.header.frame_id = target;
    s.child_frame_id = source;
    s.transform.translation.x = t[0];
    s.transform.translation.y = t[1];
    s.transform.translation.z = t[2];
    s.transform.rotation.x = q[0];
    s.transform.rotation.y = q[1];
    s.transform.rotation.z = q[2];
    s.transform.rotation.w = q[3];
    bus().tf[{target, source}] = s;
}
}  // namespace ros_stub
