// pcp_ros.hpp -- the thin layer between rclcpp messages and the node cores (pcp_nodes.hpp):
// PointCloud2 <-> pcp::PointCloud2 (the data blob is copied once, read in place by libpcp),
// TF lookups with the reference's frames and timeouts (log and skip on failure), and the one
// HIP device context a process shares.  Only built with PCP_WITH_ROS (ros/CMakeLists.txt).
#pragma once

#include <cstdlib>
#include <memory>
#include <string>

#include <geometry_msgs/msg/transform_stamped.hpp>
#include <rclcpp/rclcpp.hpp>
#include <sensor_msgs/msg/point_cloud2.hpp>
#include <tf2/exceptions.h>
#include <tf2_ros/buffer.h>
#include <tf2_ros/transform_listener.h>

#include "pcp_nodes.hpp"

namespace pcp_ros {

inline pcp::PointCloud2 from_ros(const sensor_msgs::msg::PointCloud2 &m) {
    pcp::PointCloud2 c;
    c.frame_id = m.header.frame_id;
    c.stamp = (double)m.header.stamp.sec + 1e-9 * (double)m.header.stamp.nanosec;
    c.height = m.height;
    c.width = m.width;
    c.fields.reserve(m.fields.size());
    for (const auto &f : m.fields) {
        pcp::PointField pf;
        pf.name = f.name;
        pf.offset = f.offset;
        pf.datatype = f.datatype;
        pf.count = f.count;
        c.fields.push_back(pf);
    }
    c.is_bigendian = m.is_bigendian;
    c.point_step = m.point_step;
    c.row_step = m.row_step;
    c.data = m.data;
    c.is_dense = m.is_dense;
    return c;
}

// the output header: the caller's stamp (the input's, or now() where the reference restamps)
inline sensor_msgs::msg::PointCloud2 to_ros(pcp::PointCloud2 &&c,
                                            const builtin_interfaces::msg::Time &stamp) {
    sensor_msgs::msg::PointCloud2 m;
    m.header.frame_id = c.frame_id;
    m.header.stamp = stamp;
    m.height = c.height;
    m.width = c.width;
    for (const auto &f : c.fields) {
        sensor_msgs::msg::PointField pf;
        pf.name = f.name;
        pf.offset = f.offset;
        pf.datatype = f.datatype;
        pf.count = f.count;
        m.fields.push_back(pf);
    }
    m.is_bigendian = c.is_bigendian;
    m.point_step = c.point_step;
    m.row_step = c.row_step;
    m.data = std::move(c.data);
    m.is_dense = c.is_dense;
    return m;
}

// tf_buffer_->lookupTransform(target, source, TimePointZero, timeout); false with *why set when
// it throws -- each node logs that its own way (plain, throttled) and skips, as upstream does
inline bool lookup(tf2_ros::Buffer &buf, const std::string &target, const std::string &source,
                   double timeout_s, pcp::Transform &out, std::string *why) {
    try {
        const geometry_msgs::msg::TransformStamped t = buf.lookupTransform(
            target, source, tf2::TimePointZero, tf2::durationFromSec(timeout_s));
        out.t[0] = t.transform.translation.x;
        out.t[1] = t.transform.translation.y;
        out.t[2] = t.transform.translation.z;
        out.q[0] = t.transform.rotation.x;
        out.q[1] = t.transform.rotation.y;
        out.q[2] = t.transform.rotation.z;
        out.q[3] = t.transform.rotation.w;
        return true;
    } catch (const tf2::TransformException &ex) {
        if (why) *why = ex.what();
        return false;
    }
}

// pcl::toROSMsg of an empty cloud is never published by the reference nodes
inline bool publish_nonempty(
    const rclcpp::Publisher<sensor_msgs::msg::PointCloud2>::SharedPtr &pub, pcp::PointCloud2 &&c,
    const builtin_interfaces::msg::Time &stamp) {
    if (c.empty()) return false;
    pub->publish(to_ros(std::move(c), stamp));
    return true;
}

// one libpcp context (one GPU) per process; PCP_DEVICE selects it
inline pcp::Device &device() {
    static pcp::Device dev(std::getenv("PCP_DEVICE") ? std::atoi(std::getenv("PCP_DEVICE")) : 0);
    return dev;
}

}  // namespace pcp_ros
