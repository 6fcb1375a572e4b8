// pcp_nodes.cpp -- host-side node cores over libpcp's C ABI (see pcp_nodes.hpp).
#include "pcp_nodes.hpp"

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace pcp {

// ---- PointCloud2 helpers -------------------------------------------------------------------
// a landing buffer of at least n elements: grown when short, otherwise reused as is
template <class T>
static T *landing(std::vector<T> &v, size_t n) {
    if (v.size() < n) v.resize(n);
    return v.data();
}

static PointCloud2 make_cloud(const void *rec, size_t n, uint32_t step,
                              std::vector<PointField> fields, const std::string &frame) {
    PointCloud2 m;
    m.frame_id = frame;
    m.height = 1;
    m.width = (uint32_t)n;
    m.fields = std::move(fields);
    m.point_step = step;
    m.row_step = step * m.width;
    const uint8_t *b = static_cast<const uint8_t *>(rec);
    if (n) m.data.assign(b, b + n * step);   // one pass: no zero-fill before the copy
    m.is_dense = true;
    return m;
}

PointCloud2 make_xyz_cloud(const float *xyz16, size_t n, const std::string &frame) {
    return make_cloud(xyz16, n, 16, {{"x", 0}, {"y", 4}, {"z", 8}}, frame);
}

PointCloud2 make_xyzrgb_cloud(const void *rec32, size_t n, const std::string &frame) {
    return make_cloud(rec32, n, 32, {{"x", 0}, {"y", 4}, {"z", 8}, {"rgb", 16}}, frame);
}

bool cloud_view(const PointCloud2 &m, pcp_cloud_view &v, std::string *why) {
    int ox = -1, oy = -1, oz = -1;
    for (const auto &f : m.fields) {
        if (f.datatype != PointField::FLOAT32) continue;
        if (f.name == "x") ox = (int)f.offset;
        else if (f.name == "y") oy = (int)f.offset;
        else if (f.name == "z") oz = (int)f.offset;
    }
    if (ox < 0 || oy < 0 || oz < 0) {
        if (why) *why = "cloud has no FLOAT32 x/y/z fields";
        return false;
    }
    if (m.is_bigendian || (m.size() && m.row_step != m.width * m.point_step) ||
        m.data.size() < m.size() * m.point_step) {
        if (why) *why = "unsupported PointCloud2 layout (big endian or padded rows)";
        return false;
    }
    v.data = m.data.empty() ? nullptr : m.data.data();
    v.n = m.size();
    v.point_step = m.point_step;
    v.off_x = (uint32_t)ox;
    v.off_y = (uint32_t)oy;
    v.off_z = (uint32_t)oz;
    return true;
}

Device::Device(int device) {
    const int rc = pcp_create(device, &ctx_);
    if (rc != PCP_OK) throw std::runtime_error("pcp_create failed (no gfx950 device?)");
}

Device::~Device() {
    if (owned_) pcp_destroy(ctx_);
}

MultiDevice::MultiDevice(const std::vector<int> &devices) {
    const int rc = pcp_multi_create((int)devices.size(), devices.data(), &m_);
    if (rc != PCP_OK) throw std::runtime_error("pcp_multi_create failed");
    int rccl = 0;
    pcp_multi_info(m_, &n_, &rccl);
    rccl_ = rccl != 0;
    r0_.reset(new Device(pcp_multi_ctx(m_, 0), Device::Borrow{}));
}

MultiDevice::~MultiDevice() {
    r0_.reset();
    pcp_multi_destroy(m_);
}

// ---- pointcloud_filter -----------------------------------------------------------------------
PointCloud2 SimplifiedScanMatcher::processCloudSimple(const PointCloud2 &in,
                                                      const std::string &vehicle_type) {
    err_.clear();
    // cropFrontArea parameter selection (:93-101)
    double front, side, height;
    if (vehicle_type == "robot") {
        front = p_.robot_front_range;
        side = p_.robot_side_range;
        height = p_.robot_height_range;
    } else {
        front = p_.backhoe_front_range;
        side = p_.backhoe_side_range;
        height = p_.backhoe_height_range;
    }
    const double box[6] = {0.0, front, -side, side, -1.5, height};   // :111-113
    pcp_cloud_view v{};
    PointCloud2 out = make_xyz_cloud(nullptr, 0, in.frame_id);
    out.stamp = in.stamp;   // output_msg->header = input_msg->header (:79)
    if (!cloud_view(in, v, &err_)) return out;
    float *buf = landing(out_, 4 * (v.n ? v.n : 1));
    uint64_t n_out = 0, n_crop = 0;
    if (pcp_crop_voxel(dev_.ctx(), &v, box, (float)p_.voxel_leaf_size, buf, v.n, &n_out,
                       &n_crop) != PCP_OK) {
        err_ = dev_.error();
        return out;
    }
    last_cropped_ = n_crop;
    out = make_xyz_cloud(buf, n_out, in.frame_id);
    out.stamp = in.stamp;
    return out;
}

// ---- pointcloud_merger -----------------------------------------------------------------------
GnssGicpMatcher::Output GnssGicpMatcher::processPointClouds(bool origin_set,
                                                           const Transform *robot_tf,
                                                           const Transform *zx120_tf) {
    err_.clear();
    Output o;
    o.merged = make_xyzrgb_cloud(nullptr, 0, "map");
    o.robot_colored = o.merged;
    o.backhoe_colored = o.merged;
    if (!origin_set) return o;   // :309
    pcp_cloud_view v[2];
    pcp_rigid tf[2];
    uint8_t rgb[6];
    int k = 0, which[2];
    struct Src { const PointCloud2 *m; const Transform *t; uint8_t r, g, b; };
    const Src src[2] = {{have_robot_ ? &robot_ : nullptr, robot_tf, 255, 0, 0},       // red
                        {have_backhoe_ ? &backhoe_ : nullptr, zx120_tf, 0, 0, 255}};  // blue
    for (int i = 0; i < 2; ++i) {
        if (!src[i].m || !src[i].t) continue;   // no message yet / TF lookup failed: skip
        if (!cloud_view(*src[i].m, v[k], &err_)) continue;
        std::memcpy(tf[k].t, src[i].t->t, sizeof(tf[k].t));
        std::memcpy(tf[k].q, src[i].t->q, sizeof(tf[k].q));
        rgb[3 * k] = src[i].r;
        rgb[3 * k + 1] = src[i].g;
        rgb[3 * k + 2] = src[i].b;
        which[k++] = i;
    }
    uint64_t total = 0;
    for (int i = 0; i < k; ++i) total += v[i].n;
    uint8_t *buf = landing(out_, 32 * (total ? total : 1));
    uint64_t n = 0;
    if (k && pcp_transform_concat(dev_.ctx(), k, v, tf, rgb, buf, total, &n) != PCP_OK) {
        err_ = dev_.error();
        return o;
    }
    o.merged = make_xyzrgb_cloud(buf, n, "map");
    uint64_t base = 0;
    for (int i = 0; i < k; ++i) {
        PointCloud2 part = make_xyzrgb_cloud(buf + 32 * base, v[i].n, "map");
        (which[i] == 0 ? o.robot_colored : o.backhoe_colored) = std::move(part);
        base += v[i].n;
    }
    return o;
}

// ---- filter + merger composed ------------------------------------------------------------------
ComposedFilterMerge::Output ComposedFilterMerge::frame(const PointCloud2 &robot,
                                                       const PointCloud2 &backhoe, bool origin_set,
                                                       const Transform *robot_tf,
                                                       const Transform *zx120_tf,
                                                       bool defer_messages) {
    err_.clear();
    Output o;
    o.robot_filtered = make_xyz_cloud(nullptr, 0, robot.frame_id);
    o.robot_filtered.stamp = robot.stamp;
    o.backhoe_filtered = make_xyz_cloud(nullptr, 0, backhoe.frame_id);
    o.backhoe_filtered.stamp = backhoe.stamp;
    o.merge.merged = make_xyzrgb_cloud(nullptr, 0, "map");
    o.merge.robot_colored = o.merge.merged;
    o.merge.backhoe_colored = o.merge.merged;
    pcp_cloud_view v[2];
    if (!cloud_view(robot, v[0], &err_) || !cloud_view(backhoe, v[1], &err_)) return o;
    // cropFrontArea's boxes (:93-101, :111-113), downsampleCloud's leaf
    const double boxes[12] = {0.0, p_.robot_front_range, -p_.robot_side_range, p_.robot_side_range,
                              -1.5, p_.robot_height_range,
                              0.0, p_.backhoe_front_range, -p_.backhoe_side_range,
                              p_.backhoe_side_range, -1.5, p_.backhoe_height_range};
    // the merge's clouds: the TFs found (a missing one drops that cloud from the concatenation)
    const Transform *tfs[2] = {robot_tf, zx120_tf};
    pcp_rigid tf[2];
    uint8_t rgb[6] = {255, 0, 0, 0, 0, 255};   // red robot, blue zx120 (:376-387)
    for (int i = 0; i < 2; ++i) {
        const Transform *t = tfs[i] ? tfs[i] : tfs[1 - i];   // (placeholder: the cloud is dropped)
        if (t) {
            std::memcpy(tf[i].t, t->t, sizeof(tf[i].t));
            std::memcpy(tf[i].q, t->q, sizeof(tf[i].q));
        } else {
            tf[i] = pcp_rigid{{0, 0, 0}, {0, 0, 0, 1}};
        }
    }
    // the results read where libpcp landed them (pinned): each message is one copy
    float *none[2] = {nullptr, nullptr};
    uint64_t n = 0, per[2] = {0, 0}, crop[2] = {0, 0};
    const void *landed = nullptr;
    const float *outs[2] = {nullptr, nullptr};
    if (pcp_filter_merge_nodes(dev_.ctx(), 2, v, boxes, (float)p_.voxel_leaf_size, tf, rgb,
                               nullptr, 0, &n, per, none, crop) != PCP_OK ||
        pcp_filter_merge_landed(dev_.ctx(), 2, &landed, outs) != PCP_OK) {
        err_ = dev_.error();
        return o;
    }
    Output::Pending &q = o.pending;
    q.merged = static_cast<const uint8_t *>(landed);
    q.origin_set = origin_set;
    for (int i = 0; i < 2; ++i) {
        q.filtered[i] = outs[i];
        q.per[i] = per[i];
        q.tf[i] = tfs[i] != nullptr;
    }
    // the concatenation of the clouds whose TF was found, robot first (:316-325)
    if (origin_set) {
        uint64_t base = 0;
        const bool both = robot_tf && zx120_tf;
        for (int i = 0; i < 2; ++i) {
            if (tfs[i] && !both) {
                q.keep_off = base;
                q.keep_n = per[i];
            }
            base += per[i];
        }
        if (both) q.keep_n = n;
        if (q.keep_n)
            o.merged_landed = pcp_cloud_view{q.merged + 32 * q.keep_off, q.keep_n, 32, 0, 4, 8};
    }
    o.deferred = true;
    if (defer_messages) {   // the merged message's header (its data follows in messages())
        o.merge.merged.width = (uint32_t)q.keep_n;
        o.merge.merged.row_step = 32 * o.merge.merged.width;
        return o;
    }
    messages(o);
    return o;
}

void ComposedFilterMerge::messages(Output &o) const {
    if (!o.deferred) return;
    o.deferred = false;
    const Output::Pending &q = o.pending;
    const double rs = o.robot_filtered.stamp, bs = o.backhoe_filtered.stamp;
    o.robot_filtered = make_xyz_cloud(q.filtered[0], q.per[0], o.robot_filtered.frame_id);
    o.robot_filtered.stamp = rs;
    o.backhoe_filtered = make_xyz_cloud(q.filtered[1], q.per[1], o.backhoe_filtered.frame_id);
    o.backhoe_filtered.stamp = bs;
    if (!q.origin_set) return;   // :309
    uint64_t base = 0;
    for (int i = 0; i < 2; ++i) {
        if (q.tf[i])
            (i == 0 ? o.merge.robot_colored : o.merge.backhoe_colored) =
                make_xyzrgb_cloud(q.merged + 32 * base, q.per[i], "map");
        base += q.per[i];
    }
    o.merge.merged = make_xyzrgb_cloud(q.merged + 32 * q.keep_off, q.keep_n, "map");
}

// ---- virtual_lidar ---------------------------------------------------------------------------
void SimplifiedDualLidarOptimizer::terrainCallback(const PointCloud2 &msg) {
    err_.clear();
    terrain_cloud_ = true;
    pcp_cloud_view v{};
    if (!cloud_view(msg, v, &err_)) return;
    // empty cloud: the old tree stays (:184-191), ground heights see the empty cloud
    if (multi_) {
        if (pcp_multi_set_terrain(multi_, &v) != PCP_OK) err_ = pcp_multi_last_error(multi_);
    } else if (pcp_set_terrain(dev_.ctx(), &v) != PCP_OK) {
        err_ = dev_.error();
    }
}

void SimplifiedDualLidarOptimizer::zx120PointsCallback(const PointCloud2 &msg) {
    err_.clear();
    pcp_cloud_view v{};
    if (!cloud_view(msg, v, &err_)) return;
    zx120_size_ = v.n;   // zx120_cloud_ is replaced by every message, empty ones too (:195-196)
    if (multi_) {
        if (pcp_multi_set_aux_cloud(multi_, &v) != PCP_OK) err_ = pcp_multi_last_error(multi_);
    } else if (pcp_set_aux_cloud(dev_.ctx(), &v) != PCP_OK) {
        err_ = dev_.error();
    }
}

bool SimplifiedDualLidarOptimizer::excavationAreaCallback(const PointCloud2 &msg) {
    err_.clear();
    pcp_cloud_view v;
    std::string why;
    if (!cloud_view(msg, v, &why)) {   // fromROSMsg would throw: logged, nothing rebuilt
        err_ = "excavation area: " + why;
        return false;
    }
    if (msg.empty()) return false;   // :168
    double bb[6];
    uint64_t n = 0;
    if (defer_grid_) {   // composed chain: enqueued, settled by the next tick
        if (pcp_set_excavation_area_async(dev_.ctx(), &v, p_.grid_resolution, p_.vertical_layers,
                                          bb, &n) != PCP_OK) {
            err_ = dev_.error();
            return false;
        }
        n_cells_ = n;                 // the capacity: the flags' bytes until settled
        grid_pending_ = n != 0;
        flags_.assign(n_cells_, 0);   // fresh GridCells (:259)
        std::memcpy(bbox_, bb, sizeof(bbox_));
        return true;
    }
    if (pcp_set_excavation_area(dev_.ctx(), &v, p_.grid_resolution, p_.vertical_layers, bb, &n) !=
        PCP_OK) {
        err_ = dev_.error();   // "Failed to process excavation area" (:175-177)
        return false;
    }
    if (multi_ && n) {   // rank 0 built the cells: replicate them on every rank
        std::vector<double> xyz(3 * n);
        std::vector<float> nrm(3 * n);
        uint64_t got = 0;
        if (pcp_get_cells(dev_.ctx(), xyz.data(), nrm.data(), n, &got) != PCP_OK ||
            pcp_multi_set_cells(multi_, xyz.data(), nrm.data(), got) != PCP_OK) {
            err_ = pcp_multi_last_error(multi_);
            return false;
        }
    }
    n_cells_ = n;
    flags_.assign(n_cells_, 0);   // excavation_grid_3d_ rebuilt from fresh GridCells (:259)
    std::memcpy(bbox_, bb, sizeof(bbox_));
    return true;
}

ExcavationTerrainGenerator::Output SimplifiedDualLidarOptimizer::carveCallbacks(
    ExcavationTerrainGenerator &gen, const PointCloud2 &msg, const Transform *zx120_base,
    const pcp_cloud_view *landed, const PointCloud2 *zx120) {
    // the zx120 callback's own error only when the callbacks before it left none
    auto zx_callback = [&]() {
        if (!zx120) return;
        std::string e0 = err_;
        zx120PointsCallback(*zx120);
        if (err_.empty()) err_ = std::move(e0);
    };
    // (the same bytes as the message, in pinned memory the device reads in place: then the
    // message may still be its header, ComposedFilterMerge's deferred messages)
    pcp_cloud_view v{};
    const bool in_place = landed && landed->n && landed->n == msg.size() && landed->point_step == 32;
    if (in_place) v = *landed;
    // the message the reference's callbacks see: a deferred message (header only) rebuilt from
    // its landing when a path below republishes it or hands it to the per-node callbacks
    PointCloud2 full;
    auto whole = [&]() -> const PointCloud2 & {
        if (!(in_place && msg.data.empty())) return msg;
        full = make_xyzrgb_cloud(landed->data, landed->n, msg.frame_id);
        full.stamp = msg.stamp;
        return full;
    };
    if (!defer_grid_ || multi_ || !gen.p_.enabled || !zx120_base ||
        !(in_place || cloud_view(msg, v, nullptr))) {
        ExcavationTerrainGenerator::Output o = gen.matchedCloudCallback(whole(), zx120_base);
        if (!(o.area_published && !excavationAreaCallback(o.excavation_area) && !err_.empty()))
            terrainCallback(o.excavated_terrain);
        zx_callback();
        return o;
    }
    ExcavationTerrainGenerator::Output o;
    gen.err_.clear();
    err_.clear();
    pcp_rigid tf;
    for (int a = 0; a < 3; ++a) tf.t[a] = zx120_base->t[a];
    for (int a = 0; a < 4; ++a) tf.q[a] = zx120_base->q[a];
    uint64_t nt = 0, na = 0, ncap = 0;
    double pose[4], bb[6];
    if (pcp_excavate_bounds(&gen.p_, v.n, &nt, &na) != PCP_OK) {
        gen.err_ = "excavated_surface_generator: bad parameters";
        o.excavated_terrain = whole();
        terrainCallback(o.excavated_terrain);
        zx_callback();
        return o;
    }
    // the records stay where they land (null outputs): the zx120 index is enqueued behind the
    // carve's consumers first, then the two messages are copied straight from the landing
    const void *terr = nullptr, *area = nullptr;
    if (pcp_excavate_area_async(dev_.ctx(), &v, &gen.p_, &tf, nullptr, nt, &nt, nullptr, na, &na,
                                pose, p_.grid_resolution, p_.vertical_layers, bb, &ncap) != PCP_OK ||
        pcp_excavate_landed(dev_.ctx(), &terr, &area) != PCP_OK) {
        gen.err_ = dev_.error();
        o.excavated_terrain = whole();
        zx_callback();
        return o;
    }
    zx_callback();
    o.excavated_terrain = make_xyzrgb_cloud(terr, nt, "map");
    o.excavated_terrain.stamp = msg.stamp;
    o.excavation_area = make_xyzrgb_cloud(area, na, "map");
    o.excavation_area.stamp = msg.stamp;
    o.area_published = true;
    o.center[0] = pose[0];
    o.center[1] = pose[1];
    o.center[2] = pose[2];
    o.yaw = pose[3];
    // this node as its two callbacks leave it: the terrain message arrived; a non-empty area
    // rebuilt the (deferred) grid, an empty one kept the previous (:168)
    terrain_cloud_ = true;
    if (na) {
        n_cells_ = ncap;
        grid_pending_ = ncap != 0;
        flags_.assign(n_cells_, 0);   // fresh GridCells (:259)
        std::memcpy(bbox_, bb, sizeof(bbox_));
    }
    return o;
}

size_t SimplifiedDualLidarOptimizer::lastCells() {
    if (grid_pending_) {
        uint64_t n = 0;
        if (pcp_cells_count(dev_.ctx(), &n) == PCP_OK) {
            n_cells_ = n;
            flags_.resize(n_cells_);
        } else {
            err_ = dev_.error();
        }
        grid_pending_ = false;
    }
    return n_cells_;
}

void SimplifiedDualLidarOptimizer::setExcavationGrid(const std::vector<double> &xyz,
                                                     const std::vector<float> &normals,
                                                     const double grid_bbox[6]) {
    err_.clear();
    grid_pending_ = false;   // (pcp_set_cells settles a pending setup first)
    n_cells_ = xyz.size() / 3;
    flags_.assign(n_cells_, 0);   // fresh GridCells (:259, ctor :34-43)
    std::memcpy(bbox_, grid_bbox, sizeof(bbox_));
    const int rc = multi_ ? pcp_multi_set_cells(multi_, xyz.data(), normals.data(), n_cells_)
                          : pcp_set_cells(dev_.ctx(), xyz.data(), normals.data(), n_cells_);
    if (rc != PCP_OK) {
        err_ = multi_ ? pcp_multi_last_error(multi_) : dev_.error();
        n_cells_ = 0;
    }
}

static void appendf(std::string &s, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void appendf(std::string &s, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    s += buf;
    s += '\n';
}

// the two RCLCPP_INFO tables of runOptimization, line for line: evaluateZX120Only (:419-451)
// and the dual configuration (:522-543)
std::string optimization_log(const SimplifiedDualLidarOptimizer::LidarPosition &zx120,
                             const SimplifiedDualLidarOptimizer::LidarPosition &best,
                             double best_score, const pcp_vl_report &q, size_t zx120_size) {
    std::string log;
    const int tc = q.total_cells;
    // the colour lines divide first (static_cast<double>(n) / total_cells * 100.0, :401-416,
    // :504-519); the Debug Info lines multiply first (n * 100.0 / total_cells, :427-432): the
    // two can differ by an ulp, which can move a %.1f tie
    auto pct = [tc](int v) { return tc > 0 ? (double)v / tc * 100.0 : 0.0; };
    auto pct_mul = [tc](int v) { return tc > 0 ? v * 100.0 / tc : 0.0; };
    auto ratio = [](int red, int green) {
        return green > 0 ? (double)red / green
                         : (red > 0 ? std::numeric_limits<double>::infinity() : 0.0);
    };
    const char *rule = "========================================";
    const char *thin = "----------------------------------------";
    appendf(log, "%s", rule);
    appendf(log, "ZX120 LiDAR Only Evaluation");
    appendf(log, "%s", rule);
    appendf(log, "ZX120 Position: (%.2f, %.2f, %.2f)", zx120.x, zx120.y, zx120.z);
    appendf(log, "Total Score (ZX120 only): %.2f", q.zx120_total_score);
    appendf(log, "%s", thin);
    appendf(log, "Debug Info:");
    appendf(log, "  Cells in range: %d (%.1f%%)", q.zx120_range_ok, pct_mul(q.zx120_range_ok));
    appendf(log, "  Cells in FOV: %d (%.1f%%)", q.zx120_fov_ok, pct_mul(q.zx120_fov_ok));
    appendf(log, "  Cells visible: %d (%.1f%%)", q.zx120_visible_ok, pct_mul(q.zx120_visible_ok));
    appendf(log, "  ZX120 point cloud size: %zu", zx120_size);
    appendf(log, "%s", thin);
    appendf(log, "Color-based Area Analysis (ZX120 only):");
    appendf(log, "  Total cells: %d", tc);
    appendf(log, "  Green (Observable): %d cells (%.1f%%)", q.zx120_green, pct(q.zx120_green));
    appendf(log, "  Red (Occluded): %d cells (%.1f%%)", q.zx120_red, pct(q.zx120_red));
    appendf(log, "  Blue (Out of range): %d cells (%.1f%%)", q.zx120_blue, pct(q.zx120_blue));
    appendf(log, "  Yellow (Out of FOV): %d cells (%.1f%%)", q.zx120_yellow, pct(q.zx120_yellow));
    appendf(log, "  ---");
    appendf(log, "  Red/Green Ratio: %.3f", ratio(q.zx120_red, q.zx120_green));
    const int unobs_z = q.zx120_red + q.zx120_blue + q.zx120_yellow;
    appendf(log, "  Total Unobservable: %d cells (%.1f%%)", unobs_z, pct(unobs_z));
    appendf(log, "%s", rule);
    appendf(log, "%s", "");
    appendf(log, "%s", rule);
    appendf(log, "Dual LiDAR Configuration (ZX120 + Mobile)");
    appendf(log, "%s", rule);
    appendf(log, "Best Mobile LiDAR Position: (%.2f, %.2f, %.2f)", best.x, best.y, best.z);
    appendf(log, "Total Score: %.2f", best_score);
    appendf(log, "%s", rule);
    appendf(log, "Color-based Area Analysis:");
    appendf(log, "  Total cells: %d", tc);
    appendf(log, "  Green (Observable): %d cells (%.1f%%)", q.green, pct(q.green));
    appendf(log, "  Red (Occluded): %d cells (%.1f%%)", q.red, pct(q.red));
    appendf(log, "  Blue (Out of range): %d cells (%.1f%%)", q.blue, pct(q.blue));
    appendf(log, "  Yellow (Out of FOV): %d cells (%.1f%%)", q.yellow, pct(q.yellow));
    appendf(log, "  ---");
    appendf(log, "  Red/Green Ratio: %.3f", ratio(q.red, q.green));
    const int unobs = q.red + q.blue + q.yellow;
    appendf(log, "  Total Unobservable: %d cells (%.1f%%)", unobs, pct(unobs));
    appendf(log, "%s", rule);
    return log;
}

SimplifiedDualLidarOptimizer::Result SimplifiedDualLidarOptimizer::runOptimization(
    const Transform *zx120_base) {
    Result r;
    err_.clear();
    // :455 -- no grid, no terrain message, or getZX120Position failed
    if (n_cells_ == 0 || !terrain_cloud_ || !zx120_base) return r;
    // getZX120Position (:342-358)
    r.zx120.x = zx120_base->t[0] + 0.4;
    r.zx120.y = zx120_base->t[1] + 0.5;
    r.zx120.z = zx120_base->t[2] + 3.5;
    r.zx120.pitch = -M_PI / 6;
    r.zx120.yaw = 0.0;
    const double zx[5] = {r.zx120.x, r.zx120.y, r.zx120.z, r.zx120.pitch, r.zx120.yaw};
    const pcp_vl_params p{p_.grid_resolution, p_.sensor_height, p_.search_radius, p_.max_distance,
                          p_.num_candidates, p_.vertical_layers};
    const int gs = (int)std::ceil(std::sqrt((double)p_.num_candidates));
    std::vector<double> poses(5 * (size_t)std::max(1, gs * gs));
    uint64_t n = 0;
    std::vector<double> totals(poses.size() / 5);
    int rc;
    if (multi_) {
        if (pcp_generate_candidates(dev_.ctx(), bbox_, &p, zx, poses.data(), poses.size() / 5,
                                    &n) != PCP_OK) {
            err_ = dev_.error();
            return r;
        }
        // the candidate loop (:467-475) sharded over multi_'s devices, one collective
        // (identical results)
        rc = pcp_multi_score_poses(multi_, poses.data(), n, zx, &p, flags_.data(), totals.data(),
                                   nullptr, &r.report);
    } else {   // generateCandidatePositions + the candidate loop, one round trip
        // (a deferred grid: flags_ holds the capacity's fresh bytes, settled by this call)
        rc = pcp_generate_and_score(dev_.ctx(), bbox_, &p, zx, poses.data(), poses.size() / 5, &n,
                                    flags_.data(), totals.data(), nullptr, &r.report);
    }
    if (rc != PCP_OK) {
        err_ = multi_ ? pcp_multi_last_error(multi_) : dev_.error();
        grid_pending_ = false;
        return r;
    }
    if (grid_pending_) {   // the tick settled the deferred grid: its count is final now
        lastCells();
        // :455 -- the reference never ticks over an empty grid (the results of the tick that
        // settled it are discarded, as if it had returned early)
        if (n_cells_ == 0) return Result{};
    }
    r.ran = true;
    r.candidates.resize(n);
    for (uint64_t i = 0; i < n; ++i) {
        LidarPosition &c = r.candidates[i];
        c.x = poses[5 * i];
        c.y = poses[5 * i + 1];
        c.z = poses[5 * i + 2];
        c.pitch = poses[5 * i + 3];
        c.yaw = poses[5 * i + 4];
        c.total_score = totals[i];
    }
    r.best_score = r.report.best_score;
    if (r.report.best_idx >= 0) r.best = r.candidates[r.report.best_idx];   // else default (:465)
    r.log = optimization_log(r.zx120, r.best, r.best_score, r.report, zx120_size_);
    return r;
}

// ---- ExcavationTerrainGenerator ----------------------------------------------------------------
ExcavationTerrainGenerator::Output ExcavationTerrainGenerator::matchedCloudCallback(
    const PointCloud2 &msg, const Transform *zx120_base) {
    Output o;
    err_.clear();
    if (!p_.enabled || !zx120_base) {   // :260-263, :276-279: republish the input
        o.excavated_terrain = msg;
        return o;
    }
    pcp_cloud_view v;
    std::string why;
    if (!cloud_view(msg, v, &why)) {
        err_ = "excavated_surface_generator: " + why;
        o.excavated_terrain = msg;
        return o;
    }
    pcp_rigid tf;
    for (int a = 0; a < 3; ++a) tf.t[a] = zx120_base->t[a];
    for (int a = 0; a < 4; ++a) tf.q[a] = zx120_base->q[a];
    uint64_t nt = 0, na = 0;
    double pose[4];
    if (pcp_excavate_bounds(&p_, v.n, &nt, &na) != PCP_OK) {
        err_ = "excavated_surface_generator: bad parameters";
        o.excavated_terrain = msg;
        return o;
    }
    uint8_t *terr = landing(terr_, nt * 32 + 32), *area = landing(area_, na * 32 + 32);
    if (pcp_excavate(dev_.ctx(), &v, &p_, &tf, terr, nt, &nt, area, na, &na, pose) != PCP_OK) {
        err_ = dev_.error();
        o.excavated_terrain = msg;
        return o;
    }
    o.excavated_terrain = make_xyzrgb_cloud(terr, nt, "map");   // header kept, frame map
    o.excavated_terrain.stamp = msg.stamp;
    o.excavation_area = make_xyzrgb_cloud(area, na, "map");
    o.excavation_area.stamp = msg.stamp;
    o.area_published = true;
    o.center[0] = pose[0];
    o.center[1] = pose[1];
    o.center[2] = pose[2];
    o.yaw = pose[3];
    return o;
}

// ---- DrivableAreaMapper ---------------------------------------------------------------------------
bool DrivableAreaMapper::robotCloudCallback(const PointCloud2 &msg, const Transform *cloud_to_map,
                                            const Transform *robot_base, OccupancyGrid &out) {
    err_.clear();
    if (!cloud_to_map) return false;   // "Transform ... not available yet"
    pcp_cloud_view v;
    std::string why;
    if (!cloud_view(msg, v, &why)) {
        err_ = "calc_drivable_area: " + why;
        return false;
    }
    if (msg.empty()) return false;   // "Received empty point cloud"
    if (!robot_base) return false;   // "Could not get robot transform"
    const double rx = robot_base->t[0], ry = robot_base->t[1];
    if (!start_set_) {   // :132-138
        start_x_ = rx;
        start_y_ = ry;
        start_set_ = true;
    }
    pcp_rigid tf;
    for (int a = 0; a < 3; ++a) tf.t[a] = cloud_to_map->t[a];
    for (int a = 0; a < 4; ++a) tf.q[a] = cloud_to_map->q[a];
    const int gw = (int)(p_.map_width / p_.grid_resolution);
    const int gh = (int)(p_.map_height / p_.grid_resolution);
    out.data.assign((size_t)std::max(gw, 0) * (size_t)std::max(gh, 0), -1);
    int32_t dims[2];
    double origin[2];
    if (pcp_drivable_area(dev_.ctx(), &v, &tf, rx, ry, start_x_, start_y_, &p_, out.data.data(),
                          out.data.size(), dims, origin) != PCP_OK) {
        err_ = dev_.error();
        return false;
    }
    out.frame_id = "map";
    out.resolution = p_.grid_resolution;
    out.width = (uint32_t)dims[0];
    out.height = (uint32_t)dims[1];
    out.origin_x = origin[0];
    out.origin_y = origin[1];
    return true;
}

}  // namespace pcp
