// pcp_nodes_cli.cpp -- drives the C++ node cores (pcp_nodes.hpp) from files, for the parity
// tests, and runs the streaming replay benchmark (BASELINE configs[4] on one GPU).
//
//   pcp_nodes_cli filter  IN.f32 N STEP LEAF FRONT SIDE HEIGHT OUT.f32
//   pcp_nodes_cli merge   ROBOT.f32 RN ZX.f32 ZN TR(7) TZ(7) OUT.f32        (t xyz, q xyzw)
//   pcp_nodes_cli vlidar  TERRAIN.f32 TN AUX.f32 AN CELLS.f64 NORMALS.f32 CN BBOX(6) ZXT(3) NUMC
//                         MAXD OUT_TOTALS.f64 OUT_FLAGS.u8 OUT_REPORT.txt [TICKS]
//   pcp_nodes_cli drivable IN.f32 N STEP TF(7) R1(2) R2(2) OUT.i8
//   pcp_nodes_cli replay  TERRAIN.f32 TN CELLS.f64 NORMALS.f32 CN BBOX(6) FRAMES POINTS
//
// Tuples are comma-separated doubles.  .f32 clouds are PointXYZRGB-like records of STEP bytes
// (terrain/aux: 32 B, x/y/z at 0/4/8).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <malloc.h>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "pcp_nodes.hpp"

using namespace pcp;

static std::vector<uint8_t> read_file(const char *path) {
    std::vector<uint8_t> b;
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path);
        std::exit(2);
    }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    b.resize((size_t)n);
    if (n && std::fread(b.data(), 1, (size_t)n, f) != (size_t)n) std::exit(2);
    std::fclose(f);
    return b;
}

static void write_file(const char *path, const void *p, size_t n) {
    FILE *f = std::fopen(path, "wb");
    if (!f || (n && std::fwrite(p, 1, n, f) != n)) {
        std::fprintf(stderr, "cannot write %s\n", path);
        std::exit(2);
    }
    std::fclose(f);
}

static std::vector<double> tuple(const char *s) {
    std::vector<double> v;
    std::stringstream ss(s);
    std::string tok;
    while (std::getline(ss, tok, ',')) v.push_back(std::strtod(tok.c_str(), nullptr));
    return v;
}

static PointCloud2 cloud_from(const std::vector<uint8_t> &raw, size_t n, uint32_t step,
                              const std::string &frame) {
    PointCloud2 m;
    m.frame_id = frame;
    m.width = (uint32_t)n;
    m.point_step = step;
    m.row_step = step * (uint32_t)n;
    m.fields = {{"x", 0}, {"y", 4}, {"z", 8}};
    m.data.assign(raw.begin(), raw.begin() + std::min(raw.size(), n * step));
    return m;
}

static Transform tf_from(const std::vector<double> &v) {
    Transform t;
    for (int i = 0; i < 3; ++i) t.t[i] = v[i];
    for (int i = 0; i < 4; ++i) t.q[i] = v[3 + i];
    return t;
}

static int cmd_filter(Device &dev, char **a) {
    const auto raw = read_file(a[0]);
    const size_t n = std::strtoull(a[1], nullptr, 10);
    SimplifiedScanMatcher::Params p;
    p.voxel_leaf_size = std::strtod(a[3], nullptr);
    p.robot_front_range = std::strtod(a[4], nullptr);
    p.robot_side_range = std::strtod(a[5], nullptr);
    p.robot_height_range = std::strtod(a[6], nullptr);
    SimplifiedScanMatcher node(dev, p);
    PointCloud2 in = cloud_from(raw, n, (uint32_t)std::strtoul(a[2], nullptr, 10), "velodyne_link");
    in.stamp = 12.5;
    PointCloud2 out = node.robotCloudCallback(in);
    if (!node.lastError().empty()) {
        std::fprintf(stderr, "filter: %s\n", node.lastError().c_str());
        return 1;
    }
    if (out.frame_id != in.frame_id || out.stamp != in.stamp || out.point_step != 16) return 3;
    write_file(a[7], out.data.data(), out.data.size());
    std::printf("{\"n_out\": %zu, \"n_cropped\": %zu}\n", out.size(), node.lastCroppedSize());
    return 0;
}

static int cmd_merge(Device &dev, char **a) {
    const auto r = read_file(a[0]), z = read_file(a[2]);
    const size_t rn = std::strtoull(a[1], nullptr, 10), zn = std::strtoull(a[3], nullptr, 10);
    GnssGicpMatcher node(dev);
    node.robotCloudCallback(make_xyz_cloud(reinterpret_cast<const float *>(r.data()), rn, "four_wheel_robot/velodyne_link"));
    node.backhoeCloudCallback(make_xyz_cloud(reinterpret_cast<const float *>(z.data()), zn, "zx120/velodyne_link"));
    const Transform tr = tf_from(tuple(a[4])), tz = tf_from(tuple(a[5]));
    auto o = node.processPointClouds(true, &tr, &tz);
    if (!node.lastError().empty()) {
        std::fprintf(stderr, "merge: %s\n", node.lastError().c_str());
        return 1;
    }
    if (o.merged.size() != o.robot_colored.size() + o.backhoe_colored.size()) return 3;
    auto none = node.processPointClouds(false, &tr, &tz);   // origin not set: nothing (:309)
    if (!none.merged.empty()) return 4;
    auto only_robot = node.processPointClouds(true, &tr, nullptr);   // zx120 TF failed
    if (only_robot.merged.size() != o.robot_colored.size()) return 5;
    write_file(a[6], o.merged.data.data(), o.merged.data.size());
    std::printf("{\"n_out\": %zu, \"robot\": %zu, \"backhoe\": %zu}\n", o.merged.size(),
                o.robot_colored.size(), o.backhoe_colored.size());
    return 0;
}

// PCP_DEVICES=d0,d1,...: the virtual-LiDAR node shards its poses over these devices (pcp_multi)
static std::unique_ptr<MultiDevice> multi_from_env() {
    const char *e = std::getenv("PCP_DEVICES");
    if (!e || !*e) return nullptr;
    std::vector<int> d;
    for (const char *p = e; *p;) {
        d.push_back(std::atoi(p));
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
    }
    return std::unique_ptr<MultiDevice>(new MultiDevice(d));
}

static int cmd_vlidar(Device &dev, char **a, int argc) {
    const auto t = read_file(a[0]), ax = read_file(a[2]), c = read_file(a[4]),
               nr = read_file(a[5]);
    const size_t tn = std::strtoull(a[1], nullptr, 10), an = std::strtoull(a[3], nullptr, 10),
                 cn = std::strtoull(a[6], nullptr, 10);
    const auto bbox = tuple(a[7]), zxt = tuple(a[8]);
    SimplifiedDualLidarOptimizer::Params p;
    p.num_candidates = std::atoi(a[9]);
    p.max_distance = std::strtod(a[10], nullptr);
    std::unique_ptr<MultiDevice> md = multi_from_env();
    std::unique_ptr<SimplifiedDualLidarOptimizer> nodep(
        md ? new SimplifiedDualLidarOptimizer(*md, p) : new SimplifiedDualLidarOptimizer(dev, p));
    SimplifiedDualLidarOptimizer &node = *nodep;
    Transform zx;
    zx.t[0] = zxt[0];
    zx.t[1] = zxt[1];
    zx.t[2] = zxt[2];
    // before any data: the early return of :455
    if (node.runOptimization(&zx).ran) return 3;
    node.terrainCallback(cloud_from(t, tn, 32, "map"));
    node.zx120PointsCallback(cloud_from(ax, an, 32, "velodyne_link"));
    std::vector<double> xyz(cn * 3);
    std::vector<float> nrm(cn * 3);
    std::memcpy(xyz.data(), c.data(), xyz.size() * 8);
    std::memcpy(nrm.data(), nr.data(), nrm.size() * 4);
    node.setExcavationGrid(xyz, nrm, bbox.data());
    if (node.runOptimization(nullptr).ran) return 4;   // TF missing
    const int ticks = argc > 14 ? std::atoi(a[14]) : 1;
    SimplifiedDualLidarOptimizer::Result r;
    for (int i = 0; i < ticks; ++i) r = node.runOptimization(&zx);   // flags carry over
    if (!r.ran) {
        std::fprintf(stderr, "vlidar: %s\n", node.lastError().c_str());
        return 1;
    }
    std::vector<double> tot(r.candidates.size());
    for (size_t i = 0; i < tot.size(); ++i) tot[i] = r.candidates[i].total_score;
    write_file(a[11], tot.data(), tot.size() * 8);
    write_file(a[12], node.cellFlags().data(), node.cellFlags().size());
    write_file(a[13], r.log.data(), r.log.size());
    std::printf("{\"n_candidates\": %zu, \"best_idx\": %lld, \"best\": [%.17g, %.17g, %.17g], "
                "\"devices\": %d, \"rccl\": %d}\n",
                r.candidates.size(), (long long)r.report.best_idx, r.best.x, r.best.y, r.best.z,
                md ? md->size() : 1, md && md->usesRccl() ? 1 : 0);
    return 0;
}

// HDL-64-like scan (64 rings, -24.9..+2 deg) of n points against a ground plane
static std::vector<float> synth_scan(size_t n, double h, std::mt19937_64 &rng) {
    std::uniform_real_distribution<double> ua(-M_PI, M_PI), ur(1.0, 40.0);
    std::uniform_int_distribution<int> ring(0, 63);
    std::vector<float> p(4 * n);
    for (size_t i = 0; i < n; ++i) {
        const double el = (-24.9 + 26.9 * ring(rng) / 63.0) * M_PI / 180.0, az = ua(rng);
        double r = ur(rng);
        if (el < 0) r = std::min(r, h / std::sin(-el));
        p[4 * i] = (float)(r * std::cos(el) * std::cos(az));
        p[4 * i + 1] = (float)(r * std::cos(el) * std::sin(az));
        p[4 * i + 2] = (float)(r * std::sin(el));
        p[4 * i + 3] = 0.f;
    }
    return p;
}

static int cmd_replay(Device &dev, char **a) {
    const auto t = read_file(a[0]), c = read_file(a[2]), nr = read_file(a[3]);
    const size_t tn = std::strtoull(a[1], nullptr, 10), cn = std::strtoull(a[4], nullptr, 10);
    const auto bbox = tuple(a[5]);
    const int frames = std::atoi(a[6]);
    const size_t npts = std::strtoull(a[7], nullptr, 10);
    // chain = 1: the launch file's whole per-frame chain -- the merged cloud goes through
    // excavated_surface_generator, whose /excavated_terrain and /excavation_area feed
    // virtual_lidar every frame (terrain index, normals, cell grid rebuilt per frame)
    const bool chain = a[8] && std::atoi(a[8]) != 0;
    // DUMP_DIR (optional): the inputs and every node's outputs of frames 0, 1, 2 and the last
    // one, for the oracle check of the streamed chain (tests/test_nodes_cli.py)
    const std::string dump = (a[8] && a[9]) ? a[9] : "";
    SimplifiedScanMatcher filt(dev);
    GnssGicpMatcher merger(dev);
    ComposedFilterMerge front(dev);
    bool front_fused = true;
    if (const char *ff = std::getenv("PCP_FRONT_FUSED")) front_fused = std::atoi(ff) != 0;
    // the carve node and virtual_lidar's area + terrain callbacks composed (default)
    bool carve_fused = true;
    if (const char *cf = std::getenv("PCP_CARVE_FUSED")) carve_fused = std::atoi(cf) != 0;
    // the composed carve reads the merger's landed records in place (default) / the message
    bool carve_landed = true;
    if (const char *cl = std::getenv("PCP_CARVE_LANDED")) carve_landed = std::atoi(cl) != 0;
    // the zx120 cloud's callback composed into the carve call as well (PCP_CARVE_ZX=1): its
    // index is enqueued before the carve's messages are copied out of the landing.  Off by
    // default: no faster (p50 0.644-0.673 vs 0.637-0.648 ms, profiles/r05_c5_host_bbox_zx_ab.log)
    bool carve_zx = false;
    if (const char *cz = std::getenv("PCP_CARVE_ZX")) carve_zx = std::atoi(cz) != 0;
    ExcavationTerrainGenerator gen(dev);
    SimplifiedDualLidarOptimizer vl(dev);
    // the nodes composed in one process: the grid setup is enqueued by the area callback and
    // waited for once by the tick (PCP_AREA_ASYNC=0: settled in the area callback, as a ROS shell
    // that publishes the grid markers there)
    bool area_async = true;
    if (const char *ea = std::getenv("PCP_AREA_ASYNC")) area_async = std::atoi(ea) != 0;
    vl.setDeferredGrid(area_async);
    // the filter / merger messages copied out of their landing after the composed carve has
    // read the merged cloud in place (default; only where every composition applies), while the
    // device builds the grid.  PCP_FRONT_DEFER=0: copied by the front call
    bool front_defer = true;
    if (const char *fd = std::getenv("PCP_FRONT_DEFER")) front_defer = std::atoi(fd) != 0;
    front_defer = front_defer && front_fused && chain && carve_fused && carve_landed && area_async &&
                  !carve_zx;
    // PCP_REPLAY_NO_TF=k: frame k's map -> zx120/base_link lookup fails (the carve's fallback:
    // the merged cloud republished as the terrain, no area); the line reports that frame's
    // terrain message (a deferred merged message must not go out as its header)
    long no_tf_frame = -1;
    if (const char *nt = std::getenv("PCP_REPLAY_NO_TF")) no_tf_frame = std::atol(nt);
    size_t no_tf_points = 0, no_tf_bytes = 0, no_tf_merged = 0;
    vl.terrainCallback(cloud_from(t, tn, 32, "map"));
    std::vector<double> xyz(cn * 3);
    std::vector<float> nrm(cn * 3);
    std::memcpy(xyz.data(), c.data(), xyz.size() * 8);
    std::memcpy(nrm.data(), nr.data(), nrm.size() * 4);
    vl.setExcavationGrid(xyz, nrm, bbox.data());
    std::mt19937_64 rng(20260227);
    const Transform robot_tf{{8.0, -3.0, 2.0}, {0.0, 0.0, 0.2588190451025208, 0.9659258262890683}};
    const Transform zx_tf{{0.55, 0.4, 3.5}, {0.0, 0.21633, 0.0, 0.97632}};
    const Transform zx_base{{0.0, 0.0, 0.0}, {0, 0, 0, 1}};
    std::vector<double> lat;
    std::vector<double> lat_frame;   // in frame order (the sorted copy gives the percentiles)
    // per-callback wall time (ms): filter x2, merger, carve, area, terrain, zx120 cloud, tick
    constexpr int kStages = 7;
    static const char *kStageName[kStages] = {"filter", "merge", "carve", "area",
                                              "terrain", "zx120", "tick"};
    std::vector<double> stage[kStages], stage_frame[kStages];   // sorted later / frame order
    size_t merged_n = 0, best = 0, cells_n = cn;
    uint64_t realloc_after_warmup = 0, ra0 = 0;
    std::string dumped;
    const bool alloc_trace = std::getenv("PCP_ALLOC_TRACE") != nullptr;
    for (int f = 0; f < frames + 2; ++f) {
        if (alloc_trace) std::fprintf(stderr, "replay frame %d\n", f);
        if (f == 2) pcp_alloc_stats(&ra0, nullptr, nullptr);
        auto rs = synth_scan(npts, 2.0, rng), zs = synth_scan(npts, 3.5, rng);
        PointCloud2 rm = make_xyz_cloud(rs.data(), npts, "four_wheel_robot/velodyne_link");
        PointCloud2 zm = make_xyz_cloud(zs.data(), npts, "zx120/velodyne_link");
        const auto t0 = std::chrono::steady_clock::now();
        double st[kStages] = {};
        auto lap = [&st, last = t0](int k) mutable {
            const auto now = std::chrono::steady_clock::now();
            st[k] = std::chrono::duration<double, std::milli>(now - last).count();
            last = now;
        };
        // pointcloud_filter: both sensors; pointcloud_merger: 10 Hz tick; virtual_lidar: zx120
        // filtered cloud + the pose search.  Composed (PCP_FRONT_FUSED, default): the filter
        // and merger nodes in one call and one synchronisation (stage "filter" then holds both)
        PointCloud2 rf, zf;
        GnssGicpMatcher::Output o;
        pcp_cloud_view front_landed{};
        ComposedFilterMerge::Output fo;
        // the front's messages (when deferred: after the carve call)
        auto take_front = [&]() {
            front.messages(fo);
            rf = std::move(fo.robot_filtered);
            zf = std::move(fo.backhoe_filtered);
            o = std::move(fo.merge);
        };
        if (front_fused) {
            fo = front.frame(rm, zm, true, &robot_tf, &zx_tf, front_defer);
            if (!front.lastError().empty()) {
                std::fprintf(stderr, "replay: filter+merge failed: %s\n", front.lastError().c_str());
                return 1;
            }
            front_landed = fo.merged_landed;
            if (front_defer) o.merged = fo.merge.merged;   // (its header: the carve reads the landing)
            else take_front();
            lap(0);
            lap(1);
        } else {
            rf = filt.robotCloudCallback(rm);
            zf = filt.backhoeCloudCallback(zm);
            lap(0);
            merger.robotCloudCallback(rf);
            merger.backhoeCloudCallback(zf);
            o = merger.processPointClouds(true, &robot_tf, &zx_tf);
            lap(1);
        }
        ExcavationTerrainGenerator::Output e;
        const bool zx_in_carve = chain && carve_fused && carve_zx;
        const bool no_tf = (long)f == no_tf_frame;
        if (chain && carve_fused) {   // the carve + both callbacks (stage "carve" holds all three)
            e = vl.carveCallbacks(gen, o.merged, no_tf ? nullptr : &zx_base,
                                  front_fused && carve_landed ? &front_landed : nullptr,
                                  zx_in_carve ? &zf : nullptr);
            if (no_tf) {
                no_tf_points = e.excavated_terrain.size();
                no_tf_bytes = e.excavated_terrain.data.size();
                no_tf_merged = front_landed.n;
            } else if (!e.area_published) {
                std::fprintf(stderr, "replay: carve failed: %s\n", gen.lastError().c_str());
                return 1;
            }
            if (front_defer) take_front();
            lap(2);
            lap(3);
            lap(4);
        } else if (chain) {
            e = gen.matchedCloudCallback(o.merged, &zx_base);
            if (!e.area_published) {
                std::fprintf(stderr, "replay: carve failed: %s\n", gen.lastError().c_str());
                return 1;
            }
            lap(2);
            vl.excavationAreaCallback(e.excavation_area);
            lap(3);
            vl.terrainCallback(e.excavated_terrain);
            lap(4);
        }
        if (!zx_in_carve) vl.zx120PointsCallback(zf);   // (else made by carveCallbacks)
        lap(5);
        auto r = vl.runOptimization(&zx_base);
        lap(6);
        if (chain) cells_n = vl.lastCells();   // (settled by the tick)
        const auto t1 = std::chrono::steady_clock::now();
        if (f >= 2)
            for (int k = 0; k < kStages; ++k) {
                stage[k].push_back(st[k]);
                stage_frame[k].push_back(st[k]);
            }
        if (!r.ran) {
            std::fprintf(stderr, "replay: pose search did not run: %s\n", vl.lastError().c_str());
            return 1;
        }
        merged_n = o.merged.size();
        best = (size_t)r.report.best_idx;
        if (f >= 2) lat.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        if (f >= 2) lat_frame.push_back(lat.back());
        if (!dump.empty() && chain && (f < 3 || f == frames + 1)) {
            const std::string pre = dump + "/f" + std::to_string(f) + "_";
            write_file((pre + "rscan.f32").c_str(), rs.data(), rs.size() * 4);
            write_file((pre + "zscan.f32").c_str(), zs.data(), zs.size() * 4);
            write_file((pre + "rf.bin").c_str(), rf.data.data(), rf.data.size());
            write_file((pre + "zf.bin").c_str(), zf.data.data(), zf.data.size());
            write_file((pre + "merged.bin").c_str(), o.merged.data.data(), o.merged.data.size());
            // the carve's outputs, as published (they are the node inputs of this frame)
            write_file((pre + "terrain.bin").c_str(), e.excavated_terrain.data.data(),
                       e.excavated_terrain.data.size());
            write_file((pre + "area.bin").c_str(), e.excavation_area.data.data(),
                       e.excavation_area.data.size());
            uint64_t nc = 0;
            pcp_get_cells(dev.ctx(), nullptr, nullptr, 0, &nc);
            std::vector<double> cx(3 * nc);
            std::vector<float> cnr(3 * nc);
            if (nc) pcp_get_cells(dev.ctx(), cx.data(), cnr.data(), nc, &nc);
            write_file((pre + "cells.f64").c_str(), cx.data(), cx.size() * 8);
            write_file((pre + "cnrm.f32").c_str(), cnr.data(), cnr.size() * 4);
            std::vector<double> ps, tot;
            for (const auto &c : r.candidates) {
                ps.insert(ps.end(), {c.x, c.y, c.z, c.pitch, c.yaw});
                tot.push_back(c.total_score);
            }
            write_file((pre + "poses.f64").c_str(), ps.data(), ps.size() * 8);
            write_file((pre + "tot.f64").c_str(), tot.data(), tot.size() * 8);
            char buf[128];
            std::snprintf(buf, sizeof(buf), "%s{\"frame\": %d, \"best_idx\": %lld}",
                          dumped.empty() ? "" : ", ", f, (long long)r.report.best_idx);
            dumped += buf;
        }
    }
    {
        uint64_t ra1 = 0;
        pcp_alloc_stats(&ra1, nullptr, nullptr);
        realloc_after_warmup = ra1 - ra0;
    }
    std::string lat_s;
    for (size_t i = 0; i < lat_frame.size(); ++i) {
        char b[32];
        std::snprintf(b, sizeof(b), "%s%.4f", i ? ", " : "", lat_frame[i]);
        lat_s += b;
    }
    // the stage times of the slowest frames (what the tail is made of)
    std::string slow_s;
    {
        std::vector<size_t> ord(lat_frame.size());
        for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
        std::sort(ord.begin(), ord.end(),
                  [&lat_frame](size_t a, size_t b) { return lat_frame[a] > lat_frame[b]; });
        for (size_t r = 0; r < std::min<size_t>(4, ord.size()); ++r) {
            char b[96];
            std::snprintf(b, sizeof(b), "%s{\"frame\": %zu, \"ms\": %.4f", r ? ", " : "", ord[r],
                          lat_frame[ord[r]]);
            slow_s += b;
            for (int k = 0; k < kStages; ++k) {
                std::snprintf(b, sizeof(b), ", \"%s\": %.4f", kStageName[k], stage_frame[k][ord[r]]);
                slow_s += b;
            }
            slow_s += "}";
        }
    }
    std::sort(lat.begin(), lat.end());
    auto q = [&lat](double p) { return lat[std::min(lat.size() - 1, (size_t)(p * lat.size()))]; };
    std::string stage_s;
    for (int k = 0; k < kStages; ++k) {
        auto &v = stage[k];
        std::sort(v.begin(), v.end());
        char b[64];
        std::snprintf(b, sizeof(b), "%s\"%s\": %.4f", k ? ", " : "", kStageName[k],
                      v.empty() ? 0.0 : v[v.size() / 2]);
        stage_s += b;
    }
    std::printf("{\"frames\": %zu, \"points_per_scan\": %zu, \"chain\": %d, \"p50_ms\": %.4f, "
                "\"p99_ms\": %.4f, \"max_ms\": %.4f, \"merged_points\": %zu, \"cells\": %zu, "
                "\"best_idx\": %zu, \"reallocs_after_warmup\": %llu, \"dumped\": [%s], "
                "\"stage_p50_ms\": {%s}, \"slowest\": [%s], \"lat_ms\": [%s], "
                "\"no_tf\": {\"frame\": %ld, \"terrain_points\": %zu, \"terrain_bytes\": %zu, "
                "\"merged_points\": %zu}}\n",
                lat.size(), npts, chain ? 1 : 0, q(0.5), q(0.99), lat.back(), merged_n, cells_n,
                best, (unsigned long long)realloc_after_warmup, dumped.c_str(), stage_s.c_str(),
                slow_s.c_str(), lat_s.c_str(), no_tf_frame, no_tf_points, no_tf_bytes,
                no_tf_merged);
    return 0;
}

// area AREA.f32 N_AREA TERRAIN.f32 N_TERRAIN ZX120_BASE(x,y,z) NUM_CANDIDATES MAX_DISTANCE
//      OUT_TOTAL.f64 OUT_CELLS.f64 OUT_NORMALS.f32
// the virtual_lidar node from its /excavation_area message: excavationAreaCallback (GPU normals
// + 3-D cell grid), terrainCallback, one runOptimization tick (no zx120 cloud)
static int cmd_area(Device &dev, char **a) {
    const auto ar = read_file(a[0]), t = read_file(a[2]);
    const size_t an = std::strtoull(a[1], nullptr, 10), tn = std::strtoull(a[3], nullptr, 10);
    const auto zxt = tuple(a[4]);
    SimplifiedDualLidarOptimizer::Params p;
    p.num_candidates = std::atoi(a[5]);
    p.max_distance = std::strtod(a[6], nullptr);
    SimplifiedDualLidarOptimizer node(dev, p);
    node.excavationAreaCallback(cloud_from(ar, an, 32, "map"));
    if (!node.lastError().empty()) {
        std::fprintf(stderr, "area: %s\n", node.lastError().c_str());
        return 1;
    }
    node.terrainCallback(cloud_from(t, tn, 32, "map"));
    Transform zx;
    zx.t[0] = zxt[0];
    zx.t[1] = zxt[1];
    zx.t[2] = zxt[2];
    const auto r = node.runOptimization(&zx);
    if (!r.ran) {
        std::fprintf(stderr, "area: %s\n", node.lastError().c_str());
        return 1;
    }
    std::vector<double> tot(r.candidates.size());
    for (size_t i = 0; i < tot.size(); ++i) tot[i] = r.candidates[i].total_score;
    write_file(a[7], tot.data(), tot.size() * 8);
    uint64_t nc = 0;
    pcp_get_cells(dev.ctx(), nullptr, nullptr, 0, &nc);
    std::vector<double> xyz(nc * 3);
    std::vector<float> nrm(nc * 3);
    if (pcp_get_cells(dev.ctx(), xyz.data(), nrm.data(), nc, &nc) != PCP_OK) return 1;
    write_file(a[8], xyz.data(), xyz.size() * 8);
    write_file(a[9], nrm.data(), nrm.size() * 4);
    std::printf("{\"n_cells\": %llu, \"n_candidates\": %zu, \"best_idx\": %lld}\n",
                (unsigned long long)nc, r.candidates.size(), (long long)r.report.best_idx);
    return 0;
}

// calc_drivable_area: two robotCloudCallback frames of the same cloud at robot positions R1, R2
// (the first one fixes the start-clear centre), plus the skipped cases (no TF, empty cloud)
static int cmd_drivable(Device &dev, char **a) {
    const auto raw = read_file(a[0]);
    const size_t n = std::strtoull(a[1], nullptr, 10);
    const uint32_t step = (uint32_t)std::strtoul(a[2], nullptr, 10);
    const Transform tf = tf_from(tuple(a[3]));
    const auto r1 = tuple(a[4]), r2 = tuple(a[5]);
    DrivableAreaMapper node(dev);
    const PointCloud2 msg = cloud_from(raw, n, step, "four_wheel_robot/velodyne_link");
    OccupancyGrid g1, g2, skip;
    Transform b1, b2;
    b1.t[0] = r1[0];
    b1.t[1] = r1[1];
    b2.t[0] = r2[0];
    b2.t[1] = r2[1];
    if (node.robotCloudCallback(msg, nullptr, &b1, skip) || node.startSet()) return 3;
    if (node.robotCloudCallback(msg, &tf, nullptr, skip) || node.startSet()) return 4;
    if (node.robotCloudCallback(cloud_from(raw, 0, step, msg.frame_id), &tf, &b1, skip) ||
        node.startSet())
        return 5;
    if (!node.robotCloudCallback(msg, &tf, &b1, g1) || !node.robotCloudCallback(msg, &tf, &b2, g2)) {
        std::fprintf(stderr, "drivable: %s\n", node.lastError().c_str());
        return 1;
    }
    std::vector<int8_t> both(g1.data);
    both.insert(both.end(), g2.data.begin(), g2.data.end());
    write_file(a[6], both.data(), both.size());
    std::printf("{\"width\": %u, \"height\": %u, \"resolution\": %.17g, "
                "\"origin1\": [%.17g, %.17g], \"origin2\": [%.17g, %.17g]}\n",
                g1.width, g1.height, g1.resolution, g1.origin_x, g1.origin_y, g2.origin_x,
                g2.origin_y);
    return 0;
}

int main(int argc, char **argv) {
    // the container keeps the heap it freed: every frame's messages (MBs of PointCloud2 data)
    // are allocated and freed again, and glibc's defaults would map and unmap them (or trim the
    // heap top), paying their page faults every frame (C5 p50 -17 us, p99 -30 us,
    // profiles/r05_c5_malloc_ab.log).  PCP_MALLOC_KEEP=0: glibc's defaults
    {
        const char *mk = std::getenv("PCP_MALLOC_KEEP");
        if (!mk || std::atoi(mk) != 0) {
            mallopt(M_MMAP_THRESHOLD, 256 << 20);
            mallopt(M_TRIM_THRESHOLD, 1 << 30);
        }
    }
    // waits poll the completion signals instead of sleeping on an interrupt (the container's
    // three waits per frame return ~5 us sooner; C5 p50 0.593-0.607 vs 0.600-0.616 ms,
    // profiles/r05_c5_wait_ab.log).  Before the first HIP call; PCP_HSA_POLL=0: the default
    {
        const char *hp = std::getenv("PCP_HSA_POLL");
        if (!hp || std::atoi(hp) != 0) setenv("HSA_ENABLE_INTERRUPT", "0", 0);
    }
    if (argc < 2) {
        std::fprintf(stderr, "usage: pcp_nodes_cli filter|merge|vlidar|area|drivable|replay ...\n");
        return 2;
    }
    const std::string cmd = argv[1];
    const int need = cmd == "filter"   ? 8
                     : cmd == "merge"  ? 7
                     : cmd == "vlidar" ? 14
                     : cmd == "area"   ? 10
                     : cmd == "drivable" ? 7
                     : cmd == "replay" ? 8
                                       : -1;
    if (need < 0 || argc - 2 < need) {
        std::fprintf(stderr, "bad arguments for %s\n", cmd.c_str());
        return 2;
    }
    try {
        Device dev(0);
        if (cmd == "filter") return cmd_filter(dev, argv + 2);
        if (cmd == "merge") return cmd_merge(dev, argv + 2);
        if (cmd == "vlidar") return cmd_vlidar(dev, argv + 2, argc - 2);
        if (cmd == "area") return cmd_area(dev, argv + 2);
        if (cmd == "drivable") return cmd_drivable(dev, argv + 2);
        return cmd_replay(dev, argv + 2);
    } catch (const std::exception &e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
}
