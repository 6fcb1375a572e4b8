// pcp_nodes_selftest.cpp -- the node cores' host-only logic under AddressSanitizer +
// UndefinedBehaviorSanitizer (`make -C pointcloud_processor_amd/csrc asan`): the PointCloud2
// codec (pcl::toROSMsg / fromROSMsg layouts, field lookup, rejected layouts) and the
// no-device behaviour (Device / MultiDevice construction fails loudly: no CPU fallback).
// Runs without a GPU; the GPU paths of the same code are exercised by tests/test_nodes_cli.py.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "pcp_nodes.hpp"

using namespace pcp;

static int g_fail = 0;
#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail = 1;                                                    \
        }                                                                  \
    } while (0)

int main() {
    std::vector<float> xyz(16 * 5);
    for (size_t i = 0; i < xyz.size(); ++i) xyz[i] = (float)i * 0.5f;
    PointCloud2 m = make_xyz_cloud(xyz.data(), 16, "velodyne_link");
    CHECK(m.width == 16 && m.point_step == 16 && m.row_step == 256 && m.data.size() == 256);
    pcp_cloud_view v{};
    std::string why;
    CHECK(cloud_view(m, v, &why) && v.n == 16 && v.off_x == 0 && v.off_y == 4 && v.off_z == 8);
    CHECK(std::memcmp(v.data, xyz.data(), 256) == 0);
    std::vector<float> rec(8 * 3, 1.0f);
    PointCloud2 r = make_xyzrgb_cloud(rec.data(), 3, "map");
    CHECK(r.point_step == 32 && r.fields.size() == 4 && cloud_view(r, v, &why) && v.n == 3);
    PointCloud2 e = make_xyz_cloud(nullptr, 0, "map");   // empty message
    CHECK(cloud_view(e, v, &why) && v.n == 0 && v.data == nullptr);
    PointCloud2 bad = m;                                  // no z field
    bad.fields.pop_back();
    CHECK(!cloud_view(bad, v, &why) && !why.empty());
    bad = m;                                              // a FLOAT64 x is not read
    bad.fields[0].datatype = PointField::FLOAT64;
    CHECK(!cloud_view(bad, v, &why));
    bad = m;                                              // padded rows
    bad.row_step += 4;
    CHECK(!cloud_view(bad, v, &why));
    bad = m;                                              // truncated data blob
    bad.data.resize(100);
    CHECK(!cloud_view(bad, v, &why));
    bad = m;
    bad.is_bigendian = true;
    CHECK(!cloud_view(bad, v, &why));
    int ndev = 0;
    if (pcp_device_count(&ndev) != PCP_OK || ndev == 0) {   // no GPU: loud failures
        bool threw = false;
        try {
            Device d(0);
        } catch (const std::runtime_error &) {
            threw = true;
        }
        CHECK(threw);
        threw = false;
        try {
            MultiDevice md({0, 1});
        } catch (const std::runtime_error &) {
            threw = true;
        }
        CHECK(threw);
    }
    {   // runOptimization's log tables: the Debug Info lines multiply first (n * 100.0 /
        // total_cells, virtual_lidar.cpp:427-432), the colour lines divide first (:401-416):
        // 23 of 80 cells print 28.8 and 28.7 (the double of 23 / 80 lies below .2875)
        pcp_vl_report q{};
        q.total_cells = 80;
        q.zx120_range_ok = q.zx120_fov_ok = q.zx120_visible_ok = 23;
        q.zx120_green = 23;
        q.green = 49;
        SimplifiedDualLidarOptimizer::LidarPosition zx, best;
        const std::string log = optimization_log(zx, best, 1.0, q, 7);
        CHECK(log.find("  Cells in range: 23 (28.8%)") != std::string::npos);
        CHECK(log.find("  Cells visible: 23 (28.8%)") != std::string::npos);
        CHECK(log.find("  Green (Observable): 23 cells (28.7%)") != std::string::npos);
        CHECK(log.find("  Green (Observable): 49 cells (61.3%)") != std::string::npos);
        CHECK(log.find("  ZX120 point cloud size: 7") != std::string::npos);
    }
    if (g_fail) return 1;
    std::printf("nodes selftest ok\n");
    return 0;
}
