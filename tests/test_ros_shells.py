"""The rclcpp node shells (ros/src/*_node.cpp) against a ROS stand-in.

No ROS 2 install exists in this image, so the shells are compiled and linked against
tests/ros_stub (the slice of rclcpp / message / tf2_ros API they use) plus the real
libpcp_nodes.so + libpcp.so: a renamed core method, a wrong message field or a missing
exported symbol fails here.  The stand-in is also a small in-process bus (subscriptions,
publishers with counters, timers, parameters, a static TF table), so tests/ros_stub/
shell_driver.cpp runs the virtual_lidar shell on it and reports what each topic published:
on the CPU over a test double of the C ABI (tests/ros_stub/mock_pcp.cpp), on the GPU over the
real libpcp (the driver binary build() makes).
"""
import json
import os
import re
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pointcloud_processor_amd", "_lib")
NODES = ["pointcloud_filter", "pointcloud_merger", "excavated_surface_generator",
         "virtual_lidar", "calc_drivable_area"]


def test_shells_match_reference_executables():
    # ros/CMakeLists.txt builds one executable per reference node (reference CMakeLists.txt:47-142)
    cm = open(os.path.join(ROOT, "ros", "CMakeLists.txt")).read()
    for n in NODES:
        assert n in cm
        assert os.path.exists(os.path.join(ROOT, "ros", "src", f"{n}_node.cpp"))


@pytest.mark.parametrize("node", NODES)
def test_shell_compiles_and_links(node, tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    if not os.path.exists(os.path.join(LIB, "libpcp_nodes.so")):
        pytest.skip("libpcp_nodes.so not built (run __graft_entry__.build())")
    out = tmp_path / node
    cmd = ["g++", "-std=c++17", "-O0", "-Wall", "-Wextra", "-Werror",
           "-I" + os.path.join(ROOT, "tests", "ros_stub"),
           "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "pointcloud_processor_amd", "csrc", "host"),
           "-I" + os.path.join(ROOT, "ros", "src"),
           os.path.join(ROOT, "ros", "src", f"{node}_node.cpp"),
           "-o", str(out), "-L" + LIB, "-lpcp_nodes", "-lpcp", "-Wl,-rpath," + LIB]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-4000:]


def _scene_files(tmp_path):
    sys.path.insert(0, ROOT)
    from pointcloud_processor_amd import synth

    sc = synth.terrain_scene(n_side=200, x0=-2.0, y0=-4.0)
    files = [tmp_path / "area.bin", tmp_path / "terrain.bin", tmp_path / "zx120.bin"]
    np.ascontiguousarray(sc.area, np.float32).tofile(files[0])
    np.ascontiguousarray(sc.terrain, np.float32).tofile(files[1])
    np.ascontiguousarray(synth.aux_cloud(), np.float32).tofile(files[2])
    return [str(f) for f in files]


def _run_driver(exe, files):
    r = subprocess.run([exe] + files, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    steps = {d["step"]: d for d in map(json.loads, r.stdout.splitlines())}
    return steps, r.stderr.splitlines()


def _check_grid_per_area(steps, log):
    """generateExcavationGrid3D ends in publishGridVisualization (virtual_lidar.cpp:286): one
    MarkerArray per non-empty /excavation_area message, none for an empty one (:168), and
    the 3 s tick publishes all three outputs (:545-547)."""
    grid = "/excavation_grid_visualization"
    assert [steps[k][grid] for k in ("area", "empty_area", "area_again", "tick")] == [1, 1, 2, 3]
    assert steps["tick"]["/mobile_lidar_candidate_positions"] == 1
    assert steps["tick"]["/optimal_mobile_lidar_position"] == 1
    gen = [int(m.group(1)) for m in (re.search(r"Generated 3D grid: (\d+) valid cells across 10 "
                                               r"vertical layers", l) for l in log) if m]
    assert len(gen) == 2 and gen[0] == gen[1] > 0
    for k in ("area", "area_again"):   # fresh GridCells: every flag false -> all blue (:936-940)
        g = steps[k]["grid"]
        assert g["cubes"] == gen[0] and g["blue"] == gen[0] and g["malformed"] == 0
        assert g["scale"] == pytest.approx(0.1 * 0.6)
    # after the tick the colours are the dual table's classification of the same flags (:487-501)
    g = steps["tick"]["grid"]
    table = log[log.index("INFO Color-based Area Analysis:"):]
    for colour, label in (("green", "Green (Observable)"), ("red", "Red (Occluded)"),
                          ("blue", "Blue (Out of range)"), ("yellow", "Yellow (Out of FOV)")):
        line = next(l for l in table if label in l)
        assert int(re.search(label.replace("(", r"\(").replace(")", r"\)") + r": (\d+)",
                             line).group(1)) == g[colour]
    assert g["cubes"] == gen[0] and g["malformed"] == 0
    # the evaluateZX120Only and dual tables, line for line (:419-451, :522-543)
    for heading in ("INFO ZX120 LiDAR Only Evaluation", "INFO Debug Info:",
                    "INFO Color-based Area Analysis (ZX120 only):",
                    "INFO Dual LiDAR Configuration (ZX120 + Mobile)", "INFO   ---"):
        assert heading in log
    assert any(l.startswith("INFO   ZX120 point cloud size: ") for l in log)


def test_virtual_lidar_shell_publishes_grid_per_area_mock(tmp_path):
    """CPU: the shell + the real node core over the C-ABI test double."""
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = tmp_path / "shell_driver_mock"
    stub = os.path.join(ROOT, "tests", "ros_stub")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-Werror", "-I" + stub,
           "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "pointcloud_processor_amd", "csrc", "host"),
           "-I" + os.path.join(ROOT, "ros", "src"),
           os.path.join(stub, "shell_driver.cpp"),
           os.path.join(ROOT, "pointcloud_processor_amd", "csrc", "host", "pcp_nodes.cpp"),
           os.path.join(stub, "mock_pcp.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    steps, log = _run_driver(str(exe), _scene_files(tmp_path))
    _check_grid_per_area(steps, log)
    # the double's canned flags: cell i in state i % 4 (blue, yellow, red, green)
    g = steps["tick"]["grid"]
    n = g["cubes"]
    assert (g["blue"], g["yellow"], g["red"], g["green"]) == (
        (n + 3) // 4, (n + 2) // 4, (n + 1) // 4, n // 4)


@pytest.mark.gpu
def test_virtual_lidar_shell_publishes_grid_per_area_gpu(tmp_path):
    """GPU: the same driver over the real libpcp (built by __graft_entry__.build())."""
    exe = os.path.join(LIB, "shell_driver")
    if not os.path.exists(exe):
        pytest.fail("shell_driver not built (run __graft_entry__.build())")
    steps, log = _run_driver(exe, _scene_files(tmp_path))
    _check_grid_per_area(steps, log)
    assert not any(l.startswith("ERROR") for l in log), log
