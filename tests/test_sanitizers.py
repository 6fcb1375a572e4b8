"""ASan + UBSan builds of the CPU-side code: the oracle restatement driven by
oracle/oracle_selftest.c (every entry point, NaN / empty / overflow / degenerate inputs, the
restated KdTreeFLANN against the grid scan) and the host-side node code's GPU-free logic
(pointcloud_processor_amd/csrc/host/pcp_nodes_selftest.cpp: the PointCloud2 codec and the
loud no-device failures).  Host code only: GPU sanitizers are not available on this pool."""
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _make(d, target):
    r = subprocess.run(["make", "-s", "-C", str(d), target], capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    return out


def test_oracle_asan_ubsan():
    assert "oracle selftest ok" in _make(ROOT / "oracle", "asan")


def test_host_nodes_asan_ubsan():
    assert (ROOT / "pointcloud_processor_amd" / "_lib" / "libpcp.so").exists(), "build first"
    assert "nodes selftest ok" in _make(ROOT / "pointcloud_processor_amd" / "csrc", "asan")
