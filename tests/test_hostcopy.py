"""pcp_hostcopy.hip's split copy (the C5 messages into and out of pinned memory) on the CPU:
built host-only with hipcc together with tests/native/hostcopy_check.cpp, no GPU call."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "pointcloud_processor_amd" / "csrc"


def test_split_host_copy(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("no hipcc")
    exe = tmp_path / "hostcopy_check"
    subprocess.run([hipcc, "-O2", "-std=c++17", f"-I{ROOT / 'include'}", f"-I{CSRC}",
                    str(ROOT / "tests" / "native" / "hostcopy_check.cpp"),
                    str(CSRC / "pcp_hostcopy.hip"), "-o", str(exe), "-lpthread"],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.stdout, r.stderr)
