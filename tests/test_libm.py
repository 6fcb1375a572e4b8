"""pcp_libm.h -- the GPU's restatement of glibc 2.35's float atan2f / sinf / cosf (the libm calls
of pcl::eigen33's computeRoots, virtual_lidar.cpp:209-234 through pcl::NormalEstimation) --
against the glibc this suite runs on, bit for bit.  The exact PCA normals (tests/
test_gpu_parity.py::test_excavation_area_setup) depend on it: the oracle calls glibc, the GPU
compiles this header.  CPU only."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path_factory.mktemp("libm") / "libm_check"
    # -ffp-contract=off: the header's own rule (every operation rounds on its own)
    subprocess.run([cc, "-O2", "-ffp-contract=off", f"-I{ROOT / 'pointcloud_processor_amd' / 'csrc'}",
                    str(ROOT / "tests" / "libm" / "libm_check.c"), "-o", str(exe), "-lm"],
                   check=True)
    return exe


def test_sincos_atan2_match_glibc(checker):
    """Every 61st float of [0, 1.1] (17.5 M: sinf, cosf) and 4 M atan2f argument pairs (half of
    them arbitrary bit patterns, half computeRoots' magnitudes): zero mismatches.  (The whole
    [0, 1.1] range, 1.07e9 floats, was checked once: zero mismatches, both the FMA and the SSE2
    build of glibc's sinf / cosf.)"""
    r = subprocess.run([str(checker), "61", "4000000"], capture_output=True, text=True,
                       timeout=300, check=True)
    lines = dict((l.split()[0], list(map(int, l.split()[1:]))) for l in r.stdout.splitlines())
    n, ms, mc = lines["sin_cos"]
    assert n > 17_000_000 and ms == 0 and mc == 0, lines
    n_at, ma = lines["atan2"]
    assert n_at == 4_000_000 and ma == 0, lines
