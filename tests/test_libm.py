"""pcp_libm.h -- the GPU's restatement of glibc 2.35's float atan2f / sinf / cosf (the libm calls
of pcl::eigen33's computeRoots, virtual_lidar.cpp:209-234 through pcl::NormalEstimation) --
against the glibc this suite runs on, bit for bit.  The exact PCA normals (tests/
test_gpu_parity.py::test_excavation_area_setup) depend on it: the oracle calls glibc, the GPU
compiles this header.  CPU only -- and, marked gpu as well, on the GPU box's own host (the EPYC
whose glibc the oracle runs on there), so the ifunc glibc picks is observed on both machines."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

# each test runs in both suites: here (-m "not gpu") and on the GPU box's host (-m gpu)
BOTH = [pytest.param("host"), pytest.param("gpu_box_host", marks=pytest.mark.gpu)]


def _build(out: Path, fma: int) -> Path:
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    # -ffp-contract=off: the header's own rule (every operation rounds on its own)
    subprocess.run([cc, "-O2", "-ffp-contract=off", f"-DPCP_LIBM_SINCOS_FMA={fma}",
                    f"-I{ROOT / 'pointcloud_processor_amd' / 'csrc'}",
                    str(ROOT / "tests" / "libm" / "libm_check.c"), "-o", str(out), "-lm"],
                   check=True)
    return out


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    return _build(tmp_path_factory.mktemp("libm") / "libm_check", 1)


def _run(exe: Path, stride: int, n_atan: int) -> dict:
    r = subprocess.run([str(exe), str(stride), str(n_atan)], capture_output=True, text=True,
                       timeout=300, check=True)
    return dict((l.split()[0], list(map(int, l.split()[1:]))) for l in r.stdout.splitlines())


@pytest.mark.parametrize("where", BOTH)
def test_sincos_atan2_match_glibc(checker, where):
    """Every 61st float of [0, 1.1] (17.5 M: sinf, cosf) and 4 M atan2f argument pairs (half of
    them arbitrary bit patterns, half computeRoots' magnitudes): zero mismatches.  (The whole
    [0, 1.1] range, 1.07e9 floats, was checked once: zero mismatches, both the FMA and the SSE2
    build of glibc's sinf / cosf.)"""
    lines = _run(checker, 61, 4_000_000)
    n, ms, mc = lines["sin_cos"]
    assert n > 17_000_000 and ms == 0 and mc == 0, lines
    n_at, ma = lines["atan2"]
    assert n_at == 4_000_000 and ma == 0, lines


@pytest.mark.parametrize("where", BOTH)
def test_sincos_ifunc_does_not_matter(tmp_path, where):
    """The restatement's one assumption about the reference's host -- that x86-64 glibc
    dispatches sinf / cosf to their FMA build (PCP_LIBM_SINCOS_FMA=1, the default) -- does not
    decide any result: over the angles computeRoots passes them ([0, pi/3] in [0, 1.1]) the SSE2
    restatement (PCP_LIBM_SINCOS_FMA=0) matches this host's glibc bit for bit as well, so the
    normals are the same whichever build a host's glibc picks.  Observed here and on the GPU
    box's host."""
    lines = _run(_build(tmp_path / "libm_check_sse2", 0), 61, 1000)
    n, ms, mc = lines["sin_cos"]
    assert n > 17_000_000 and ms == 0 and mc == 0, lines
