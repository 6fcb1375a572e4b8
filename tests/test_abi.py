"""The C ABI boundary (include/pcp_abi.h) without a GPU: libpcp.so loads, exports every
declared entry point, the binding covers them, host-only helpers work, and compute entry
points fail loudly (no CPU fallback) when no device is present."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from pointcloud_processor_amd import _abi

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "pcp_abi.h"


def declared_symbols():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(pcp_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("pcp_crop_box", "pcp_voxel_grid", "pcp_crop_voxel", "pcp_transform_concat",
              "pcp_filter_merge", "pcp_set_terrain", "pcp_set_aux_cloud", "pcp_set_cells",
              "pcp_generate_candidates", "pcp_score_poses", "pcp_raycast_fan"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    assert _abi.LIB_PATH.exists(), "build libpcp.so first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], check=True,
                         capture_output=True, text=True).stdout
    exported = set(re.findall(r"\sT\s(pcp_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    lib = _abi.load_library()
    for s in declared_symbols():
        assert hasattr(lib, s)


def test_binding_covers_the_header():
    assert sorted(_abi.ABI_SYMBOLS) == declared_symbols()


def test_host_only_entry_points():
    lib = _abi.load_library()
    assert lib.pcp_abi_version() == 2
    s = _abi.step_table(15.0 - 0.08)
    ref, x = [], 0.5
    while x < 14.92:
        ref.append(x)
        x += 0.3
    assert np.array_equal(s, ref)
    assert lib.pcp_kernel_name(0) == b"raycast_fan"
    assert lib.pcp_kernel_name(99) == b"unknown"
    assert lib.pcp_last_error(None) == b"null context"


def test_null_and_invalid_arguments_are_rejected():
    lib = _abi.load_library()
    assert lib.pcp_create(0, None) == _abi.PCP_E_INVALID
    assert lib.pcp_synchronize(None) == _abi.PCP_E_INVALID
    assert lib.pcp_raycast_fan(None, None, 0, None, None, None, None, None) == _abi.PCP_E_INVALID
    assert lib.pcp_step_table(1.0, None, 5, None) == _abi.PCP_E_INVALID


def test_no_cpu_fallback_without_gpu():
    n = C.c_int(-1)
    _abi.load_library().pcp_device_count(C.byref(n))
    if n.value > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_abi.PcpError):
        _abi.Context(0)


def _assert_opt_rocm_runtime():
    import sys

    info = _abi.runtime_info()
    print("libpcp runtime:", info)
    assert info["hip_path"] and info["hip_path"].startswith("/opt/rocm"), info
    assert info["rccl_path"] and info["rccl_path"].startswith("/opt/rocm"), info
    assert info["hip_runtime_version"] >= 70200000, info   # the image's ROCm 7.2
    assert "torch" not in sys.modules   # torch's bundled copies never joined this process


def test_libpcp_runs_on_opt_rocm_runtime():
    """libpcp is loaded before anything imports torch (conftest.py), so its NEEDED
    libamdhip64.so.7 / librccl.so.1 are /opt/rocm's, not a PyTorch wheel's (pcp_get_runtime_info:
    versions + dladdr paths; no device call)."""
    _assert_opt_rocm_runtime()


@pytest.mark.gpu
def test_libpcp_runs_on_opt_rocm_runtime_gpu(gpu):
    """The same on the GPU box, with a context created (the runtime initialised)."""
    _assert_opt_rocm_runtime()
