import os
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))

# libpcp before anything can import torch: a PyTorch wheel bundles its own HIP runtime and RCCL
# under the SONAMEs libpcp links, and whichever copy is loaded first serves both.  Loaded here
# (RTLD_GLOBAL), libpcp runs on /opt/rocm's, the runtime it ships with; no test module imports
# torch in this process (torch-side checks run in their own processes).
try:
    from pointcloud_processor_amd import _abi as _pcp_abi

    _pcp_abi.load_library()
except OSError:   # not built yet: the ABI tests say so
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libpcp.so")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def scene():
    from pointcloud_processor_amd import synth

    return synth.terrain_scene()


@pytest.fixture(scope="session")
def small_scene():
    """A 200 x 200 lattice (10 m x 10 m) with the same pit: fast for brute-force checks."""
    from pointcloud_processor_amd import synth

    return synth.terrain_scene(n_side=200, x0=-2.0, y0=-4.0)


@pytest.fixture(scope="session")
def cells(scene):
    from pointcloud_processor_amd import synth

    return synth.excavation_cells(scene.area)


@pytest.fixture(scope="session")
def aux():
    from pointcloud_processor_amd import synth

    return synth.aux_cloud()


@pytest.fixture(scope="session")
def gpu():
    """A libpcp context on cuda:0.  Fails loudly (no fallback) if the library or GPU is absent."""
    from pointcloud_processor_amd import _abi

    ctx = _abi.Context(0)
    yield ctx
    ctx.close()
