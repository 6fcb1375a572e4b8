"""Source stamps of the kernels a profile was measured on (bench.py, tools/pmc_traffic.py).

A committed PMC traffic figure (profiles/r0*_pmc_traffic.json) holds the stamp of the sources its
kernel was built from; bench.py compares it with the stamp of the tree it runs and reports the
traffic as stale (no hbm_frac) when they differ, instead of silently quoting bytes of an older
kernel."""
from __future__ import annotations

import hashlib
import os
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "pointcloud_processor_amd" / "csrc"
_COMMON = ["pcp_internal.hpp", "Makefile", "../../include/pcp_abi.h"]
# the sources each profiled workload's kernels are compiled from
WORKLOAD_SOURCES = {
    "fan": ["pcp_vlidar.hip", "pcp_fine.hip", "pcp_index.hip", "pcp_stencil.hpp",
            "pcp_grid.hpp"] + _COMMON,
    "filter": ["pcp_filter.hip", "pcp_rigid.hpp"] + _COMMON,
    # reference mode (k_score_cells: the same march over the same terrain copy)
    "cells": ["pcp_vlidar.hip", "pcp_fine.hip", "pcp_index.hip", "pcp_stencil.hpp",
              "pcp_grid.hpp"] + _COMMON,
}


def workload_stamp(key: str) -> str:
    """sha256 (16 hex) of the workload's source files and the EXTRA build flags."""
    h = hashlib.sha256(os.environ.get("EXTRA", "").encode())
    for name in WORKLOAD_SOURCES[key]:
        f = (CSRC / name).resolve()
        h.update(name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]
