"""Diagnostic: phase times of k_nb_lists<false> / k_nb_sums<false> (the area normals' sorted
neighbour lists and ordered sums) from s_memrealtime stamps (100 MHz), diagnostic build
`make -C pointcloud_processor_amd/csrc stamps`.  The area is C1's (bench._c1_scans through the
GPU chain: crop + voxel, merge, carve); the stamps are those of the last of 3 setups."""
import ctypes as C
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from pointcloud_processor_amd import _abi  # noqa: E402

DIAG = os.environ.get("PCP_DIAG_LIB", str(ROOT / "pointcloud_processor_amd" / "_lib" / "diag" /
                                         "libpcp.so"))
ctx = _abi.Context(0, lib_path=DIAG)
lib = ctx.lib
lib.pcp_diag_nb_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
scans = bench._c1_scans()
filtered = [ctx.crop_voxel(sc, bench.C1_BOX, bench.C1_LEAF)[0] for sc in scans]
merged = ctx.transform_concat(filtered, bench.C1_TFS, [(255, 0, 0), (0, 0, 255)])
terr, area, _ = ctx.excavate(merged, bench.C1_ZX_BASE)
for _ in range(3):
    ctx.set_excavation_area(area, 0.1, 10)
print("area points", area.shape[0])
B, Q, PH = 2048, 4, 8
for which, names in ((0, ["clear", "stencil", "scan", "group", "rank+write"]), (1, ["sums"])):
    st = np.zeros(B * Q * PH, np.uint64)
    lib.pcp_diag_nb_stamps(ctx.h, which, st.ctypes.data, st.size)
    st = st.reshape(B, Q, PH).astype(np.int64)
    t0 = st[:, :, 0][st[:, :, 0] > 0].min()
    rows = st.reshape(-1, PH)
    ok = rows[:, 0] > 0
    rows = rows[ok]
    nph = len(names)
    d = np.diff(rows[:, :nph + 1], axis=1) / 100.0    # us
    print(f"{['k_nb_lists<false>', 'k_nb_sums<false>'][which]}: {rows.shape[0]} (block, round)s, "
          f"span {(rows[:, nph].max() - t0) / 100:.1f} us")
    for k, nm in enumerate(names):
        print(f"   {nm:12s} mean {d[:, k].mean():7.2f}  p50 {np.median(d[:, k]):7.2f}  max {d[:, k].max():7.2f} us")
    m = rows[:, 7]
    per = d.sum(1)
    print(f"   length mean {m.mean():.0f} max {m.max()}; us per 1k entries {1e3 * per.sum() / max(m.sum(), 1):.2f}")
    starts = (rows[:, 0] - t0) / 100
    print(f"   round starts: " + ", ".join(f"r{q}: {np.median((st[:, q, 0][st[:, q, 0] > 0] - t0) / 100):.1f}"
                                          for q in range(Q) if (st[:, q, 0] > 0).any()))
