"""Diagnostic: per-tile phase times of k_radix_scatter / k_seg_centroid from s_memrealtime
stamps (100 MHz), diagnostic build `make -C pointcloud_processor_amd/csrc stamps`.
One 5M-pt C3 cloud through pcp_crop_voxel; the stamps are those of the last launch."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: F401,E402  (torch's HIP runtime first, as bench.py does)

from pointcloud_processor_amd import _abi, synth  # noqa: E402

DIAG = ROOT / "pointcloud_processor_amd" / "_lib" / "diag" / "libpcp.so"
ctx = _abi.Context(0, lib_path=DIAG)
lib = ctx.lib
lib.pcp_diag_filter_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
cloud = synth.lidar_cloud(5_000_000, sensor_height=2.0, seed=1)
box = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])
for _ in range(3):
    out, ncrop = ctx.crop_voxel(cloud, box, 0.05)
print("cropped", ncrop, "voxels", out.shape[0])
names = {0: ["load", "rank", "prefix", "layout", "store"],
         1: ["stage+prefix", "heads", "hpos", "setup", "sums+store"]}
for which in (0, 1):
    st = np.zeros(4096 * 8, np.uint64)
    lib.pcp_diag_filter_stamps(ctx.h, which, st.ctypes.data, st.size)
    st = st.reshape(4096, 8).astype(np.int64)
    act = st[:, 0] > 0
    st = st[act]
    if not len(st):
        continue
    d = np.diff(st[:, :6], axis=1) * 10 / 1000.0   # us
    t0 = st[:, 0].min()
    print(["k_radix_scatter", "k_seg_centroid"][which], f"tiles {len(st)}",
          f"span {(st[:, 5].max() - t0) * 10 / 1000:.2f} us",
          f"start spread {(st[:, 0].max() - t0) * 10 / 1000:.2f} us")
    for k, nm in enumerate(names[which]):
        print(f"   {nm:14s} mean {d[:, k].mean():7.2f}  p50 {np.median(d[:, k]):7.2f}  max {d[:, k].max():7.2f} us")
