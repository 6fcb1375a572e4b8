"""Diagnostic: phase times of the bucket chain's k_bk_group / k_bk_sort blocks from
s_memrealtime stamps (100 MHz), diagnostic build `make -C pointcloud_processor_amd/csrc stamps`.
The C3 frame (2 x 5 M points) through pcp_filter_merge; the stamps are those of the last call."""
import ctypes as C
import math
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from pointcloud_processor_amd import _abi, synth  # noqa: E402

import os  # noqa: E402

DIAG = os.environ.get("PCP_DIAG_LIB", str(ROOT / "pointcloud_processor_amd" / "_lib" / "diag" /
                                         "libpcp.so"))
ctx = _abi.Context(0, lib_path=DIAG)
lib = ctx.lib
lib.pcp_diag_filter_stamps.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
a = synth.lidar_cloud(5_000_000, sensor_height=2.0, seed=1)
b = synth.lidar_cloud(5_000_000, sensor_height=3.5, seed=2)
box = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])
yaw = math.radians(30.0)
tfs = [((8.0, -3.0, 0.0), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))),
       ((0.55, 0.4, 3.5), (0.0, math.sin(0.4363 / 2), 0.0, math.cos(0.4363 / 2)))]
for _ in range(3):
    out, per = ctx.filter_merge([a, b], [box, box], 0.05, tfs, [(255, 0, 0), (0, 0, 255)])
print("voxels", list(per))
names = {0: ["params", "passA", "scan+row", "passB"],
         1: ["rows+scan", "gather+atom", "tabscan", "place", "rank+src", "sums"]}
allst = {}
for which in (0, 1):
    st = np.zeros(4096 * 8, np.uint64)
    lib.pcp_diag_filter_stamps(ctx.h, which, st.ctypes.data, st.size)
    allst[which] = st.reshape(4096, 8).astype(np.int64).copy()
e = allst[0][1024:2048, :3]
e = e[(e[:, 0] > 0) & (e[:, 2] > 0)]
if len(e):
    d = np.diff(e, axis=1) * 10 / 1000.0
    t0 = e[:, 0].min()
    print("k_bk_emit", f"blocks {len(e)}", f"span {(e[:, 2].max() - t0) * 10 / 1000:.2f} us",
          f"start spread {(e[:, 0].max() - t0) * 10 / 1000:.2f} us",
          f"prefix mean {d[:, 0].mean():.2f} max {d[:, 0].max():.2f} us, copy mean {d[:, 1].mean():.2f} max {d[:, 1].max():.2f} us")
# the fused emit (PCP_BK_FUSE=1): phase 7 = after the look-back; rank + look-back = ph7 - ph4
s1 = allst[1]
m = (s1[:, 0] > 0) & (s1[:, 7] > 0)
if m.any():
    lb = (s1[m, 7] - s1[m, 4]) * 10 / 1000.0
    pub = (s1[m, 3] - s1[m, 0]) * 10 / 1000.0
    t0 = s1[m, 0].min()
    print("k_bk_sort fused:", f"blocks {m.sum()}", f"rank+look-back mean {lb.mean():.2f} "
          f"p50 {np.median(lb):.2f} p90 {np.percentile(lb, 90):.2f} max {lb.max():.2f} us",
          f"publish at mean {pub.mean():.2f} us after start",
          f"span {(s1[m, 6].max() - t0) * 10 / 1000:.2f} us")
    idx = np.nonzero(m)[0]
    for lo in range(0, len(idx), max(1, len(idx) // 8)):
        sel = idx[lo:lo + max(1, len(idx) // 8)]
        print(f"  buckets {sel[0]}-{sel[-1]}: start {(s1[sel, 0].mean() - t0) * 10 / 1000:.2f} us, "
              f"look-back {((s1[sel, 7] - s1[sel, 4]) * 10 / 1000).mean():.2f} us")
for which in (0, 1):
    st = np.zeros(4096 * 8, np.uint64)
    lib.pcp_diag_filter_stamps(ctx.h, which, st.ctypes.data, st.size)
    st = st.reshape(4096, 8).astype(np.int64)
    if which == 0:
        st = st[:1024]
    np_ = len(names[which]) + 1
    st = st[(st[:, 0] > 0) & (st[:, np_ - 1] > 0)][:, :np_]
    if not len(st):
        continue
    d = np.diff(st, axis=1) * 10 / 1000.0   # us
    t0 = st[:, 0].min()
    print(["k_bk_group", "k_bk_sort"][which], f"blocks {len(st)}",
          f"span {(st[:, -1].max() - t0) * 10 / 1000:.2f} us",
          f"start spread {(st[:, 0].max() - t0) * 10 / 1000:.2f} us",
          f"block life mean {(st[:, -1] - st[:, 0]).mean() * 10 / 1000:.2f} us")
    for k, nm in enumerate(names[which]):
        print(f"   {nm:14s} mean {d[:, k].mean():7.2f}  p50 {np.median(d[:, k]):7.2f}  max {d[:, k].max():7.2f} us")
    if which == 1:   # start times in block order: how the rounds progress
        s0 = (st[:, 0] - t0) * 10 / 1000.0
        e0 = (st[:, -1] - t0) * 10 / 1000.0
        for q in (0, 256, 512, 768, 1024, 1536, 2048, len(st) - 1):
            if q < len(st):
                print(f"   block {q:5d}: start {s0[q]:7.2f} end {e0[q]:7.2f} us")
