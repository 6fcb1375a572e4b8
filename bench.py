#!/usr/bin/env python3
"""Benchmark of the virtual-LiDAR pose search (BASELINE.json metric, configs[1]).

A step = one pass of the hot path over one batch: the candidate poses of this rank (256 per
GPU: BASELINE configs[1] at N=1; --poses-per-gpu 512 on 8 GPUs = configs[3]'s 4096) each cast the dense
1024 x 256 azimuth x elevation fan against the 1M-point excavation terrain with the
reference's march rule (virtual_lidar.cpp:765-797), plus ONE collective: all-reduce(MIN)
of the per-pose blocked-ray counts (RCCL over xGMI when N > 1), then the argmin.

value = ray-hit tests/s: sample queries the reference would execute (samples up to and
including the first hit, else all), summed over all ranks, / max-over-ranks wall time.
Inputs (terrain index, direction tables, poses) are resident in HBM before timing starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode fan|filter|cells]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "ray-hit tests/sec + candidate poses/sec (whole node), 1M-pt terrain"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8 TB/s spec


def _dist_init(n_gpus: int):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # one process per GPU over RCCL; PCP_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs
        backend = os.environ.get("PCP_DIST_BACKEND",
                                 "nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return torch, (dist if world > 1 else None), world, rank, local


def _poses_for(ctx, grid_bbox, zx, total: int):
    """generateCandidatePositions with num_candidates grown until >= total survive."""
    from pointcloud_processor_amd import _abi

    nc = max(total, 100)
    while True:
        p = _abi.default_vl_params(num_candidates=nc)
        poses = ctx.generate_candidates(grid_bbox, p, zx)
        if poses.shape[0] >= total:
            return poses[:total], nc
        nc = int(nc * 1.3) + 16


def _grid_bbox(area, res=0.1):
    import numpy as np

    p = area[:, :3].astype(np.float64)
    return np.array([p[:, 0].min() - res, p[:, 0].max() + res, p[:, 1].min() - res,
                     p[:, 1].max() + res, p[:, 2].min() - res, p[:, 2].max() + res])


def _traffic_from_profiles(workload_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_traffic.py), or
    None when no measurement for this workload is committed."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text()).get(workload_key)
        return None if d is None else float(d["bytes_per_launch"])
    except Exception:
        return None


def _gbs(nbytes, seconds):
    """Bytes per launch / launch time in GB/s (None when either is unknown)."""
    return nbytes / seconds / 1e9 if nbytes and seconds else None


def _host_cpu():
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    share = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"model": model, "nproc": os.cpu_count(), "affinity": share}


def cpu_baseline_fan(terrain, poses, fan, budget_s: float, threads: int = 1):
    """The oracle (CPU restatement) on a bounded sample: the first k poses of this workload,
    whole fans, until ~budget_s elapsed.  threads = 1 is the reference's single-threaded
    executor; threads > 1 is the OpenMP variant SURVEY 8d asks for beside it."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    pyoracle.set_threads(threads)
    T = pyoracle.Cloud(terrain)
    units = 0
    k = 0
    t0 = time.perf_counter()
    while k < len(poses) and time.perf_counter() - t0 < budget_s:
        _, u, _ = pyoracle.raycast_fan(T, poses[k:k + 1], fan.n_az, fan.n_el, fan.el_min,
                                       fan.el_max, fan.max_distance, want_first_hit=False)
        units += int(u.sum())
        k += 1
    dt = time.perf_counter() - t0
    pyoracle.set_threads(1)
    return {"value": units / dt, "unit": "ray-hit tests/s", "cores": threads, "kind": "port",
            "sample": f"{k} of {len(poses)} poses x full {fan.n_az}x{fan.n_el} fan, "
                      f"{units} sample queries in {dt:.1f} s (oracle/pcp_oracle.c, "
                      f"{threads} thread{'s' if threads > 1 else ''})"}


def run_fan(args, torch, dist, world, rank, local):
    import numpy as np

    from pointcloud_processor_amd import _abi, synth

    ctx = _abi.Context(local)
    scene = synth.terrain_scene()
    ctx.set_terrain(scene.terrain, point_step=32)
    bbox = _grid_bbox(scene.area)
    from pointcloud_processor_amd import dist as pd

    P_total = args.poses_per_gpu * world
    poses_all, nc = _poses_for(ctx, bbox, scene.zx120_pose5, P_total)
    lo, hi = pd.shard(P_total, world, rank)
    poses = np.ascontiguousarray(poses_all[lo:hi])
    fan = _abi.fan_params(n_az=args.n_az, n_el=args.n_el)
    on_gpu = torch.cuda.is_available()
    dev = torch.device("cuda", local) if on_gpu else torch.device("cpu")

    def step():
        blocked, units, _, _ = ctx.raycast_fan(poses, fan)
        keys, best = pd.reduce_fan(blocked, lo, hi, P_total, dist, dev)   # the one collective
        return int(units.sum()), best, keys

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        if on_gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    ctx.profile(True)
    ctx.profile_reset()
    barrier_sync()
    t0 = time.perf_counter()
    units_local = 0
    best = -1
    for _ in range(args.steps):
        u, best, keys = step()
        units_local += u
    barrier_sync()
    dt = time.perf_counter() - t0
    ctx.profile(False)
    k_ms, k_n = ctx.profile_get("raycast_fan")
    # max-over-ranks time, sum-over-ranks units
    t = torch.tensor([dt], dtype=torch.float64)
    u = torch.tensor([units_local], dtype=torch.float64)
    if dist is not None:
        t = t.to(dev); u = u.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
    dt_max, units_all = float(t.item()), float(u.item())
    # diagnostic (untimed): algorithmic bytes of one launch
    st = ctx.raycast_fan_stats(poses, fan)
    units_per_launch = units_local / max(args.steps, 1)
    alg_bytes = 64.0 * units_per_launch + 12.0 * st["point_tests"]
    avg_kernel_s = (k_ms / max(k_n, 1)) * 1e-3
    achieved = alg_bytes / avg_kernel_s / 1e9 if avg_kernel_s > 0 else None
    out = {
        "metric": METRIC,
        "value": units_all / dt_max,
        "unit": "ray-hit tests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max / max(args.steps, 1) * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64 march / f32 point test",
        "data": "synthetic (seeded T1M L-pit terrain, reference candidate lattice)",
        "config": {"workload": "C2: 1M-pt L-shape excavation terrain, 1024x256 ray fan, "
                               f"{args.poses_per_gpu} candidate poses per GPU",
                   "terrain_points": int(scene.terrain.shape[0]),
                   "poses_total": P_total, "fan": [args.n_az, args.n_el],
                   "num_candidates_lattice": nc, "parallelism": f"pose-shard x{world}"},
        "poses_per_s": P_total * args.steps / dt_max,
        "best_pose": best,
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": _traffic_from_profiles("fan"),
            # the survey's model charges 64 B to every sample query the reference would make;
            # the kernel skips ~95 % of them exactly, so frac > 1.  What it really moves:
            "traffic_gbs": _gbs(_traffic_from_profiles("fan"), avg_kernel_s),
            "limiter": "vector-memory address/data path of dependent L2 gathers (TA 83 %, TD "
                       "93 % busy, profiles/r01_fan_pmc.txt), not HBM",
            "kernel": "k_raycast_fan<0, 64, true>", "avg_kernel_ms": avg_kernel_s * 1e3,
            "alg_bytes_per_launch": alg_bytes,
            "model": "64 B/sample query + 12 B/point test (SURVEY 8d)",
            "diag": st,
        },
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_fan(scene.terrain, poses, fan, args.cpu_seconds)
        host = _host_cpu()
        mt = max(1, min(16, host["affinity"] or 1))     # the box's CPU share is 16
        out["cpu_baseline_mt"] = cpu_baseline_fan(scene.terrain, poses, fan,
                                                  args.cpu_seconds / 2, threads=mt)
        out["cpu_baseline_mt"]["host"] = host
    ctx.close()
    return out


def _pcie_inclusive(ctx, clouds, box, tfs, n_in, cap, reps=5):
    """Host-buffer filter_merge (the PointCloud2 boundary: H2D of the raw clouds, the same
    pipeline, D2H of the merged cloud), pageable numpy buffers vs the same buffers pinned in
    place with pcp_host_register.  Reported beside `value`, never as it."""
    import numpy as np

    rgbs = [(255, 0, 0), (0, 0, 255)]
    out = np.empty((cap, 8), np.float32)
    res = {"unit": "input points/s", "reps": reps,
           "h2d_bytes": int(sum(c.nbytes for c in clouds))}

    def timed():
        ctx.filter_merge(clouds, [box, box], 0.05, tfs, rgbs, out=out)   # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            got, _ = ctx.filter_merge(clouds, [box, box], 0.05, tfs, rgbs, out=out)
        dt = (time.perf_counter() - t0) / reps
        return dt, got.shape[0]

    dt, n_out = timed()
    res["pageable_ms"] = dt * 1e3
    res["pageable"] = n_in / dt
    res["d2h_bytes"] = int(n_out * 32)
    pinned = []
    try:
        for a in clouds + [out]:
            ctx.host_register(a)
            pinned.append(a)
        dt, _ = timed()
        res["pinned_ms"] = dt * 1e3
        res["pinned"] = n_in / dt
        res["pinned_link_gbs"] = (res["h2d_bytes"] + res["d2h_bytes"]) / dt / 1e9
    except RuntimeError as e:           # pinning refused (e.g. locked-memory limit)
        res["pinned_error"] = str(e)
    finally:
        for a in pinned:
            ctx.host_unregister(a)
    return res


def run_filter(args, torch, dist, world, rank, local):
    """C3: crop + voxel(0.05) + transform on a 10M-pt dual-LiDAR frame, inputs in HBM."""
    import math

    import numpy as np

    from pointcloud_processor_amd import _abi, synth

    ctx = _abi.Context(local)
    n_each = args.filter_points // 2
    clouds = [synth.lidar_cloud(n_each, sensor_height=2.0, seed=1 + 2 * rank),
              synth.lidar_cloud(n_each, sensor_height=3.5, seed=2 + 2 * rank)]
    dptr = []
    views = []
    for c in clouds:
        p = ctx.dev_alloc(c.nbytes)
        ctx.h2d(p, c)
        dptr.append(p)
        views.append(_abi.CloudView(p, c.shape[0], 16, 0, 4, 8))
    box = [0.0, 15.0, -10.0, 10.0, -1.5, 10.0]
    yaw = math.radians(30.0)
    tfs = [((8.0, -3.0, 0.0), (0.0, 0.0, math.sin(yaw / 2), math.cos(yaw / 2))),
           ((0.55, 0.4, 3.5), (0.0, math.sin(0.4363 / 2), 0.0, math.cos(0.4363 / 2)))]
    cap = sum(c.shape[0] for c in clouds)
    out_d = ctx.dev_alloc(cap * 32)

    def step():
        return ctx.filter_merge_device(views, [box, box], 0.05, tfs, [(255, 0, 0), (0, 0, 255)],
                                       out_d, cap)

    for _ in range(args.warmup):
        n_out, per = step()
    ctx.profile(True)
    ctx.profile_reset()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        n_out, per = step()
    dt = time.perf_counter() - t0
    ctx.profile(False)
    g_ms, g_n = ctx.profile_get("filter_merge")
    n_in = sum(c.shape[0] for c in clouds)
    step_dev_ms = g_ms / max(g_n, 1)
    # per-stage breakdown from one eager (non-graph) context, untimed
    os.environ["PCP_NO_GRAPHS"] = "1"
    ectx = _abi.Context(local)
    os.environ.pop("PCP_NO_GRAPHS")
    ectx.profile(True)
    for _ in range(3):
        ectx.filter_merge_device(views, [box, box], 0.05, tfs, [(255, 0, 0), (0, 0, 255)], out_d,
                                 cap)
    stages = {k: ectx.profile_get(k)[0] / 3 for k in ("crop", "voxel", "transform", "filter_merge")}
    ectx.close()
    pcie = None if args.no_pcie else _pcie_inclusive(ctx, clouds, box, tfs, n_in, cap)
    alg = 12.0 * n_in + 16.0 * n_out
    res = {
        "metric": "crop+voxel+transform points/s (C3)", "value": n_in * args.steps / dt,
        "unit": "input points/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / max(args.steps, 1) * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic 2 x LiDAR-like clouds, point_step 16, resident in HBM",
        "config": {"workload": f"C3: crop+voxel(0.05)+transform, {n_in} pts", "n_out": n_out,
                   "per_cloud": [int(x) for x in per], "graph": True},
        "roofline": {"bound": "hbm", "achieved": alg / (step_dev_ms * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": alg / (step_dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": _traffic_from_profiles("filter"),
                     "traffic_gbs": _gbs(_traffic_from_profiles("filter"), step_dev_ms * 1e-3),
                     "limiter": "crop streams at ~4.8 TB/s; the voxel stage (sort of the ~1 M "
                                "cropped points) is launch- and latency-bound",
                     "kernel": "filter_merge graph (all stages)", "avg_kernel_ms": step_dev_ms,
                     "eager_stage_ms": stages,
                     "model": "12 B/input point + 16 B/output point (SURVEY 8d)"},
        "pcie_inclusive": pcie,
    }
    for p in dptr + [out_d]:
        ctx.dev_free(p)
    ctx.close()
    return res


def run_cells(args, torch, dist, world, rank, local):
    """Reference-mode scoring (runOptimization) for the same poses: poses/s."""
    import numpy as np

    from pointcloud_processor_amd import _abi, synth

    ctx = _abi.Context(local)
    scene = synth.terrain_scene()
    cells = synth.excavation_cells(scene.area)
    ctx.set_terrain(scene.terrain, point_step=32)
    ctx.set_aux_cloud(synth.aux_cloud(), point_step=32)
    ctx.set_cells(cells.xyz, cells.normals)
    P_total = args.poses_per_gpu * world
    poses_all, nc = _poses_for(ctx, cells.grid_bbox, scene.zx120_pose5, P_total)
    poses = np.ascontiguousarray(poses_all[rank * args.poses_per_gpu:(rank + 1) * args.poses_per_gpu])
    params = _abi.default_vl_params()
    flags = np.zeros(cells.xyz.shape[0], np.uint8)
    for _ in range(args.warmup):
        ctx.score_poses(poses, scene.zx120_pose5, params, flags)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        tot, cov, rep = ctx.score_poses(poses, scene.zx120_pose5, params, flags)
    dt = time.perf_counter() - t0
    ctx.close()
    return {"metric": "candidate poses/sec (reference cell scoring)",
            "value": P_total * args.steps / dt, "unit": "poses/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic", "config": {"workload": f"{P_total} poses x {cells.xyz.shape[0]} cells"},
            "best_pose": int(rep.best_idx)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--mode", choices=["fan", "filter", "cells"], default="fan")
    ap.add_argument("--poses-per-gpu", type=int, default=256)
    ap.add_argument("--n-az", type=int, default=1024)
    ap.add_argument("--n-el", type=int, default=256)
    ap.add_argument("--filter-points", type=int, default=10_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true",
                    help="filter mode: skip the host-buffer (PCIe-inclusive) measurement")
    args = ap.parse_args()
    torch, dist, world, rank, local = _dist_init(args.gpus)
    fn = {"fan": run_fan, "filter": run_filter, "cells": run_cells}[args.mode]
    out = fn(args, torch, dist, world, rank, local)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
