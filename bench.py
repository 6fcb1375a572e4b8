#!/usr/bin/env python3
"""Benchmark of the virtual-LiDAR pose search (BASELINE.json metric, configs[1]).

A step = one pass of the hot path over one batch: the candidate poses of this rank (256 per
GPU: BASELINE configs[1] at N=1, weak-scaled) each cast the dense 1024 x 256 azimuth x elevation fan against the 1M-point excavation terrain with the
reference's march rule (virtual_lidar.cpp:765-797), plus ONE collective: all-reduce(MIN)
of the per-pose blocked-ray counts (RCCL over xGMI when N > 1), then the argmin.

value = ray-hit tests/s: sample queries the reference would execute (samples up to and
including the first hit, else all), summed over all ranks, / max-over-ranks wall time.
Inputs (terrain index, direction tables, poses) are resident in HBM before timing starts.
The same line carries the rest of the metric ("+ candidate poses/sec (whole node)"):
poses_per_s_reference_mode (runOptimization over the excavation cells, virtual_lidar.cpp:
454-548) and c3 (crop + voxel + transform frame, BASELINE configs[2]), each its own timed loop
of K steps, and CPU baselines (the oracle restatement, 1 thread and the host's CPU share) for
all three on rank 0 at N = 1.  With N > 1 the line also carries c4 (BASELINE configs[3]: 4096
poses strong-scaled over the N ranks, oracle-checked on a sample); at N = 1 it carries c1 and
c5 (configs[0] / configs[4]: the per-frame chain through the C++ node cores).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode all|fan|filter|cells|c1|c4|c5]

--gpus N without WORLD_SIZE starts N ranks itself (one process per GPU).  The rank processes
never import torch (their control plane is hostgroup.py's helper), so libpcp runs on the HIP
runtime and RCCL of /opt/rocm (the line's "runtime").
"""
from __future__ import annotations

import argparse
import gc
import json
import math
import os
import sys
import time
from pathlib import Path

import numpy as np

# waits poll the completion signals instead of sleeping on an interrupt (the host-bound chains'
# synchronisations return sooner, profiles/r05_c5_wait_ab.log); set before libpcp's first HIP
# call, inherited by the ranks and the C5 replay.  PCP_HSA_POLL=0: the runtime's default
if os.environ.get("PCP_HSA_POLL", "1") != "0":
    os.environ.setdefault("HSA_ENABLE_INTERRUPT", "0")

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "ray-hit tests/sec + candidate poses/sec (whole node), 1M-pt terrain"
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: 8 TB/s spec


def _self_launch(n: int) -> int:
    """--gpus N without a launcher: start N ranks of this script (one process per GPU, as
    torch.distributed.run would), before this process touches the GPU.  Rank 0 prints the
    JSON line; the exit code is the worst rank's."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # own process group: a rank's control-plane helper (hostgroup.py) goes with it
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] +
                                      sys.argv[1:], env=env, start_new_session=True))
    rc = 0
    try:
        # any rank may die first: poll them all, and a non-zero exit ends the others (they
        # would wait in a collective for the dead rank until the backend's timeout)
        live = list(procs)
        while live and not rc:
            for p in list(live):
                code = p.poll()
                if code is not None:
                    live.remove(p)
                    rc = max(rc, code if code >= 0 else 128 - code)
            if live and not rc:
                time.sleep(0.05)
    finally:
        import signal

        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGKILL)   # the rank and its helper, if still there
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()
    return rc


def _dist_init(n_gpus: int):
    """The host-side control plane (barriers, the max-over-ranks timing, the RCCL id hand-off):
    a hostgroup.HostGroup, i.e. torch.distributed over gloo in a helper child process, so that
    THIS process never imports torch and libpcp runs on the HIP runtime and RCCL its RUNPATH
    names (/opt/rocm/lib) -- a PyTorch wheel bundles its own copies under the same SONAMEs
    (pcp_get_runtime_info reports which ones ran: the line's "runtime").  The data-path
    collective (`backend`): "rccl" = libpcp's own RCCL communicator (pcp_comm_init_rank), one
    process per GPU; "gloo" = a rehearsal with more ranks than GPUs (ranks share devices, the
    keys go through the host group)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}")
    # libpcp first (RTLD_GLOBAL): its NEEDED libamdhip64.so.7 / librccl.so.1 resolve to /opt/rocm
    try:
        from pointcloud_processor_amd import _abi

        _abi.load_library()
        ndev = _abi.device_count()
    except OSError:          # no library (the CPU launch check)
        ndev = 0
    backend = None
    group = None
    # PCP_DIST_FORCE=1: the distributed path at one rank too (the host group, libpcp's RCCL
    # communicator, the one-collective queries, c4) -- a hardware check of the SCALE path's code
    # on a one-GPU box (profiles/r06_bench_rccl_n1.json)
    if world > 1 or os.environ.get("PCP_DIST_FORCE") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
        backend = os.environ.get("PCP_DIST_BACKEND", "rccl" if ndev >= world else "gloo")
        backend = "rccl" if backend == "nccl" else backend
        if ndev:
            local = local % ndev
        from pointcloud_processor_amd.hostgroup import HostGroup

        group = HostGroup()
    return group, world, rank, local, backend


def _runtime():
    """pcp_get_runtime_info: the HIP runtime and RCCL libpcp ran on in this process."""
    try:
        from pointcloud_processor_amd import _abi

        return _abi.runtime_info()
    except OSError:
        return None


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


TRAFFIC_FILES = ("r06_pmc_traffic.json", "r05_pmc_traffic.json", "r04_pmc_traffic.json",
                 "r03_pmc_traffic.json", "pmc_traffic.json")


def _traffic_from_profiles(workload_key: str):
    """HBM-side bytes per launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    (tools/pmc_traffic.py: fetch_factor x FETCH_SIZE + WRITE_SIZE) -> (bytes, info).  The newest
    file holding the workload decides; its source stamp must equal the stamp of the kernels this
    tree builds (pointcloud_processor_amd/_stamps.py), else the bytes are of another kernel:
    bytes None, info["traffic_stale"] True.  (None, None) when nothing is committed."""
    from pointcloud_processor_amd._stamps import workload_stamp

    for name in TRAFFIC_FILES:
        f = ROOT / "profiles" / name
        if not f.exists():
            continue
        try:
            d = json.loads(f.read_text()).get(workload_key)
        except ValueError:
            continue
        if d is None:
            continue
        info = {"traffic_source": f"profiles/{name}",
                "traffic_stamp": d.get("source_stamp"),
                "tree_stamp": workload_stamp(workload_key),
                "fetch_factor": d.get("fetch_factor", 2.0),
                "fetch_factor_source": d.get("fetch_factor_source",
                                             "x2 (guide, 16-B streaming reads)"),
                "traffic_raw": d.get("bytes_per_launch_raw")}
        info["traffic_stale"] = info["traffic_stamp"] != info["tree_stamp"]
        return (None if info["traffic_stale"] else float(d["bytes_per_launch"])), info
    return None, None


def _gbs(nbytes, seconds):
    """Bytes per launch / launch time in GB/s (None when either is unknown)."""
    return nbytes / seconds / 1e9 if nbytes and seconds else None


def _host_cpu():
    """The host's CPU share: affinity list, cgroup quota, and the threads the MT baselines
    use (min of the two: threads beyond the quota only time-slice)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff,
            "cgroup_quota_cores": quota, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"),
            "threads_used": threads}


def _ulps(a, b) -> np.ndarray:
    """Units in the last place between two float64 arrays (0: the same bits; +-0 equal)."""
    def key(x):
        u = np.ascontiguousarray(np.asarray(x, np.float64)).ravel().view(np.int64)
        return np.array([int(v) if v >= 0 else -(2**63) - int(v) for v in u], dtype=object)
    return np.abs(key(a) - key(b)).astype(np.float64)


def _totals_bar(got, ref) -> dict:
    """tests/parity.py's bar for the per-pose totals: <= 2 ulps each, at most max(2, 5 %) not
    bit-identical (glibc's acos / sin in the oracle, correctly rounded ones on the device)."""
    got, ref = np.asarray(got, np.float64).ravel(), np.asarray(ref, np.float64).ravel()
    if got.shape != ref.shape:
        return {"ok": False, "shape": [got.size, ref.size]}
    d = _ulps(got, ref) if got.size else np.zeros(0)
    n_diff = int((d != 0).sum())
    return {"ok": bool(d.max(initial=0) <= 2 and n_diff <= max(2, math.ceil(0.05 * got.size))),
            "max_ulps": float(d.max(initial=0)), "differ": n_diff, "n": int(got.size)}


def _oracle():
    sys.path.insert(0, str(ROOT / "oracle"))
    import pyoracle

    return pyoracle


def cpu_baseline_fan(terrain, poses, fan, budget_s: float, threads: int = 1,
                     kdtree: bool = False):
    """The oracle (CPU restatement) on a bounded sample: the first k poses of this workload,
    whole fans, until ~budget_s elapsed.  threads = 1 is the reference's single-threaded
    executor; threads > 1 is the OpenMP variant SURVEY 8d asks for beside it.  kdtree: every
    sample query answered by the restated KdTreeFLANN radiusSearch (oracle/pcp_flann.c) --
    the reference's own search structure (virtual_lidar.cpp:782) -- instead of the exact
    grid scan."""
    pyoracle = _oracle()
    pyoracle.set_threads(threads)
    T = pyoracle.Cloud(terrain, flann=kdtree)
    units = 0
    k = 0
    chunk = 1 if threads == 1 else max(1, threads // 16)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:   # cycles through the poses until the budget
        j = k % len(poses)
        sel = poses[j:j + chunk]
        _, u, _ = pyoracle.raycast_fan(T, sel, fan.n_az, fan.n_el, fan.el_min, fan.el_max,
                                       fan.max_distance, want_first_hit=False)
        units += int(u.sum())
        k += sel.shape[0]
    dt = time.perf_counter() - t0
    pyoracle.set_threads(1)
    return {"value": units / dt, "unit": "ray-hit tests/s", "cores": threads, "kind": "port",
            "sample": f"{k} pose fans (cycling the {len(poses)} poses) x full "
                      f"{fan.n_az}x{fan.n_el}, "
                      f"{units} sample queries in {dt:.1f} s ("
                      + ("KdTreeFLANN restatement, oracle/pcp_flann.c, " if kdtree else
                         "oracle/pcp_oracle.c, ")
                      + f"{threads} thread{'s' if threads > 1 else ''})"}


def cpu_baseline_cells(terrain, aux, cells, poses, zx, budget_s: float, threads: int = 1,
                       kdtree: bool = False):
    """runOptimization's candidate loop on the CPU: 1 thread = the reference's own loop
    (orc_score_poses, flags and all); threads > 1 = per-pose totals over OpenMP.  kdtree:
    the radius searches on the restated KdTreeFLANN (oracle/pcp_flann.c), as the reference."""
    pyoracle = _oracle()
    import numpy as np

    T, A = pyoracle.Cloud(terrain, flann=kdtree), pyoracle.Cloud(aux, flann=kdtree)
    prm = pyoracle.vl_params()
    flags = np.zeros(cells.xyz.shape[0], np.uint8)
    chunk = 1 if threads == 1 else threads
    pyoracle.set_threads(threads)
    k = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:   # cycles through the poses until the budget
        j = k % len(poses)
        sel = poses[j:j + chunk]
        if threads == 1:
            pyoracle.score_poses(T, A, cells.xyz, cells.normals, sel, zx, prm, flags)
        else:
            pyoracle.score_totals(T, A, cells.xyz, cells.normals, sel, zx, prm)
        k += sel.shape[0]
    dt = time.perf_counter() - t0
    pyoracle.set_threads(1)
    return {"value": k / dt, "unit": "poses/s", "cores": threads, "kind": "port",
            "sample": f"{k} pose evaluations (cycling the {len(poses)} poses) x "
                      f"{cells.xyz.shape[0]} cells in {dt:.1f} s "
                      f"({'orc_score_poses' if threads == 1 else 'orc_score_totals, OpenMP'}"
                      + (", KdTreeFLANN restatement oracle/pcp_flann.c)" if kdtree else ")")}


def cpu_baseline_c3(clouds, box, leaf, tfs, budget_s: float = 4.0, threads: int = 1):
    """processCloudSimple (crop + VoxelGrid) per cloud, then processRobotCloud's transform +
    colour, on the CPU restatement: one whole C3 frame.  threads = 1: the reference's own
    single-threaded path (orc_crop_box + orc_voxel_grid + orc_transform_rgb); threads > 1: the
    same bytes from the OpenMP frame (oracle/pcp_oracle_mt.c: chunked crop, parallel stable
    radix sort of the voxel keys, per-voxel in-order sums, parallel transform)."""
    pyoracle = _oracle()
    n_in = sum(c.shape[0] for c in clouds)
    rgbs = [(255, 0, 0), (0, 0, 255)]
    frames = 0
    t0 = time.perf_counter()
    while frames == 0 or time.perf_counter() - t0 < budget_s:
        if threads == 1:
            n_out = 0
            for c, (t, q), rgb in zip(clouds, tfs, rgbs):
                kept = pyoracle.crop_box(c, box)
                vox, _, _, _ = pyoracle.voxel_grid(c[kept], leaf)
                out = pyoracle.transform_rgb(vox, t, q, rgb)
                n_out += out.shape[0]
        else:
            out, _ = pyoracle.filter_frame_mt(clouds, [box] * len(clouds), leaf, tfs, rgbs,
                                              threads)
            n_out = out.shape[0]
        frames += 1
    dt = (time.perf_counter() - t0) / frames
    how = ("oracle crop_box + voxel_grid + transform_rgb, 1 thread" if threads == 1 else
           f"oracle filter_frame_mt, OpenMP, {threads} threads")
    return {"value": n_in / dt, "unit": "input points/s", "cores": threads, "kind": "port",
            "sample": f"{frames} whole frames: {n_in} input points -> {n_out} merged, "
                      f"{dt:.3f} s per frame ({how})"}


def _rank_vector(dist, x):
    """Every rank's value of x, in rank order (rank r's entry of a sum-reduced vector): the
    per-rank figures SCALE lines carry beside their max-over-ranks ones."""
    if dist is None:
        return [x]
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    v = np.zeros(world, np.float64)
    v[rank] = np.nan if x is None else x
    v = dist.allreduce(v, "sum")
    return [None if not np.isfinite(a) else float(a) for a in v]


def _timed(step, args, dist, sync):
    """W untimed warmup steps, then exactly K steps between barrier + device synchronize on both
    sides (sync: the library context's stream synchronisation -- all of a step's work is on that
    stream); -> (max-over-ranks seconds, sum-over-ranks units, last step's result)."""

    def barrier_sync():
        if dist is not None:
            dist.barrier()
        sync()

    for _ in range(args.warmup):
        step()
    gc_was = gc.isenabled()
    gc.collect()
    gc.disable()   # no collector pause inside the K timed steps (host-side jitter only)
    try:
        barrier_sync()
        t0 = time.perf_counter()
        units = 0.0
        res = None
        for _ in range(args.steps):
            u, res = step()
            units += u
        barrier_sync()
        dt = time.perf_counter() - t0
    finally:
        if gc_was:
            gc.enable()
    _timed.per_rank_s = _rank_vector(dist, dt)   # each rank's own K-step time
    if dist is not None:   # host-side (the control plane)
        dt = float(dist.allreduce(np.array([dt]), "max")[0])
        units = float(dist.allreduce(np.array([units], np.float64), "sum")[0])
    return dt, units, res


def _profiled(ctx, step, reps, names):
    """Per-launch event times of `names` over `reps` extra steps run AFTER the timed loop: the
    library's event instrumentation (ctx.profile) stays out of the timed region."""
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(reps):
        step()
    ctx.profile(False)
    out = {}
    for k in names:
        ms, n = ctx.profile_get(k)
        out[k] = ms / max(n, 1)
    return out


GATHER_PATH_FILES = {"fan": ("r06_fan_gather_path.json", "r05_fan_gather_path.json"),
                     "cells": ("r06_cells_gather_path.json",)}


def _gather_path(workload="fan"):
    """A gather kernel's texture-path counters (tools/pmc_fan.sh or tools/pmc_cells.sh +
    tools/pmc_gather.py): TA / TD busy, L1 tag lookups per instruction, wave wait / VALU
    shares -- stamped with the kernel's sources like the traffic file, and marked stale
    (gather_path_stale) when this tree's sources differ."""
    from pointcloud_processor_amd._stamps import workload_stamp

    for name in GATHER_PATH_FILES[workload]:
        f = ROOT / "profiles" / name
        try:
            d = json.loads(f.read_text())
        except (OSError, ValueError):
            continue
        d = {k: v for k, v in d.items() if k != "counters_mean_per_dispatch"}
        d["source"] = f"profiles/{name}"
        d["gather_path_stale"] = d.get("source_stamp") != workload_stamp(workload)
        return d
    return None


GATHER_CEILING_FILE = "r05_gather_ceiling.json"


def _gather_ceiling():
    """Measured divergent lane-load ceilings per lane width (tools/mb/gather_ceiling.hip ->
    profiles/r05_gather_ceiling.json): {2: rate, 4: rate, 12: rate} lane-loads/s, or None."""
    f = ROOT / "profiles" / GATHER_CEILING_FILE
    try:
        d = json.loads(f.read_text())
        return {int(w): float(r) for w, r in d["ceiling_lane_loads_per_s"].items()}, d
    except (OSError, ValueError, KeyError):
        return None, None


def _fan_npw(n_poses):
    """Poses per wave of the production fan kernel: the library's rule (pcp_vlidar.hip
    raycast_fan_impl) -- PCP_FAN_NPW (default 8), halved until it divides the XCD pose chunk."""
    npw = int(os.environ.get("PCP_FAN_NPW", "8"))
    npw = npw if npw in (1, 2, 4, 8, 16, 32) else 1
    while npw > 1 and n_poses % (8 * npw):
        npw //= 2
    return npw


def _fan_roofline(ctx, poses, fan, avg_kernel_s, units_per_launch):
    """Roofline of k_raycast_fan.  The kernel's bound is the texture path of its
    gathers, not HBM: each lane of a probe, walk-start or point-record load hits its own cache
    line.  `achieved` = the gather lane-loads of one launch (pcp_raycast_fan_stats: z-band probes
    + candidate walk starts + point records + directory loads) / the launch time; `peak` = the
    measured ceiling of that load shape for the launch's own mix of widths
    (profiles/r05_gather_ceiling.json, tools/mb/gather_ceiling.hip: 2-B probes, 4-B walk starts,
    12-B point records, each at its width's measured chip-wide rate), so frac = lane-loads /
    kernel time / peak by one division.  No ceiling file: peak and frac are None (nothing is
    assumed).  HBM beside it from the stamped PMC bytes (hbm_frac), the bytes the loads request
    (served by L1/L2/MALL: the terrain copy is cache-resident) as requested_*, the texture-path
    busy fractions as gather_path (stamped; stale when the fan's sources changed)."""
    st = ctx.raycast_fan_stats(poses, fan)
    layout = ctx.terrain_info()["scan_layout"]
    split = layout == "fine" and ctx.terrain_info().get("fine_tile") == 2
    probe_b = 8.0 if layout == "fine" and not split else 2.0
    cand_b = 4.0 if split else 8.0
    rays = poses.shape[0] * fan.n_az * fan.n_el
    waves = poses.shape[0] * ((fan.n_az * fan.n_el + 63) // 64)
    npw = _fan_npw(poses.shape[0]) if layout == "fine" else 1
    gathers = (st["samples_visited"] + st["scanned_stencils"] + st["point_tests"]
               + st["directory_loads"])
    req = probe_b * st["samples_visited"] + cand_b * st["scanned_stencils"] \
        + 8.0 * st["directory_loads"] + 12.0 * st["point_tests"] + 16.0 * rays / npw \
        + 8.0 * waves
    ref_model = 64.0 * units_per_launch + 12.0 * st["point_tests"]
    traffic, tinfo = _traffic_from_profiles("fan")
    achieved = gathers / avg_kernel_s if avg_kernel_s else None
    hbm_gbs = _gbs(traffic, avg_kernel_s)
    ceil, cfile = _gather_ceiling()
    peak = None
    mix = {int(probe_b) if split else 2: st["samples_visited"],
           int(cand_b) if split else 4: st["scanned_stencils"],
           12: st["point_tests"] + st["directory_loads"]}
    if ceil and all(w in ceil for w in mix):
        # the time the launch's lane-loads take at their widths' ceilings -> one rate
        t_ceil = sum(n / ceil[w] for w, n in mix.items())
        peak = gathers / t_ceil if t_ceil else None
    return {
        "bound": "gather (TA/TD)",
        "achieved": achieved / 1e9 if achieved else None,
        "peak": peak / 1e9 if peak else None,
        "unit": "G lane-loads/s",
        "frac": achieved / peak if achieved and peak else None,
        "peak_source": (f"profiles/{GATHER_CEILING_FILE} (source_sha16 "
                        f"{cfile.get('source_sha16')}): per-width ceilings "
                        + ", ".join(f"{w} B: {r / 1e9:.1f} G/s" for w, r in sorted(ceil.items()))
                        + f", weighted by this launch's lane-load mix {mix}")
        if cfile else "none committed: peak / frac not computed",
        "traffic": traffic,
        **(tinfo or {}),
        "hbm_gbs": hbm_gbs,
        "hbm_frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs else None,
        "gather_lane_loads_per_launch": gathers,
        "executed_lane_loads": gathers,
        "executed_point_tests": st["point_tests"],
        "executed_point_tests_per_s": st["point_tests"] / avg_kernel_s if avg_kernel_s else None,
        "model": "frac = (probes + walk starts + point records + directory loads per launch, "
                 "pcp_raycast_fan_stats) / avg_kernel_ms / peak, peak = those lane-loads / sum "
                 "over widths of (lane-loads of the width / measured ceiling of the width); "
                 "hbm_frac = traffic (PMC: fetch_factor x FETCH_SIZE + WRITE_SIZE per launch, "
                 "fetch_factor from the gather calibration, fetch_factor_source) / avg_kernel_ms "
                 "/ 8 TB/s; executed_point_tests_per_s = the point tests the kernel actually runs "
                 "per second (value counts the reference's sample queries)",
        "kernel": (f"k_raycast_fan_xcd<0, 64, true, 8, {8 if split else 4}, true, {npw}>"
                   if layout == "fine"
                   else "k_raycast_fan<0, 64, true, 7, 0>"),
        "poses_per_wave": npw,
        "avg_kernel_ms": avg_kernel_s * 1e3, "scan_layout": layout,
        "requested_bytes_per_launch": req,
        "requested_gbs": _gbs(req, avg_kernel_s),
        "requested_model": f"{probe_b:.0f} B/probe + {cand_b:.0f} B/candidate + 8 B/directory "
                           "load + 12 B/point record + 16 B/ray/NPW + 8 B/wave partial",
        "alg_reference_bytes_per_launch": ref_model,
        "alg_reference_bytes_frac": (ref_model / avg_kernel_s / 1e9 / HBM_PEAK_GBS)
        if avg_kernel_s else None,
        "alg_reference_model": "SURVEY 8d: 64 B per reference sample query + 12 B per point "
                               "test; > 1 because the kernel skips ~95 % of the sample "
                               "queries exactly (DESIGN.md §5)",
        "diag": st,
        "gather_path": _gather_path(),
    }


CHAIN_FILE = "r06_chain.json"   # tools/mb/chain.hip on the box: dependent f64 add latency


def _cells_roofline(ctx, cposes, zx5, params, n_cells, kern):
    """Roofline of the reference's own ray march (runOptimization's k_score_cells, VERDICT r5
    item 3), on the fan's terms: `achieved` = the gather lane-loads of one launch (z-band probes
    + walk starts + point records + directory loads, counted by the kernel's STATS twin,
    pcp_score_poses_stats) / the launch time (the production launch 20 times back-to-back
    between two events, pcp_score_poses_burst); `peak` = the measured ceilings of
    profiles/r05_gather_ceiling.json weighted by this launch's mix of widths.  HBM from the
    stamped PMC bytes (hbm_frac).  Beside it the row sums' kernel (k_sum_flags, per-launch
    event time) against its dependent-add floor: C adds per row chain x the measured latency of
    one dependent v_add_f64 (profiles/r06_chain.json, tools/mb/chain.hip)."""
    st = ctx.score_poses_stats(cposes, zx5, params)
    ms = ctx.score_poses_burst(cposes, zx5, params, reps=20)
    s = ms * 1e-3
    gathers = st["probes"] + st["walk_starts"] + st["point_tests"] + st["directory_loads"]
    mix = {2: st["probes"], 4: st["walk_starts"], 12: st["point_tests"] + st["directory_loads"]}
    ceil, cfile = _gather_ceiling()
    peak = None
    if ceil and all(w in ceil for w in mix):
        t_ceil = sum(n / ceil[w] for w, n in mix.items())
        peak = gathers / t_ceil if t_ceil else None
    achieved = gathers / s if s else None
    traffic, tinfo = _traffic_from_profiles("cells")
    hbm_gbs = _gbs(traffic, s)
    rays = (cposes.shape[0] + 1) * n_cells
    chain = None
    try:
        chain = json.loads((ROOT / "profiles" / CHAIN_FILE).read_text())
    except (OSError, ValueError):
        pass
    sum_ms = kern.get("pose_sum")
    floor_ms = n_cells * chain["ns_per_dependent_f64_add"] * 1e-6 if chain else None
    return {
        "bound": "gather (TA/TD)", "kernel": "k_score_cells<true>",
        "achieved": achieved / 1e9 if achieved else None,
        "peak": peak / 1e9 if peak else None, "unit": "G lane-loads/s",
        "frac": achieved / peak if achieved and peak else None,
        "peak_source": (f"profiles/{GATHER_CEILING_FILE} (source_sha16 "
                        f"{cfile.get('source_sha16')}), weighted by this launch's lane-load mix "
                        f"{mix}") if cfile else "none committed: peak / frac not computed",
        "avg_kernel_ms": ms, "kernel_time_source": "pcp_score_poses_burst: 20 back-to-back "
                                                   "launches between two HIP events",
        "gather_lane_loads_per_launch": gathers, "diag": st, "rays_per_launch": rays,
        "lane_loads_per_ray": gathers / rays if rays else None,
        "traffic": traffic, **(tinfo or {}), "hbm_gbs": hbm_gbs,
        "hbm_frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs else None,
        "sum_flags": {"kernel": "k_sum_flags (ordered row sums + stale flags)",
                      "event_ms": sum_ms, "floor_ms": floor_ms,
                      "frac_of_floor": floor_ms / sum_ms if floor_ms and sum_ms else None,
                      "floor_model": f"{n_cells} dependent f64 adds per row chain x "
                                     + (f"{chain['ns_per_dependent_f64_add']:.3f} ns "
                                        f"(profiles/{CHAIN_FILE})" if chain else
                                        "(no chain measurement committed)")},
        "model": "frac = (probes + walk starts + point records + directory loads per launch, "
                 "pcp_score_poses_stats) / avg_kernel_ms / mix-weighted gather ceiling; "
                 "hbm_frac = PMC traffic per launch / avg_kernel_ms / 8 TB/s",
        "gather_path": _gather_path("cells"),
        "limiter": "latency: ~950 k short rays (8.3 lane-loads each) in ~2.4 rounds of waves at 6 "
                   "waves per SIMD -- texture data path 67 % busy, waves waiting 55 % of their "
                   "life (gather_path); the furthest of the hot kernels below its ceiling",
    }


def _fan_stepper(ctx, poses, fan, lo, P_total, dist, backend):
    """One step of the pose-sharded fan search for this rank's poses [lo, lo + len(poses)) of
    P_total -> (step() -> (ray-hit tests of this rank, blocked counts), best {"fan": argmin},
    the all-poses blocked vector the step fills).  N > 1 over RCCL: libpcp's own communicator --
    the per-pose keys (blocked << 32) | pose are written into the context's device vector, ONE
    ncclAllReduce(MIN) runs on the library's stream, only the reduced vector comes back
    (pcp_raycast_fan_allreduce).  The gloo rehearsal (ranks sharing one GPU) reduces a host
    vector through the control plane (dist.reduce_fan)."""
    from pointcloud_processor_amd import dist as pd

    best = {}
    blocked_h = np.zeros(max(poses.shape[0], 1), np.uint32)
    units_h = np.zeros(max(poses.shape[0], 1), np.uint64)
    # one rank: its own blocked vector is the whole one (no copy inside the timed steps)
    blocked_all = blocked_h if dist is None else np.zeros(max(P_total, 1), np.uint32)
    if backend == "rccl":
        def fan_step():
            best["fan"], _ = ctx.raycast_fan_allreduce(poses, fan, lo, P_total, blocked_all,
                                                       units_h)
            return int(units_h[:poses.shape[0]].sum()), blocked_all
    else:
        def fan_step():
            b = ctx.raycast_fan_into(poses, fan, blocked_h, units_h)   # argmin of its poses
            if dist is None:   # one rank: the library's argmin is the node's answer
                keys = blocked_h
            else:
                keys, b = pd.reduce_fan(blocked_h[:poses.shape[0]], lo, lo + poses.shape[0],
                                        P_total, dist)
            if dist is not None:
                blocked_all[:P_total] = np.asarray(keys[:P_total], np.uint32)
            best["fan"] = b   # ^ the one collective
            return int(units_h[:poses.shape[0]].sum()), keys
    return fan_step, best, blocked_all


C4_POSES = 4096   # BASELINE configs[3]: 4096 candidate poses sharded over the GPUs


def _c4_checks(dist, ctx=None, poses=None, fan=None, lo=0, p_total=0, backend=None):
    """What lets a SCALE line's c4 be checked on its own: each rank's fan
    kernel time for its shard (the production kernel 10 times back-to-back between two events,
    pcp_raycast_fan_burst) and its max / min over ranks, the collective's own time (events
    around libpcp's ncclAllReduce, median of 3), the ranks RCCL's communicator saw
    (pcp_comm_info: 0 when no RCCL communicator exists, e.g. the gloo rehearsal) and the runtime
    libpcp ran on.  ctx None (the CPU launch check): no kernel or collective figures."""
    kms = None
    coll = None
    nranks = 0
    if ctx is not None:
        kms = ctx.raycast_fan_burst(poses, fan, reps=10) if poses.shape[0] else 0.0
        nranks = ctx.comm_info()[0]
        if backend == "rccl":
            ms = [ctx.raycast_fan_allreduce(poses, fan, lo, p_total, timed=True)[1]
                  for _ in range(3)]
            coll = float(np.median(ms))
    per = _rank_vector(dist, kms)
    known = [k for k in per if k is not None]
    return {"kernel_ms_per_rank": per,
            "kernel_ms_max": max(known) if known else None,
            "kernel_ms_min": min(known) if known else None,
            "kernel_time_source": "pcp_raycast_fan_burst: 10 back-to-back launches of the "
                                  "rank's shard between two HIP events",
            "collective_ms": coll, "rccl_nranks": nranks, "runtime": _runtime()}


def run_c4(args, dist, world, rank, local, backend, ctx=None, scene=None):
    """BASELINE configs[3]: the 4,096-pose search STRONG-scaled over the N ranks (rank r casts
    poses [r*4096/N, (r+1)*4096/N), the split of runOptimization's candidate loop,
    virtual_lidar.cpp:467-475), one all-reduce(MIN) per step.  value = ray-hit tests of all
    ranks / max-over-ranks time.  Rank 0 re-casts a sample of the poses on the oracle (the best
    one among them) and compares their blocked counts with the reduced vector."""
    from pointcloud_processor_amd import _abi, synth
    from pointcloud_processor_amd import dist as pd

    own = ctx is None
    if own:
        ctx = _abi.Context(local)
        if backend == "rccl":
            uid = dist.broadcast_bytes(_abi.comm_unique_id() if rank == 0 else None, src=0)
            ctx.comm_init_rank(world, uid, rank)
        scene = synth.terrain_scene()
        ctx.set_terrain(scene.terrain, point_step=32)
    fan = _abi.fan_params(n_az=args.n_az, n_el=args.n_el)
    poses_all, nc = _poses_for(ctx, _grid_bbox(scene.area), scene.zx120_pose5, C4_POSES)
    lo, hi = pd.shard(C4_POSES, world, rank)
    poses = np.ascontiguousarray(poses_all[lo:hi])
    step, best, blocked_all = _fan_stepper(ctx, poses, fan, lo, C4_POSES, dist, backend)
    dt, units_all, _ = _timed(step, args, dist, ctx.synchronize)
    shards = [pd.shard(C4_POSES, world, r) for r in range(world)]
    res = {"workload": "C4 (configs[3]): 4096 candidate poses strong-scaled over the ranks, "
                       f"1024x256 fan each, one all-reduce(MIN) per step ({backend or 'none'})",
           "value": units_all / dt, "unit": "ray-hit tests/s", "n_gpus": world,
           "scaling": "strong", "steps": args.steps, "ms_per_step": dt / args.steps * 1e3,
           "poses_total": C4_POSES, "poses_per_rank": [h - l for l, h in shards],
           "poses_per_s": C4_POSES * args.steps / dt, "best_pose": best["fan"],
           "num_candidates_lattice": nc,
           "ms_per_step_per_rank": [t / args.steps * 1e3 for t in _timed.per_rank_s]}
    res.update(_c4_checks(dist, ctx, poses, fan, lo, C4_POSES, backend))
    if rank == 0 and not args.no_cpu_baseline:
        # oracle check: the argmin pose plus 7 poses spread over every rank's shard
        pyoracle = _oracle()
        pyoracle.set_threads(_host_cpu()["threads_used"])
        pick = sorted({int(best["fan"])} | {int(i) for i in
                                            np.linspace(0, C4_POSES - 1, 7).astype(int)})
        rb, _, _ = pyoracle.raycast_fan(pyoracle.Cloud(scene.terrain), poses_all[pick], fan.n_az,
                                        fan.n_el, fan.el_min, fan.el_max, fan.max_distance,
                                        want_first_hit=False)
        pyoracle.set_threads(1)
        res["oracle_check"] = {"poses": pick,
                               "blocked_equal": bool(np.array_equal(
                                   np.asarray(rb, np.int64),
                                   blocked_all[pick].astype(np.int64))),
                               "best_blocked": int(blocked_all[best["fan"]]),
                               "min_of_reduced_vector": int(blocked_all[:C4_POSES].min())}
    if own:
        ctx.close()
    return res


def run_all(args, dist, world, rank, local, backend):
    """Default line: the C2 fan (value), reference-mode scoring of the same node
    (runOptimization, poses/s) and the C3 filter frame, each timed as its own loop of K steps
    with the barrier / max-over-ranks discipline; CPU baselines on rank 0 at N = 1."""
    import numpy as np

    from pointcloud_processor_amd import _abi, synth
    from pointcloud_processor_amd import dist as pd

    ctx = _abi.Context(local)
    if backend == "rccl":   # libpcp's own communicator; the id travels over the gloo group
        uid = dist.broadcast_bytes(_abi.comm_unique_id() if rank == 0 else None, src=0)
        ctx.comm_init_rank(world, uid, rank)
    scene = synth.terrain_scene()
    ctx.set_terrain(scene.terrain, point_step=32)
    P_total = args.poses_per_gpu * world
    poses_all, nc = _poses_for(ctx, _grid_bbox(scene.area), scene.zx120_pose5, P_total)
    lo, hi = pd.shard(P_total, world, rank)
    poses = np.ascontiguousarray(poses_all[lo:hi])
    fan = _abi.fan_params(n_az=args.n_az, n_el=args.n_el)

    # ---- C2: the fan (the headline) --------------------------------------------------------
    fan_step, best, blocked_all = _fan_stepper(ctx, poses, fan, lo, P_total, dist, backend)
    own_comm = backend == "rccl"
    dt, units_all, _ = _timed(fan_step, args, dist, ctx.synchronize)
    units_h = np.zeros(max(poses.shape[0], 1), np.uint64)
    collective = None
    if own_comm:
        ms = []
        for _ in range(max(args.steps, 3)):   # after the timed loop: events around the collective
            ms.append(ctx.raycast_fan_allreduce(poses, fan, lo, P_total, blocked_all, units_h,
                                                timed=True)[1])
        collective = {"op": "ncclAllReduce(ncclUint64, ncclMin)", "backend": "rccl (libpcp)",
                      "bytes": 8 * P_total, "collective_ms": float(np.median(ms)),
                      "path": "device keys in libpcp's vector (written by k_fan_reduce), libpcp's "
                              "own RCCL communicator on its stream (pcp_raycast_fan_allreduce), "
                              "the reduced vector and the shard's units landed by one copy "
                              "kernel; torch.distributed (gloo, in a helper process: "
                              "hostgroup.py) only for the id hand-off and barriers"}
        nr, rr = ctx.comm_info()
        collective["rccl_nranks"] = nr   # the ranks RCCL's communicator saw (pcp_comm_info)
        collective["runtime"] = _runtime()
    elif dist is not None:
        collective = {"op": "all_reduce(MIN) int64", "backend": backend, "bytes": 8 * P_total,
                      "path": "host vector (gloo rehearsal: ranks share devices)"}
    k_avg = _profiled(ctx, fan_step, max(args.steps, 3), ["raycast_fan"])["raycast_fan"]
    # the kernel's launch time: the same launch 20 times back-to-back between two events on the
    # library's stream (the per-step events of the synchronous loop also hold the idle queue's
    # wake-up before each launch; kept below as event_avg_ms_in_loop)
    burst_ms = ctx.raycast_fan_burst(poses, fan, reps=20)
    avg_kernel_s = burst_ms * 1e-3
    units_per_launch = units_all / max(world, 1) / max(args.steps, 1)
    out = {
        "metric": METRIC,
        "value": units_all / dt,
        "unit": "ray-hit tests/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / max(args.steps, 1) * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64 march / f32 point test",
        "data": "synthetic (seeded T1M L-pit terrain, reference candidate lattice)",
        "config": {"workload": "C2: 1M-pt L-shape excavation terrain, 1024x256 ray fan, "
                               f"{args.poses_per_gpu} candidate poses per GPU",
                   "terrain_points": int(scene.terrain.shape[0]),
                   "poses_total": P_total, "fan": [args.n_az, args.n_el],
                   "num_candidates_lattice": nc, "parallelism": f"pose-shard x{world}",
                   "collective": None if dist is None else f"all-reduce(MIN) over {backend}"},
        "collective": collective,
        "poses_per_s": P_total * args.steps / dt,
        # each rank's own time for its 256 poses: the N = 1-comparable figure of a SCALE line
        "ms_per_step_per_rank": [t / max(args.steps, 1) * 1e3 for t in _timed.per_rank_s],
        "best_pose": best["fan"],
        "roofline": _fan_roofline(ctx, poses, fan, avg_kernel_s, units_per_launch),
    }
    out["roofline"]["kernel_time_source"] = ("HIP events around 20 back-to-back launches "
                                             "(pcp_raycast_fan_burst)")
    out["roofline"]["event_avg_ms_in_loop"] = k_avg
    if dist is not None and backend == "gloo":
        out["rehearsal"] = (f"{world} ranks on {_abi.device_count()} GPU(s): collective "
                            "over gloo, ranks share devices")
    if dist is not None:   # configs[3]: the 4096-pose search strong-scaled over these ranks
        out["c4"] = run_c4(args, dist, world, rank, local, backend, ctx=ctx, scene=scene)
    host = _host_cpu()
    cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    if not args.fan_only and not getattr(args, "cells_only", False) and rank == 0 and world == 1:
        # the host-bound chains first, before the CPU baselines below load the host's cores:
        # configs[4] on this GPU (200 frames of the whole chain through the node cores, the
        # first and last dumped frames re-run through the oracle chain after the timed frames),
        # then configs[0] (its one-thread oracle frames after its own timed ones)
        out["c5"] = run_c5(args, None, 1, 0, local, None, frames=200, check=cpu)
        out["c1"] = run_c1(args, local, cpu)
    if cpu:
        out["cpu_baseline"] = cpu_baseline_fan(scene.terrain, poses, fan, args.cpu_seconds)
        out["cpu_baseline_mt"] = cpu_baseline_fan(scene.terrain, poses, fan,
                                                  args.cpu_seconds / 2,
                                                  threads=host["threads_used"])
        out["cpu_baseline_mt"]["host"] = host
        # the reference's own search structure on one core: the march of virtual_lidar.cpp:
        # 765-797 with radiusSearch on the restated KdTreeFLANN (FLANN 1.9.1 as PCL configures it)
        out["cpu_baseline_kdtree"] = cpu_baseline_fan(scene.terrain, poses, fan,
                                                      args.cpu_seconds / 2, kdtree=True)

    # ---- reference mode: runOptimization over the excavation cells (poses/s) -----------
    if not args.fan_only:
        cells = synth.excavation_cells(scene.area)
        aux = synth.aux_cloud()
        ctx.set_aux_cloud(aux, point_step=32)
        ctx.set_cells(cells.xyz, cells.normals)
        cposes_all, cnc = _poses_for(ctx, cells.grid_bbox, scene.zx120_pose5, P_total)
        cposes = np.ascontiguousarray(cposes_all[lo:hi])
        params = _abi.default_vl_params()
        flags = np.zeros(cells.xyz.shape[0], np.uint8)

        tot = np.zeros(max(cposes.shape[0], 1), np.float64)
        cov = np.zeros(max(cposes.shape[0], 1), np.int32)
        rep = _abi.VlReport()
        zx5 = np.ascontiguousarray(scene.zx120_pose5, np.float64)

        tot_all = np.zeros(max(P_total, 1), np.float64)
        cov_all = np.zeros(max(P_total, 1), np.int32)
        if backend == "rccl":
            # ONE ncclAllReduce(MAX) per query over [totals | covered | newest-pose flag keys |
            # health] on libpcp's own communicator; stale flags + argmax on every rank
            def cells_step():
                ctx.score_poses_allreduce(cposes, zx5, params, lo, P_total, flags, tot_all,
                                          cov_all, rep)
                best["cells"] = rep.best_idx
                return cposes.shape[0], tot_all
        else:
            def cells_step():
                ctx.score_poses_into(cposes, zx5, params, flags, tot, cov, rep)
                if dist is None:   # one rank: the library's strict-'>' argmax (rep.best_idx)
                    b = rep.best_idx
                else:   # gloo rehearsal (ranks share devices): totals over the host group
                    _, b, _ = pd.reduce_scores(tot[:cposes.shape[0]], lo, hi, P_total, dist)
                best["cells"] = b
                return cposes.shape[0], tot

        cdt, cunits, _ = _timed(cells_step, args, dist, ctx.synchronize)
        kern = _profiled(ctx, cells_step, max(args.steps, 3),
                         ("score_cells", "pose_sum", "cell_flags"))
        out["poses_per_s_reference_mode"] = cunits / cdt
        out["reference_mode"] = {
            "workload": f"runOptimization: {P_total} candidate poses x {cells.xyz.shape[0]} "
                        "cells, visibility by ray march (virtual_lidar.cpp:454-548)",
            "value": cunits / cdt, "unit": "poses/s", "ms_per_step": cdt / args.steps * 1e3,
            "best_pose": best["cells"], "num_candidates_lattice": cnc,
            "kernel_avg_ms": kern, "dtype": "f64",
            "roofline": _cells_roofline(ctx, cposes, zx5, params, cells.xyz.shape[0], kern),
        }
        if backend == "rccl":
            ms = [ctx.score_poses_allreduce(cposes, zx5, params, lo, P_total, flags, tot_all,
                                            cov_all, rep, timed=True) for _ in range(3)]
            out["reference_mode"]["collective"] = {
                "op": "ncclAllReduce(ncclUint64, ncclMax)", "backend": "rccl (libpcp)",
                "words": 2 * P_total + 3 * cells.xyz.shape[0] + 1,
                "vector": "[P totals | P covered | 3 x C newest-pose flag keys | health]",
                "collective_ms": float(np.median(ms)), "rccl_nranks": ctx.comm_info()[0],
                "path": "pcp_score_poses_allreduce: keys on the device, one all-reduce on the "
                        "context's stream, stale flags + strict-'>' argmax on every rank"}
        elif dist is not None:
            out["reference_mode"]["collective"] = {
                "op": "all_reduce(MAX) float64 totals", "backend": backend, "rccl_nranks": 0,
                "path": "host vector (gloo rehearsal: ranks share devices)"}
        if cpu:
            out["reference_mode"]["cpu_baseline"] = cpu_baseline_cells(
                scene.terrain, aux, cells, cposes, scene.zx120_pose5, args.cpu_seconds / 2)
            out["reference_mode"]["cpu_baseline_mt"] = cpu_baseline_cells(
                scene.terrain, aux, cells, cposes, scene.zx120_pose5, args.cpu_seconds / 2,
                threads=host["threads_used"])
            out["reference_mode"]["cpu_baseline_kdtree"] = cpu_baseline_cells(
                scene.terrain, aux, cells, cposes, scene.zx120_pose5, args.cpu_seconds / 2,
                kdtree=True)
        if not getattr(args, "cells_only", False):
            out["c3"] = run_filter(args, dist, world, rank, local, backend, embedded=True,
                                   cpu=cpu)
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


def run_filter(args, dist, world, rank, local, backend=None, embedded=False, cpu=False):
    """C3: crop + voxel(0.05) + transform on a 10M-pt dual-LiDAR frame, inputs in HBM.  Every
    rank runs its own frame (replicas); value = input points of all ranks / max-over-ranks
    time."""
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
    n_in = sum(c.shape[0] for c in clouds)
    last = {}

    frame = ctx.filter_merge_device_prepared(views, [box, box], 0.05, tfs,
                                             [(255, 0, 0), (0, 0, 255)], out_d, cap)

    def step():
        n_out, per = frame()
        last["n_out"], last["per"] = n_out, per
        return n_in, n_out

    dt, units_all, _ = _timed(step, args, dist, ctx.synchronize)
    step_dev_ms = _profiled(ctx, step, max(args.steps, 3), ["filter_merge"])["filter_merge"]
    n_out = last["n_out"]
    stages = None
    pcie = None
    if not embedded:
        # per-stage breakdown from one eager (non-graph) context, untimed
        os.environ["PCP_NO_GRAPHS"] = "1"
        ectx = _abi.Context(local)
        os.environ.pop("PCP_NO_GRAPHS")
        ectx.profile(True)
        for _ in range(3):
            ectx.filter_merge_device(views, [box, box], 0.05, tfs, [(255, 0, 0), (0, 0, 255)],
                                     out_d, cap)
        stages = {k: ectx.profile_get(k)[0] / 3 for k in ("crop", "voxel", "transform",
                                                          "filter_merge")}
        ectx.close()
        pcie = None if args.no_pcie else _pcie_inclusive(ctx, clouds, box, tfs, n_in, cap)
    alg = 12.0 * n_in + 16.0 * n_out
    traffic, tinfo = _traffic_from_profiles("filter")
    hbm_gbs = _gbs(traffic, step_dev_ms * 1e-3)
    res = {
        "metric": "crop+voxel+transform points/s (C3)", "value": units_all / dt,
        "unit": "input points/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / max(args.steps, 1) * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic 2 x LiDAR-like clouds, point_step 16, resident in HBM",
        "config": {"workload": f"C3: crop+voxel(0.05)+transform, {n_in} pts per GPU",
                   "n_out": n_out, "per_cloud": [int(x) for x in last["per"]], "graph": True},
        "roofline": {"bound": "hbm", "achieved": alg / (step_dev_ms * 1e-3) / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": alg / (step_dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "traffic": traffic, **(tinfo or {}),
                     "hbm_gbs": hbm_gbs,
                     "hbm_frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs else None,
                     "traffic_over_alg": traffic / alg if traffic else None,
                     "limiter": "crop streams its 160 MB at ~5 TB/s (1/3 of the frame); the "
                                "voxel stage -- bucket chain: k_bk_group (per-group counting sort "
                                "by bucket), k_bk_sort (per-bucket LDS sort + input-order sums), "
                                "k_bk_emit -- is three dependent launches of latency-bound "
                                "blocks (global round trips + barriers), not bytes",
                     "chain": {1: "LSD", 2: "bucket"}.get(
                         int(os.environ.get("PCP_FM_FAST", "2") or 2), "general"),
                     "kernel": "filter_merge graph (all stages)", "avg_kernel_ms": step_dev_ms,
                     "model": "achieved = 12 B/input point + 16 B/output point (SURVEY 8d) / "
                              "device time of the frame; hbm_frac = traffic (PMC fetch_factor x "
                              "FETCH_SIZE + WRITE_SIZE per frame) / device time / 8 TB/s"},
    }
    if stages is not None:
        res["roofline"]["eager_stage_ms"] = stages
    if pcie is not None:
        res["pcie_inclusive"] = pcie
    if cpu or (not embedded and rank == 0 and world == 1 and not args.no_cpu_baseline):
        res["cpu_baseline"] = cpu_baseline_c3(clouds, np.array(box), 0.05, tfs)
        host = _host_cpu()
        res["cpu_baseline_mt"] = cpu_baseline_c3(clouds, np.array(box), 0.05, tfs, budget_s=2.0,
                                                 threads=host["threads_used"])
        res["cpu_baseline_mt"]["host"] = host
    for p in dptr + [out_d]:
        ctx.dev_free(p)
    ctx.close()
    return res


C1_BOX = [0.0, 15.0, -10.0, 10.0, -1.5, 10.0]   # pointcloud_filter.cpp:30-36 defaults
C1_LEAF = 0.2                                    # voxel_leaf_size (:39)
C1_TFS = [((8.0, -3.0, 2.0), (0.0, 0.0, 0.2588190451025208, 0.9659258262890683)),   # robot
          ((0.55, 0.4, 3.5), (0.0, 0.21633, 0.0, 0.97632))]   # tf_zx120.launch.xml extrinsic
C1_ZX_BASE = ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))        # map -> zx120/base_link


def _c1_scans(points=60_032, seed=101):
    """One rosbag frame of BASELINE configs[0]: an HDL-64-like scan per sensor (64 rings,
    -24.9..+2 deg, ranges clipped at the ground; sensor heights 2.0 / 3.5 m)."""
    from pointcloud_processor_amd import synth

    return [synth.lidar_cloud(points, sensor_height=2.0, seed=seed),
            synth.lidar_cloud(points, sensor_height=3.5, seed=seed + 1)]


def c1_frame_gpu(ctx, scans, nc_lattice=1):
    """The launch file's per-frame chain on one GPU through the C ABI, host buffers in and out
    (a rosbag message is a host buffer): pointcloud_filter x2 (crop + VoxelGrid 0.2) ->
    pointcloud_merger (transform + colour + concat) -> excavated_surface_generator (carve) ->
    virtual_lidar (normals + cell grid, terrain index, zx120 cloud, runOptimization with ONE
    candidate pose).  -> (n_candidates, best_idx, totals).  The nodes composed as the C5 chain
    composes them (pcp_filter_merge_nodes: both filters + the merger, one wait;
    pcp_excavate_area_async: the carve + the area and terrain callbacks, the grid setup left in
    flight on its side stream while the zx120 index and the candidates are built; the scoring
    settles it); PCP_C1_CALLS=1: every node callback as its own call (rounds 1-4)."""
    from pointcloud_processor_amd import _abi

    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])   # getZX120Position on zx120/base_link
    params = _abi.default_vl_params(num_candidates=nc_lattice)
    if os.environ.get("PCP_C1_CALLS", "0") == "1":
        filtered = [ctx.crop_voxel(sc, C1_BOX, C1_LEAF)[0] for sc in scans]
        merged = ctx.transform_concat(filtered, C1_TFS, [(255, 0, 0), (0, 0, 255)])
        terr, area, _ = ctx.excavate(merged, C1_ZX_BASE)
        bbox, nc = ctx.set_excavation_area(area, 0.1, 10)
        ctx.set_terrain(terr, point_step=32)
        ctx.set_aux_cloud(filtered[1])
        cand = ctx.generate_candidates(bbox, params, zx)[:1]   # ONE candidate pose is scored
        tot, _, rep = ctx.score_poses(cand, zx, params, np.zeros(nc, np.uint8))
        return cand.shape[0], int(rep.best_idx), tot, cand, nc
    merged, filtered, _ = ctx.filter_merge_nodes(scans, [C1_BOX, C1_BOX], C1_LEAF, C1_TFS,
                                                 [(255, 0, 0), (0, 0, 255)])
    # (the carve's messages copied out by the call, split over libpcp's copy threads: reading
    # them from the landing afterwards, one numpy copy each, measured no faster --
    # profiles/r05_c1_landed_ab.log, r05_c1_poll_ab.log)
    terr, area, _, bbox, cap = ctx.excavate_area_async(merged, C1_ZX_BASE)
    ctx.set_aux_cloud(filtered[1])
    cand = ctx.generate_candidates(bbox, params, zx)[:1]   # ONE candidate pose is scored
    # fresh flags (:259) for the setup's capacity; the scoring settles the count first
    tot, _, rep = ctx.score_poses(cand, zx, params, np.zeros(max(cap, 1), np.uint8))
    return cand.shape[0], int(rep.best_idx), tot, cand, ctx.cells_count()


def c1_frame_oracle(pyoracle, scans, nc_lattice=1):
    """The same frame on the CPU restatement, one thread (the reference's executor)."""
    filtered = []
    for sc in scans:
        kept = pyoracle.crop_box(sc, np.array(C1_BOX))
        filtered.append(pyoracle.voxel_grid(sc[kept], C1_LEAF)[0])
    merged = np.concatenate([pyoracle.transform_rgb(f, t, q, rgb) for f, (t, q), rgb in
                             zip(filtered, C1_TFS, [(255, 0, 0), (0, 0, 255)])])
    keep, surf, area, _ = pyoracle.excavate(merged, *C1_ZX_BASE)
    terr = np.concatenate([merged[keep][:, [0, 1, 2, 4]], surf])
    xyz, cn, bbox, _ = pyoracle.excavation_grid(area, 0.1, 10, pyoracle.area_normals(area, 1.5))
    T = pyoracle.Cloud(terr)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    params = pyoracle.vl_params(num_candidates=nc_lattice)
    cand = pyoracle.generate_candidates(T, bbox, params, zx)[:1]
    flt = np.zeros((filtered[1].shape[0], 4), np.float32)
    flt[:, :3] = filtered[1]
    tot, _, rep = pyoracle.score_poses(T, pyoracle.Cloud(flt), xyz, cn, cand, zx, params,
                                       np.zeros(xyz.shape[0], np.uint8))
    return cand.shape[0], int(rep.best_idx), tot, cand, xyz.shape[0]


def run_c1(args, local, cpu: bool):
    """BASELINE configs[0]: rosbag replay, 2 x 60,032-pt scans per frame, 1 candidate pose.
    ms per frame of the GPU chain (K frames after W warm-up frames, host buffers, PCIe and
    every host round trip included) and of the oracle chain on one thread, same frame."""
    from pointcloud_processor_amd import _abi

    ctx = _abi.Context(local)
    scans = _c1_scans()
    # the smallest candidate lattice (num_candidates = 1, 4, 9, ...) in which a pose survives
    # generateCandidatePositions' filters (:550-598) on this frame; its first pose is scored
    nc_lattice = 1
    while c1_frame_gpu(ctx, scans, nc_lattice)[0] == 0 and nc_lattice < 400:
        nc_lattice = (int(math.isqrt(nc_lattice)) + 1) ** 2
    for _ in range(max(args.warmup, 1)):
        res = c1_frame_gpu(ctx, scans, nc_lattice)
    lat = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        res = c1_frame_gpu(ctx, scans, nc_lattice)
        lat.append((time.perf_counter() - t0) * 1e3)
    ctx.close()
    out = {"workload": "C1: 2 x 60,032-pt HDL-64-like scans -> filter (crop + voxel 0.2) x2 -> "
                       "merge -> carve -> normals + cell grid -> 1-candidate pose search",
           "unit": "ms/frame", "higher_is_better": False,
           "value": float(np.median(lat)), "p99_ms": float(np.percentile(lat, 99)),
           "frames": args.steps, "candidates": res[0], "best_idx": res[1],
           "num_candidates_lattice": nc_lattice,
           "data": "synthetic scans (bench._c1_scans), host buffers"}
    if cpu:
        pyoracle = _oracle()
        pyoracle.set_threads(1)
        t0 = time.perf_counter()
        frames = 0
        while frames == 0 or (time.perf_counter() - t0 < 4.0 and frames < 3):
            ref = c1_frame_oracle(pyoracle, scans, nc_lattice)
            frames += 1
        dt = (time.perf_counter() - t0) / frames
        out["cpu_baseline"] = {"value": dt * 1e3, "unit": "ms/frame", "cores": 1, "kind": "port",
                               "sample": f"{frames} frames of the same scans through the oracle "
                                         "chain (crop_box, voxel_grid, transform_rgb, excavate, "
                                         "area_normals + excavation_grid, score_poses), 1 thread"}
        # the oracle chain on its own (its own normals and cells): the same
        # candidate pose (x, y, z exact, angles <= 1 ulp), the same cells, the same best index;
        # the totals within the parity bar (tests/parity.py: glibc vs ocml acos in the score,
        # the normals are bit-identical)
        bar = _totals_bar(res[2], ref[2])
        out["matches_oracle"] = bool(
            ref[0] == res[0] and ref[1] == res[1] and ref[4] == res[4] and
            np.array_equal(ref[3][:, :3], res[3][:, :3]) and
            _ulps(ref[3][:, 3:], res[3][:, 3:]).max(initial=0) <= 1 and bar["ok"])
        out["totals_bar"] = bar
        out["best_idx_matches_oracle"] = bool(ref[1] == res[1])
        out["score_rel_diff"] = (float(np.max(np.abs(ref[2] - res[2]) / np.abs(ref[2])))
                                 if len(ref[2]) and len(res[2]) else None)
        # the margin of the argmax: (best - second) / |best| over the oracle's totals (None with
        # one candidate: C1 scores ONE pose)
        srt = np.sort(np.asarray(ref[2], np.float64))[::-1]
        out["top2_gap"] = (float((srt[0] - srt[1]) / abs(srt[0])) if srt.size >= 2 and srt[0]
                           else None)
    return out


C5_BOX = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])       # pointcloud_filter.cpp:30-36
C5_RT = ((8.0, -3.0, 2.0), (0.0, 0.0, 0.2588190451025208, 0.9659258262890683))   # replay's TFs
C5_ZT = ((0.55, 0.4, 3.5), (0.0, 0.21633, 0.0, 0.97632))


def c5_oracle_check(pyoracle, dump: Path, frame: int, best_idx: int) -> dict:
    """One dumped frame of the streamed chain re-run through the oracle chain ON ITS OWN, from
    the raw scans (every stage fed by the oracle's previous stage, never by a GPU output), and
    compared with what the node cores published: filtered clouds, merged cloud, carved terrain,
    excavation area, cells + cell normals (bits), candidate poses (xyz bits, angles 1e-12), the
    per-candidate totals (largest relative difference) and the best index."""
    pre = f"f{frame}_"

    def ld(name, dt, cols):
        return np.fromfile(dump / (pre + name), dt).reshape(-1, cols)

    ok = {}
    filt = []
    for tag, k in (("rscan", "rf"), ("zscan", "zf")):
        scan = ld(tag + ".f32", np.float32, 4)
        vox, _, _, _ = pyoracle.voxel_grid(scan[pyoracle.crop_box(scan, C5_BOX)], 0.2)
        ok[f"filtered_{k}"] = bool(np.array_equal(ld(k + ".bin", np.float32, 4)[:, :3], vox))
        filt.append(vox)
    ref = np.concatenate([pyoracle.transform_rgb(filt[0], C5_RT[0], C5_RT[1], (255, 0, 0)),
                          pyoracle.transform_rgb(filt[1], C5_ZT[0], C5_ZT[1], (0, 0, 255))])
    merged = ld("merged.bin", np.float32, 8)
    ok["merged"] = bool(merged.shape[0] == ref.shape[0] and np.array_equal(
        merged[:, :5].view(np.uint32), ref[:, :5].view(np.uint32)))
    keep, surf, area, _ = pyoracle.excavate(ref, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
    r_terr = np.concatenate([ref[keep][:, [0, 1, 2, 4]], surf])
    terr = ld("terrain.bin", np.float32, 8)
    ok["terrain"] = bool(terr.shape[0] == r_terr.shape[0] and np.array_equal(
        terr[:, [0, 1, 2, 4]].view(np.uint32), r_terr.view(np.uint32)))
    got_area = ld("area.bin", np.float32, 8)
    ok["area"] = bool(got_area.shape[0] == area.shape[0] and np.array_equal(
        got_area[:, [0, 1, 2, 4]].view(np.uint32), area.view(np.uint32)))
    r_xyz, r_cn, bb, _ = pyoracle.excavation_grid(area, 0.1, 10, pyoracle.area_normals(area, 1.5))
    cx, cn = ld("cells.f64", np.float64, 3), ld("cnrm.f32", np.float32, 3)
    ok["cells"] = bool(cx.shape == r_xyz.shape and np.array_equal(cx, r_xyz) and
                       np.array_equal(cn.view(np.uint32), r_cn.view(np.uint32)))
    T = pyoracle.Cloud(r_terr)
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])     # getZX120Position on the origin
    poses = ld("poses.f64", np.float64, 5)
    r_poses = pyoracle.generate_candidates(T, bb, pyoracle.vl_params(), zx)
    ok["candidates"] = bool(poses.shape == r_poses.shape and
                            np.array_equal(poses[:, :3], r_poses[:, :3]) and
                            _ulps(poses[:, 3:], r_poses[:, 3:]).max(initial=0) <= 1 and
                            int((_ulps(poses[:, 3:], r_poses[:, 3:]) != 0).sum()) <= 2)
    aux = np.zeros((filt[1].shape[0], 4), np.float32)
    aux[:, :3] = filt[1]
    tot, _, rep = pyoracle.score_poses(T, pyoracle.Cloud(aux), r_xyz, r_cn, r_poses, zx,
                                       pyoracle.vl_params(), np.zeros(r_xyz.shape[0], np.uint8))
    got = np.fromfile(dump / (pre + "tot.f64"), np.float64)
    top = np.sort(np.asarray(tot))[::-1]
    bar = _totals_bar(got, tot)
    ok["totals"] = bar["ok"]
    return {"frame": frame, **ok, "totals_bar": bar, "best_idx": best_idx,
            "oracle_best_idx": int(rep.best_idx),
            "best_idx_matches": best_idx == int(rep.best_idx),
            "totals_max_rel_diff": (float(np.max(np.abs(got - tot) / np.abs(tot)))
                                    if got.shape == tot.shape and tot.size else None),
            "top2_gap": float((top[0] - top[1]) / abs(top[0])) if top.size >= 2 and top[0]
            else None}


def run_c5(args, dist, world, rank, local, backend=None, frames=None, check=False):
    """BASELINE configs[4] (8 GPUs x 60k-pt streams): C5 is replicas only -- each
    rank streams its own frames through the C++ node cores (pcp_nodes_cli replay, full chain:
    filter x2 -> merge -> carve -> normals + grid -> terrain index -> pose search), nothing is
    exchanged on the data path.  value = frames/s of all replicas (each rank's frames over its
    mean frame latency, summed by one reduction at the end); p50/p99 = the worst rank's.
    check: rank 0 re-runs the first and the last dumped frame through the oracle chain on its
    own (c5_oracle_check) -- after the timed frames, outside them."""
    import subprocess
    import tempfile

    from pointcloud_processor_amd import synth

    sc = synth.terrain_scene()
    cells = synth.excavation_cells(sc.area)
    d = Path(tempfile.mkdtemp(prefix=f"pcp_c5_r{rank}_"))
    np.ascontiguousarray(sc.terrain).tofile(d / "t.f32")
    np.ascontiguousarray(cells.xyz).tofile(d / "c.f64")
    np.ascontiguousarray(cells.normals).tofile(d / "n.f32")
    bb = ",".join(repr(float(v)) for v in cells.grid_bbox)
    cli = Path(__file__).resolve().parent / "pointcloud_processor_amd" / "_lib" / "pcp_nodes_cli"
    env = dict(os.environ)
    from pointcloud_processor_amd import _abi

    ndev = _abi.device_count()
    if ndev:   # the replica's own GPU (device 0 of the child)
        env["HIP_VISIBLE_DEVICES"] = str(local % ndev)
    frames = frames or max(args.steps, 20)
    if dist is not None:
        dist.barrier()
    cmd = [str(cli), "replay", str(d / "t.f32"), str(sc.terrain.shape[0]), str(d / "c.f64"),
           str(d / "n.f32"), str(cells.xyz.shape[0]), bb, str(frames), "60032", "1"]
    if check and rank == 0:
        cmd.append(str(d))   # dump frames 0, 1, 2 and the last one
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise SystemExit(f"bench.py --mode c5: replay failed (rank {rank}): {r.stderr[-400:]}")
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    lat = np.array(res["lat_ms"])
    vals = [1e3 / float(lat.mean()), res["p50_ms"], res["p99_ms"]]
    if dist is not None:   # host-side (the control plane)
        s = dist.allreduce(np.array(vals, np.float64), "sum")
        m = dist.allreduce(np.array(vals, np.float64), "max")
        vals = [float(s[0]), float(m[1]), float(m[2])]
    out = {"metric": "C5 frames/s (full chain, replicas)", "value": vals[0], "unit": "frames/s",
           "n_gpus": world, "steps": frames, "warmup": 2, "ms_per_step": vals[1],
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "f32 points / f64 scoring", "data": "synthetic 60,032-pt HDL-64-like scans",
           "config": {"workload": "C5: 60k-pt stream per GPU, filter x2 -> merge -> carve -> "
                                  "normals + grid -> terrain index -> pose search",
                      "parallelism": f"replicas x{world}"},
           "p50_ms": vals[1], "p99_ms": vals[2], "max_ms_rank0": res.get("max_ms"),
           "p50_ms_worst_rank": vals[1], "p99_ms_worst_rank": vals[2],
           "stage_p50_ms_rank0": res.get("stage_p50_ms"),
           # the tail's make-up: rank 0's four slowest frames with their stage times
           "slowest_frames_rank0": res.get("slowest"),
           "reallocs_after_warmup": res.get("reallocs_after_warmup"),
           "candidates_best_idx_last_frame": res.get("best_idx")}
    if check and rank == 0 and res.get("dumped"):
        pyoracle = _oracle()
        pyoracle.set_threads(1)
        dumped = res["dumped"]
        out["oracle_check"] = [c5_oracle_check(pyoracle, d, fr["frame"], int(fr["best_idx"]))
                               for fr in (dumped[0], dumped[-1])]
        out["matches_oracle"] = all(all(v for k, v in c.items() if isinstance(v, bool))
                                    for c in out["oracle_check"])
    import shutil

    shutil.rmtree(d, ignore_errors=True)
    return out


def run_cells(args, dist, world, rank, local, backend=None):
    """Reference-mode scoring (runOptimization) alone: poses/s."""
    a = argparse.Namespace(**vars(args))
    a.cells_only = True   # (the fan loop still runs first: it builds the terrain copies)
    out = run_all(a, dist, world, rank, local, backend)
    rm = out["reference_mode"]
    return {"metric": "candidate poses/sec (reference cell scoring)", "value": rm["value"],
            "unit": "poses/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": rm["ms_per_step"], "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": rm["workload"]}, "best_pose": rm["best_pose"],
            "detail": rm}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--mode", choices=["all", "fan", "filter", "cells", "c1", "c4", "c5",
                                       "launch-check"],
                    default="all",
                    help="all (default): the fan line with reference-mode scoring and C3 as "
                         "extra keys; fan: the fan alone (profiling); filter: C3 with PCIe and "
                         "stage breakdown; cells: reference mode alone; c4: 4096 poses strong-"
                         "scaled over the ranks (configs[3]); c1 / c5: the streaming chain "
                         "(configs[0] / configs[4], replicas)")
    ap.add_argument("--poses-per-gpu", type=int, default=256)
    ap.add_argument("--n-az", type=int, default=1024)
    ap.add_argument("--n-el", type=int, default=256)
    ap.add_argument("--filter-points", type=int, default=10_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true",
                    help="filter mode: skip the host-buffer (PCIe-inclusive) measurement")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    args.fan_only = args.mode == "fan"
    dist, world, rank, local, backend = _dist_init(args.gpus)
    if args.mode == "launch-check":   # the launch path alone (CPU test): ranks + one collective
        t = np.array([float(rank)])
        if dist is not None:
            t = dist.allreduce(t, "sum")
        from pointcloud_processor_amd import dist as pd

        lo, hi = pd.shard(C4_POSES, world, rank)   # the C4 plan each rank would cast
        c4 = np.array([hi - lo, lo], np.int64)
        got = dist.allreduce(c4, "sum") if dist is not None else c4
        out = {"n_gpus": world, "backend": backend, "rank_sum": float(t[0]),
               "torch_in_rank_process": "torch" in sys.modules,
               "c4": {"poses_total": int(got[0]), "scaling": "strong",
                      "poses_per_rank": [h - l for l, h in
                                         (pd.shard(C4_POSES, world, r) for r in range(world))],
                      **_c4_checks(dist)}}
    elif args.mode == "filter":
        out = run_filter(args, dist, world, rank, local, backend)
    elif args.mode == "cells":
        out = run_cells(args, dist, world, rank, local, backend)
    elif args.mode == "c1":
        out = run_c1(args, local, cpu=not args.no_cpu_baseline)
    elif args.mode == "c5":
        out = run_c5(args, dist, world, rank, local, backend)
    elif args.mode == "c4":
        out = run_c4(args, dist, world, rank, local, backend)
    else:
        out = run_all(args, dist, world, rank, local, backend)
    if rank == 0 and args.mode != "launch-check":
        out["runtime"] = _runtime()
        out["runtime"] = dict(out["runtime"] or {}, torch_in_process="torch" in sys.modules)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.close()


if __name__ == "__main__":
    main()
