"""Multi-process (world_size 2, gloo on CPU) coverage of the pose-sharded search: each rank
scores its contiguous shard and ONE all-reduce yields the same best pose and score vector as a
single process over all poses.  The per-rank scorer stands in for the GPU
kernel: the oracle (CPU restatement) of the fan march / cell scoring on the golden mini scene.

torch is imported only inside the spawned ranks: the test process itself has loaded libpcp
(conftest.py), and a PyTorch wheel's bundled HIP / HSA stack must not join it (hostgroup.py).
"""
import importlib.util
import multiprocessing as mp
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

if importlib.util.find_spec("torch") is None:
    pytest.skip("torch not installed", allow_module_level=True)

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pose_bits(pyoracle, Ts, A, s, poses, vp):
    """[n, C] result bits of each pose alone on zeroed GridCells (the kernel's mbits rows)"""
    from pointcloud_processor_amd import dist as pd

    rows = []
    for q in range(poses.shape[0]):
        f = np.zeros(s["cells"].shape[0], np.uint8)
        pyoracle.score_poses(Ts, A, s["cells"], s["normals"], poses[q:q + 1], s["zx"], vp, f)
        rows.append(pd.pose_bits(f))
    return np.array(rows, np.uint8).reshape(poses.shape[0], s["cells"].shape[0])


def _worker(rank, world, port, out_q):
    import torch.distributed as dist

    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pyoracle

        from pointcloud_processor_amd import dist as pd

        d = np.load(GOLD / "fan.npz")
        T = pyoracle.Cloud(d["terrain"])
        poses = np.concatenate([d["poses"], d["poses"][:, :] + [0.3, -0.2, 0.0, 0.0, 0.5]])
        P = poses.shape[0]
        lo, hi = pd.shard(P, world, rank)
        b, _, _ = pyoracle.raycast_fan(T, poses[lo:hi], int(d["n_az"]), int(d["n_el"]),
                                       float(d["el_min"]), float(d["el_max"]),
                                       float(d["max_distance"]), want_first_hit=False)
        keys, best = pd.reduce_fan(b, lo, hi, P, dist, "cpu")
        s = np.load(GOLD / "score.npz")
        Ts, A = pyoracle.Cloud(s["terrain"]), pyoracle.Cloud(s["aux"])
        cand = s["candidates"]
        lo2, hi2 = pd.shard(cand.shape[0], world, rank)
        flags = np.zeros(s["cells"].shape[0], np.uint8)
        vp = pyoracle.vl_params(max_distance=float(s["max_distance"]))
        tot, cov, _ = pyoracle.score_poses(Ts, A, s["cells"], s["normals"], cand[lo2:hi2], s["zx"],
                                           vp, flags)
        vec, bidx, bscore = pd.reduce_scores(tot, lo2, hi2, cand.shape[0], dist, "cpu")
        # the GPU path's one reference-mode collective (pcp_score_poses_allreduce), restated:
        # this shard's key vector, all-reduced by MAX (int64 view: every key is below 2^63)
        bits = _pose_bits(pyoracle, Ts, A, s, cand[lo2:hi2], vp)
        v = pd.score_keys(tot, cov, bits, lo2, cand.shape[0])
        red = pd._reduce(v.view(np.int64), "max", dist, "cpu").view(np.uint64)
        out_q.put((rank, keys, best, vec, bidx, bscore, red))
    finally:
        dist.destroy_process_group()


def test_shard_partition():
    from pointcloud_processor_amd import dist as pd

    for total in (0, 1, 7, 256, 4096, 4097):
        for world in (1, 2, 3, 8):
            parts = [pd.shard(total, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
            sizes = [h - l for l, h in parts]
            assert max(sizes) - min(sizes) <= 1


def test_reduce_single_process_semantics():
    from pointcloud_processor_amd import dist as pd

    keys, best = pd.reduce_fan(np.array([5, 3, 3, 9]), 0, 4, 4)
    assert best == 1                                  # ties -> lowest index
    vec, bidx, bs = pd.reduce_scores(np.array([1.0, 4.0, 4.0, 2.0]), 0, 4, 4)
    assert bidx == 1 and bs == 4.0                    # strict '>' keeps the first maximum
    vec, bidx, bs = pd.reduce_scores(np.zeros(0), 0, 0, 0)
    assert bidx == -1 and bs == -np.inf


def test_two_rank_gloo_matches_single_process():
    import pyoracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference over all poses
    d = np.load(GOLD / "fan.npz")
    T = pyoracle.Cloud(d["terrain"])
    poses = np.concatenate([d["poses"], d["poses"][:, :] + [0.3, -0.2, 0.0, 0.0, 0.5]])
    b, _, _ = pyoracle.raycast_fan(T, poses, int(d["n_az"]), int(d["n_el"]), float(d["el_min"]),
                                   float(d["el_max"]), float(d["max_distance"]),
                                   want_first_hit=False)
    s = np.load(GOLD / "score.npz")
    from pointcloud_processor_amd import dist as pd

    Ts, A = pyoracle.Cloud(s["terrain"]), pyoracle.Cloud(s["aux"])
    vp = pyoracle.vl_params(max_distance=float(s["max_distance"]))
    cand = s["candidates"]
    P, C = cand.shape[0], s["cells"].shape[0]
    f_all = np.zeros(C, np.uint8)
    tot1, cov1, _ = pyoracle.score_poses(Ts, A, s["cells"], s["normals"], cand, s["zx"], vp, f_all)
    v1 = pd.score_keys(tot1, cov1, _pose_bits(pyoracle, Ts, A, s, cand, vp), 0, P)
    fz = np.zeros(C, np.uint8)   # evaluateZX120Only alone: the zx120 bits
    pyoracle.score_poses(Ts, A, s["cells"], s["normals"], cand[:0], s["zx"], vp, fz)
    for rank, keys, best, vec, bidx, bscore, red in res:
        np.testing.assert_array_equal(keys, b.astype(np.int64))
        assert best == int(np.argmin(b))
        np.testing.assert_array_equal(vec, s["total"])     # golden: one process, all poses
        assert bidx == int(s["report"][0])
        assert bscore == float(s["best_score"])
        # the reference-mode key vector: the shards' MAX is the one-process vector, and it
        # resolves to the reference's stale flags from a fresh GridCell state
        np.testing.assert_array_equal(red, v1)
        np.testing.assert_array_equal(red[:P].view(np.float64), s["total"])
        np.testing.assert_array_equal(red[P:2 * P] & np.uint64(0xFFFFFFFF), s["covered"])
        assert np.all(red[P:2 * P] & pd.SCORE_WRITTEN)      # every pose scored by some rank
        np.testing.assert_array_equal(pd.flags_from_keys(red, fz & 7, np.zeros(C, np.uint8), P),
                                      f_all)
        np.testing.assert_array_equal(f_all, s["flags"])


@pytest.mark.parametrize("n", [2, 3])
def test_bench_self_launch(n):
    """`bench.py --gpus N` with no launcher starts N ranks itself (one process per GPU): the
    line reports n_gpus = N and one collective over all ranks ran (gloo here, no GPU)."""
    import json
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(n),
                        "--mode", "launch-check"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["rank_sum"] == n * (n - 1) / 2
    assert out["torch_in_rank_process"] is False   # the control plane lives in the helper
    # configs[3]: 4096 poses strong-scaled over the N ranks (not 256 per GPU)
    assert out["c4"]["poses_total"] == 4096 and out["c4"]["scaling"] == "strong"
    assert sum(out["c4"]["poses_per_rank"]) == 4096 and len(out["c4"]["poses_per_rank"]) == n
    # a SCALE line's c4 checks itself: per-rank kernel times and their
    # spread, the collective's time, the ranks RCCL saw (none in the gloo rehearsal), the runtime
    c4 = out["c4"]
    for k in ("kernel_ms_per_rank", "kernel_ms_max", "kernel_ms_min", "collective_ms",
              "rccl_nranks", "runtime"):
        assert k in c4, k
    assert len(c4["kernel_ms_per_rank"]) == n
    assert c4["rccl_nranks"] == 0 and c4["collective_ms"] is None
    assert c4["runtime"] is None or "hip_runtime_version" in c4["runtime"]


def test_bench_rejects_mismatched_world():
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2",
                        "--mode", "launch-check"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
def test_bench_rccl_one_rank_gpu():
    """The SCALE path's own code on the GPU at one rank (PCP_DIST_FORCE=1): the host group,
    libpcp's RCCL communicator (pcp_comm_init_rank over the id the group hands out) and the
    one-collective fan query every step; the line names RCCL with one rank, and the reduced
    vector's argmin is the plain query's best pose (the same seeded workload, no collective)."""
    import json
    import subprocess

    def run(extra):
        env = {k: v for k, v in os.environ.items() if k != "MASTER_PORT"}
        env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", **extra)
        r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--mode",
                            "fan", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"],
                           capture_output=True, text=True, env=env, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])

    dist_line = run({"PCP_DIST_FORCE": "1"})
    col = dist_line["collective"]
    assert col["backend"].startswith("rccl") and col["rccl_nranks"] == 1
    assert col["collective_ms"] is None or col["collective_ms"] >= 0.0
    assert dist_line["runtime"]["torch_in_process"] is False
    plain = run({})
    assert plain["collective"] is None
    assert dist_line["best_pose"] == plain["best_pose"]
