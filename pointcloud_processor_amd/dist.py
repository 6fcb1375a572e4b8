"""Pose sharding across GPUs: one process per GPU, poses partitioned
contiguously, terrain index replicated, and ONE collective per pose search:

  * fan mode      -- all-reduce(MIN) over an int64 P-vector of blocked-ray counts (the
                     reference-style occlusion score); INT64_MAX marks other ranks' poses.
  * reference mode -- all-reduce(MAX) over a float64 P-vector of total scores (-inf marks
                     other ranks' poses); every rank then runs runOptimization's strict-'>'
                     argmax (virtual_lidar.cpp:471-474) over all scores, so the best pose and
                     the candidate scores for publishCandidatePositions (:845-851) are
                     identical on every rank.

Each position of the vector is written by exactly one rank, so MIN/MAX reductions are exact
(no arithmetic on the values).  `dist_mod` is torch.distributed (gloo: the CPU tests) or a
hostgroup.HostGroup (bench.py's ranks, whose processes never import torch); the GPU data path's
collective is libpcp's own RCCL communicator (pcp_raycast_fan_allreduce).
"""
from __future__ import annotations

import numpy as np

INT64_MAX = np.iinfo(np.int64).max


def shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [lo, hi) of `total` items for `rank` (first total % world ranks get +1)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _reduce(vec: np.ndarray, op: str, dist_mod, device):
    if dist_mod is None:
        return vec
    if hasattr(dist_mod, "allreduce_np"):   # hostgroup.HostGroup (bench.py's ranks)
        return dist_mod.allreduce_np(vec, op)
    import torch

    t = torch.from_numpy(vec).to(device)
    red = dist_mod.ReduceOp.MIN if op == "min" else dist_mod.ReduceOp.MAX
    dist_mod.all_reduce(t, op=red)
    return t.cpu().numpy()


def reduce_fan(blocked_local: np.ndarray, lo: int, hi: int, total: int, dist_mod=None,
               device="cpu"):
    """-> (blocked counts of all poses, argmin with ties to the lowest index, or -1)."""
    key = np.full(total, INT64_MAX, np.int64)
    key[lo:hi] = np.asarray(blocked_local, np.int64)
    key = _reduce(key, "min", dist_mod, device)
    return key, (int(np.argmin(key)) if total else -1)


def reduce_scores(total_local: np.ndarray, lo: int, hi: int, total: int, dist_mod=None,
                  device="cpu"):
    """-> (total_score of all poses, reference strict-'>' argmax, best score or -inf)."""
    vec = np.full(total, -np.inf, np.float64)
    vec[lo:hi] = np.asarray(total_local, np.float64)
    vec = _reduce(vec, "max", dist_mod, device)
    # runOptimization :471-474: `if (total > best)` from best = -inf, so the first maximum wins
    # and no NaN or -inf total is ever taken -- np.argmax over the NaN-free values gives the
    # first occurrence of the maximum
    finite = np.where(np.isnan(vec), -np.inf, vec)
    if total == 0 or not (finite.max() > -np.inf):
        return vec, -1, -np.inf
    best_idx = int(np.argmax(finite))
    return vec, best_idx, float(finite[best_idx])
