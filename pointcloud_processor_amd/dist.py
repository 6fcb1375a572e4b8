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
(no arithmetic on the values).

The GPU path's reference mode reduces a wider vector in ONE collective
(pcp_score_poses_allreduce / pcp_multi_score_poses): [P totals | P covered | 3 x C newest-pose
flag keys | health].  `score_keys` and `flags_from_keys` restate its two kernels (k_score_keys,
k_flags_from_keys in pcp_vlidar.hip) on the host, so the gloo tests can check that one rank's
vector per shard, reduced by MAX, is the single-process vector and resolves to the reference's
stale GridCell flags (virtual_lidar.cpp:480-519).  `dist_mod` is torch.distributed (gloo: the CPU tests) or a
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


# GridCell flag bits (include/pcp_abi.h PCP_F_*): zx120 range / fov / visible, then the mobile's
F_RANGE_Z, F_FOV_Z, F_VIS_Z, F_RANGE_M, F_FOV_M, F_VIS_M = 1, 2, 4, 8, 16, 32


def pose_bits(flags_after: np.ndarray) -> np.ndarray:
    """One pose's result bits per cell (range | fov << 1 | visible << 2, the kernel's mbits row)
    from the mobile flags a single-pose scoring leaves on zeroed GridCells (evaluateCellScore
    :662-687 sets fov only in range, visible only in range and fov)."""
    f = np.asarray(flags_after, np.uint8)
    return (((f & F_RANGE_M) != 0) | (((f & F_FOV_M) != 0) << 1)
            | (((f & F_VIS_M) != 0) << 2)).astype(np.uint8)


SCORE_WRITTEN = np.uint64(1 << 32)   # kScoreWritten: a covered key of a pose some rank scored


def score_keys(tot_local: np.ndarray, cov_local: np.ndarray, bits_local: np.ndarray, lo: int,
               total: int) -> np.ndarray:
    """k_score_keys restated: this rank's vector [P total bits | P covered | C range keys | C fov
    keys | C visible keys] for ALL-REDUCE(MAX).  Totals are >= +0.0, so their IEEE bits order
    like the values and 0 (= +0.0) marks other ranks' poses; a covered key is SCORE_WRITTEN | the
    count, so a pose no rank scored reduces to 0 (pcp_score_poses_allreduce reports it).  Per cell and stale-flag assignment,
    the newest pose of this shard that made it: ((global index + 1) << 1) | bit, 0 = none.
    bits_local: [n, C] pose_bits rows of the shard's poses in order."""
    tot = np.asarray(tot_local, np.float64)
    n = tot.shape[0]
    bits = np.asarray(bits_local, np.uint8).reshape(n, -1) if n else np.zeros((0, 0), np.uint8)
    C = bits.shape[1]
    v = np.zeros(2 * total + 3 * C, np.uint64)
    v[lo:lo + n] = tot.view(np.uint64)
    v[total + lo:total + lo + n] = (np.asarray(cov_local, np.int64).astype(np.uint32)
                                    .astype(np.uint64) | SCORE_WRITTEN)
    if n and C:
        g1 = (lo + np.arange(n, dtype=np.uint64) + 1) << np.uint64(1)   # (global + 1) << 1

        def newest(mask, bit):
            # the last pose q (in shard order) with mask[q, c]; 0 where none
            rev = mask[::-1]
            any_ = rev.any(axis=0)
            q = n - 1 - rev.argmax(axis=0)
            key = g1[q] | ((bits[q, np.arange(C)] >> bit) & 1).astype(np.uint64)
            return np.where(any_, key, np.uint64(0))

        v[2 * total:2 * total + C] = newest(np.ones_like(bits, bool), 0)   # every pose assigns range
        v[2 * total + C:2 * total + 2 * C] = newest((bits & 1) != 0, 1)
        v[2 * total + 2 * C:] = newest((bits & 3) == 3, 2)
    return v


def flags_from_keys(v: np.ndarray, zbits: np.ndarray, flags: np.ndarray, total: int) -> np.ndarray:
    """k_flags_from_keys restated: the caller's stale GridCell flags -> the zx120 evaluation's
    bits (evaluateZX120Only) then the newest pose's assignments from the reduced keys."""
    f = np.asarray(flags, np.uint8).astype(np.uint32).copy()
    z = np.asarray(zbits, np.uint32)
    C = f.shape[0]
    f = np.where(z & 1, f | F_RANGE_Z, f & ~np.uint32(F_RANGE_Z))
    f = np.where(z & 1, np.where(z & 2, f | F_FOV_Z, f & ~np.uint32(F_FOV_Z)), f)
    f = np.where((z & 3) == 3, np.where(z & 4, f | F_VIS_Z, f & ~np.uint32(F_VIS_Z)), f)
    for j, bitf in enumerate((F_RANGE_M, F_FOV_M, F_VIS_M)):
        k = np.asarray(v[2 * total + j * C:2 * total + (j + 1) * C], np.uint64)
        f = np.where(k != 0, np.where(k & np.uint64(1), f | bitf, f & ~np.uint32(bitf)), f)
    return f.astype(np.uint8)
