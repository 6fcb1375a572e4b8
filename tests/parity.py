"""The parity bars of the scoring, at what the kernels achieve (the census
profiles/r04_ulp_census.log: 3-5 % of the per-pose totals differ from the oracle's glibc acos /
sin scoring, by at most 2 ulps (5 of 32 on test_excavation_area_node's small tick); candidate angles bit-identical but for glibc's own near-tie
misroundings, 2 of 7,090).  Shared by the GPU parity tests and the node tests."""
import math

import numpy as np

TOTAL_MAX_ULPS = 2          # per total
# totals not bit-identical: round 6 scores with correctly rounded acos / sin (pcp_crmath.h), as
# glibc rounds them but for rare near ties -- 0 of 91 totals differ on the 91-candidate tick and
# on the C5 frames (with ocml's acos / sin it was 2-20 %).  At most 5 % (at least 2) may differ;
# the bar fails a one-ulp error of every cell score (make perturb: 61 of 91) and of every 8th
# cell's (make perturb8: 10 of 91) -- test_parity_bar_catches_one_ulp.  The per-cell bar below
# sees the same drifts cell by cell.
TOTAL_DIFFER_FRAC = 0.05
TOTAL_DIFFER_FLOOR = 2


def ulps(a, b) -> np.ndarray:
    """Distance in units in the last place between float64 arrays (0 = same bits; +0 / -0 equal)."""
    def key(x):
        u = np.asarray(x, np.float64).view(np.int64)
        return np.where(u < 0, np.int64(-2**63) - u, u)   # monotone in the value
    a, b = np.broadcast_arrays(np.atleast_1d(np.asarray(a, np.float64)),
                               np.atleast_1d(np.asarray(b, np.float64)))
    return np.abs(key(a).astype(object) - key(b).astype(object)).astype(np.float64)


def totals_report(got, ref) -> dict:
    got, ref = np.asarray(got, np.float64).ravel(), np.asarray(ref, np.float64).ravel()
    assert got.shape == ref.shape, (got.shape, ref.shape)
    d = ulps(got, ref) if got.size else np.zeros(0)
    return {"n": int(got.size), "max_ulps": float(d.max()) if d.size else 0.0,
            "differ": int((d != 0).sum()),
            "allowed_differ": max(TOTAL_DIFFER_FLOOR, math.ceil(TOTAL_DIFFER_FRAC * got.size))}


def totals_match(got, ref) -> bool:
    r = totals_report(got, ref)
    return r["max_ulps"] <= TOTAL_MAX_ULPS and r["differ"] <= r["allowed_differ"]


def assert_totals(got, ref):
    r = totals_report(got, ref)
    assert r["max_ulps"] <= TOTAL_MAX_ULPS and r["differ"] <= r["allowed_differ"], r


ANGLE_DIFFER_MAX = 2        # candidate pitch / yaw values not bit-identical to glibc's


def assert_angles(got, ref):
    """Candidate pitch / yaw: at most ANGLE_DIFFER_MAX values differ, each by one ulp."""
    d = ulps(got, ref)
    assert d.max(initial=0) <= 1 and int((d != 0).sum()) <= ANGLE_DIFFER_MAX, \
        (int((d != 0).sum()), d.max(initial=0))


# per-cell bar (evaluateCellScore values, test_parity_bar_per_cell / the C5 frames): glibc's
# near-tie misroundings leave 0.16-0.17 % of the positive cell scores off by 1-4 ulps (round 6,
# both ways, 2:1 downward); at most 1 % may differ, by at most 8 ulps each.  make perturb8 moves
# 12.5 % of the cells, make perturb all of them.
CELL_MAX_ULPS = 8
CELL_DIFFER_FRAC = 0.01


def cell_bar(census: dict) -> bool:
    return (census["max_ulps"] <= CELL_MAX_ULPS
            and census["differ"] <= max(5, CELL_DIFFER_FRAC * census["positive"]))
