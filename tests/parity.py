"""The parity bars of the scoring, at what the kernels achieve (the census
profiles/r04_ulp_census.log: 3-5 % of the per-pose totals differ from the oracle's glibc acos /
sin scoring, by at most 2 ulps (5 of 32 on test_excavation_area_node's small tick); candidate angles bit-identical but for glibc's own near-tie
misroundings, 2 of 7,090).  Shared by the GPU parity tests and the node tests."""
import math

import numpy as np

TOTAL_MAX_ULPS = 4          # per total: twice the census's largest gap
# totals not bit-identical: the census's 3-5 % on the 91-1,418-candidate ticks, up to 5 of 32
# (16 %) on the small area test's tick -- a one-ulp error of every cell score moves nearly all
TOTAL_DIFFER_FRAC = 0.25


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
            "allowed_differ": max(2, math.ceil(TOTAL_DIFFER_FRAC * got.size))}


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
