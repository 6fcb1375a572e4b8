"""The exponent bound k_cell_sums_exact relies on (csrc/pcp_excav.hip).

computeCellSurfaceNormal (virtual_lidar.cpp:301-340) adds the finite neighbours' float normals
as doubles in FLANN's order.  With E_min / E_max the smallest / largest exponent of the nonzero
components and n their count, E_min - E_max >= ceil(log2 n) - 29 makes every partial sum exact,
so every order gives the same double.  CPU check (numpy, no GPU): sums that meet the bound agree
bit for bit over many random orders; sums that break it (a component far below the largest)
are order-dependent, which is why such cells take the ordered path.
"""
import math

import numpy as np


def _bound_ok(v):
    nz = np.abs(v[v != 0]).astype(np.float32)
    if nz.size == 0:
        return True
    e = np.frexp(nz)[1] - 1          # floor(log2 |v|) for normal floats
    n = v.size
    lg = 0 if n <= 1 else math.ceil(math.log2(n))
    return int(e.min()) - int(e.max()) >= lg - 29


def _sums_over_orders(v, rng, orders=64):
    out = set()
    for _ in range(orders):
        acc = 0.0
        for x in rng.permutation(v):
            acc += float(x)
        out.add(acc)
    return out


def test_bound_holds_every_order_equal():
    rng = np.random.default_rng(5)
    for n in (3, 100, 2500):
        # unit-normal-like components, none tinier than 2^-16 of the largest
        v = rng.uniform(-1.0, 1.0, n).astype(np.float32)
        v[np.abs(v) < 2.0 ** -16] = 2.0 ** -16
        assert _bound_ok(v)
        assert len(_sums_over_orders(v, rng)) == 1


def test_bound_broken_orders_differ():
    # components 2^-53 of the largest: lost next to +-1.0, kept once those cancelled
    rng = np.random.default_rng(6)
    v = np.array([1.0, -1.0, 0.5] + [2.0 ** -53] * 12, np.float32)
    assert not _bound_ok(v)
    assert len(_sums_over_orders(v, rng)) > 1
