"""CPU check behind DESIGN.md §8 next step 3: glibc's double atan2 / acos / sin (Python's math
module calls them) against the x87 64-bit-mantissa results (numpy longdouble) rounded once to
double.  Near-total agreement means glibc rounds these correctly except in rare cases, so a
correctly rounded device version would reproduce them.  (numpy's own float64 ufuncs are not
glibc's here: they take SIMD implementations; printed for contrast.)"""
import json
import math

import numpy as np

rng = np.random.default_rng(1)
n = 300_000
y, x = rng.uniform(-50, 50, n), rng.uniform(-50, 50, n)
d = rng.uniform(0, 1, n)
t = rng.uniform(0, np.pi / 2, n)
ld = np.longdouble
res = {"samples": n,
       "atan2_glibc_vs_x87_rounded": int((np.array([math.atan2(b, c) for b, c in zip(y, x)]) !=
                                          np.arctan2(y.astype(ld), x.astype(ld)).astype(np.float64)).sum()),
       "acos_glibc_vs_x87_rounded": int((np.array([math.acos(v) for v in d]) !=
                                         np.arccos(d.astype(ld)).astype(np.float64)).sum()),
       "sin_glibc_vs_x87_rounded": int((np.array([math.sin(v) for v in t]) !=
                                        np.sin(t.astype(ld)).astype(np.float64)).sum()),
       "numpy_f64_arctan2_vs_glibc": int((np.arctan2(y, x) != np.array([math.atan2(b, c) for b, c in zip(y, x)])).sum())}
print(json.dumps(res))
