"""Per-kernel HBM-side bytes of a FETCH_SIZE / WRITE_SIZE pass pair (tools/pmc_filter_traffic.sh
layout): mean per dispatch, FETCH_SIZE x the fetch factor (2 for 16-B/lane streaming reads,
MI355X_MICROARCH.md) + WRITE_SIZE.  python3 tools/pmc_by_kernel.py FETCH_DIR WRITE_DIR [factor]"""
import collections
import csv
import sys


def load(path, cname):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == cname:
            d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(float(r["Counter_Value"]))
    return d


fdir, wdir = sys.argv[1], sys.argv[2]
factor = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
f = load(f"{fdir}/pmc_counter_collection.csv", "FETCH_SIZE")
w = load(f"{wdir}/pmc_counter_collection.csv", "WRITE_SIZE")
total = 0.0
for k in sorted(set(f) | set(w)):
    fm = sum(f[k]) / max(len(f[k]), 1) * 1024 * factor / 1e6
    wm = sum(w[k]) / max(len(w[k]), 1) * 1024 / 1e6
    total += fm + wm
    print("%-28s dispatches %3d  fetch (x%.0f) %7.1f MB  write %6.1f MB" % (k, len(f[k]), factor, fm, wm))
print("total per frame %.1f MB" % total)
