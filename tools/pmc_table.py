"""Mean per-dispatch counter values of one kernel from rocprofv3 --pmc csv passes.
usage: python tools/pmc_table.py KERNEL_SUBSTRING gpurun_out/pmcf*"""
import csv
import glob
import sys
from collections import defaultdict

sub = sys.argv[1]
vals = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if sub in row.get("Kernel_Name", ""):
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:40s} {sum(v) / len(v):16.4g}  (n={len(v)})")
