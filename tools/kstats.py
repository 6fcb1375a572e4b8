"""Per-kernel table of a rocprofv3 *_kernel_stats.csv: calls, average us, total per step.

    python tools/kstats.py STATS_CSV STEPS_IN_RUN
"""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
print(path)
for r in csv.DictReader(open(path)):
    name = r["Name"].split("(")[0].replace("void ", "")[:44]
    print(f"  {name:44s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:9.2f} us"
          f"  per step {float(r['TotalDurationNs']) / steps / 1e3:9.2f} us")
