"""One C3 frame's kernel timeline from a rocprofv3 kernel trace (--kernel-trace, csv): the frames
are cut at each crop launch of cloud 0 (the first k_crop_tile after a k_bk_emit); prints the
median frame's kernels as start / end offsets from the frame's first start, in us.
  python3 tools/c3_timeline.py <dir containing *kernel_trace.csv>"""
import csv
import glob
import statistics
import sys

path = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(path)))
rows = [r for r in rows if "pcp::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
frames, cur, seen_emit = [], [], False
for r in rows:
    name = r["Kernel_Name"]
    short = name.split("(")[0].replace("void ", "").replace("pcp::", "")
    if short.startswith("k_crop_tile") and (seen_emit or not cur):
        if cur:
            frames.append(cur)
        cur, seen_emit = [], False
    if short.startswith("k_bk_emit"):
        seen_emit = True
    cur.append((short, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "")))
if cur:
    frames.append(cur)
frames = [f for f in frames if len(f) >= 4 and all(k[0].startswith("k_") for k in f)]
spans = [(max(k[2] for k in f) - min(k[1] for k in f)) / 1e3 for f in frames]
med = statistics.median(spans)
i = min(range(len(frames)), key=lambda j: abs(spans[j] - med))
t0 = min(k[1] for k in frames[i])
print(f"{len(frames)} frames, span median {med:.1f} us (min {min(spans):.1f}, max {max(spans):.1f})")
for k in frames[i]:
    print(f"  {k[0]:<24} q{k[3]:<3} {(k[1] - t0) / 1e3:7.1f} -> {(k[2] - t0) / 1e3:7.1f}  ({(k[2] - k[1]) / 1e3:5.1f})")
