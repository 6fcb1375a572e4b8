"""One steady-state C5 frame from a replay trace (tools/replay_trace.sh) as a sequence: host API
calls (thread time) and kernels (device time), offsets in us from the frame's first crop launch.

    python tools/c5_sequence.py [TRACE_DIR] [FRAME_INDEX] [CROPS_PER_FRAME]
"""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5tl"
K = list(csv.DictReader(open(f"{d}/c5_kernel_trace.csv")))
A = list(csv.DictReader(open(f"{d}/c5_hip_api_trace.csv")))
starts = sorted(int(r["Start_Timestamp"]) for r in K if "k_crop_tile" in r["Kernel_Name"])
per = int(sys.argv[3]) if len(sys.argv) > 3 else 1   # crops per frame (2: the filters one by one)
fr = starts[::per]
i = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2] else len(fr) // 2
t0, t1 = fr[i], fr[i + 1]
# the frame's host side begins before its first kernel: take API calls from the previous
# frame's last kernel end
ev = []
for r in K:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 - 200000 <= s < t1:
        ev.append((s, e, "K", r["Kernel_Name"].split("(")[0].replace("void ", "")[:44]))
for r in A:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if r["Function"] in ("hipGetLastError", "hipSetDevice"):
        continue
    if t0 - 200000 <= s < t1:
        ev.append((s, e, "H", r["Function"]))
try:
    for r in csv.DictReader(open(f"{d}/c5_memory_copy_trace.csv")):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 - 200000 <= s < t1:
            ev.append((s, e, "C", r["Direction"].replace("MEMORY_COPY_", "")))
except FileNotFoundError:
    pass
ev.sort()
base = t0
for s, e, kind, nm in ev:
    print(f"{(s - base) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {kind} {nm}")
