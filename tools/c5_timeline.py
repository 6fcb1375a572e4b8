"""Per-frame breakdown of a C5 replay trace (tools/replay_trace.sh): host API time by call,
device time by kernel, and the device idle time, averaged over the steady-state frames.
Frames are delimited by the first crop launch of each frame."""
import collections
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c5tl"
K = list(csv.DictReader(open(f"{d}/c5_kernel_trace.csv")))
A = list(csv.DictReader(open(f"{d}/c5_hip_api_trace.csv")))
K.sort(key=lambda r: int(r["Start_Timestamp"]))
A.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
starts = [int(r["Start_Timestamp"]) for r in K if "k_crop_tile" in r["Kernel_Name"]]
# crops per frame: 2 with the filter nodes called one by one, 1 composed (PCP_FRONT_FUSED=1);
# argv[2] = the replay's frames (+ 2 warm-up) to infer it
per = round(len(starts) / int(sys.argv[2])) if len(sys.argv) > 2 else 2
fr = starts[::max(per, 1)]
fr = fr[len(fr) // 3:]   # steady state
nf = len(fr) - 1
kt = collections.Counter()
kc = collections.Counter()
busy = 0
for r in K:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if fr[0] <= s < fr[-1]:
        kt[name(r)] += e - s
        kc[name(r)] += 1
        busy += e - s
at = collections.Counter()
ac = collections.Counter()
for r in A:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if fr[0] <= s < fr[-1]:
        at[r["Function"]] += e - s
        ac[r["Function"]] += 1
wall = (fr[-1] - fr[0]) / nf / 1e3
print(f"{nf} frames, {wall:.1f} us per frame wall, device busy {busy / nf / 1e3:.1f} us")
print("-- kernels per frame (count, us)")
for k, v in kt.most_common(30):
    print(f"  {k:50s} {kc[k] / nf:5.1f} {v / nf / 1e3:8.1f}")
print("-- host API per frame (count, us)")
for k, v in at.most_common(15):
    print(f"  {k:50s} {ac[k] / nf:5.1f} {v / nf / 1e3:8.1f}")
