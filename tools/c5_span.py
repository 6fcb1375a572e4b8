"""Per-frame device span of a C5 replay kernel trace: from the frame's crop kernel start to its
scoring's row sums (k_sum_flags) end, and the k_score_cells / k_score_finish / normals kernels'
places in it (medians over the steady-state frames).
    python3 tools/c5_span.py DIR [DIR ...]   (each with a *kernel_trace.csv)"""
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/*kernel_trace.csv")[0]
    K = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    nm = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pcp::", "")
    frames, cur = [], None
    for r in K:
        n = nm(r)
        if n.startswith("k_crop_tile"):
            cur = {"t0": int(r["Start_Timestamp"]), "k": []}
            frames.append(cur)
        if cur is not None:
            cur["k"].append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    spans, marks = [], {}
    for fr in frames[len(frames) // 3:-1]:
        t0 = fr["t0"]
        sf = [e for n, s, e in fr["k"] if n.startswith("k_sum_flags")]
        if not sf:
            continue
        spans.append((sf[-1] - t0) / 1e3)
        for n, s, e in fr["k"]:
            if n.startswith(("k_score_cells", "k_score_finish", "k_nb_lists<false", "k_nb_sums<false",
                             "k_cell_sums_exact", "k_nb_sums<true", "k_candidates", "k_lattice_compact")):
                key = n.split("<")[0] + ("<t>" if "<true" in n else "")
                marks.setdefault(key, []).append(((s - t0) / 1e3, (e - t0) / 1e3))
    print(f"{d}: {len(spans)} frames, span crop -> sum_flags end: median {statistics.median(spans):.1f} us "
          f"(min {min(spans):.1f}, max {max(spans):.1f})")
    for k, v in sorted(marks.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        print(f"    {k:24s} start {statistics.median(x[0] for x in v):7.1f}  end {statistics.median(x[1] for x in v):7.1f} us")
