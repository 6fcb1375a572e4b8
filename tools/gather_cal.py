"""Join tools/mb/gather_fetch's launch times with its FETCH_SIZE pass ->
profiles/r04_fetch_calibration.json: per access shape and table size, the FETCH_SIZE bytes the
counter reports per 128-byte line touched (each line exactly once per launch), and the factor
that turns FETCH_SIZE into line bytes (128 / reported).  The guide calibrates k_stream16 (x2);
the gather rows calibrate the fan's probes (2 B), walk starts (4 B) and point records (12 B).

    python tools/gather_cal.py TIMES.jsonl FETCH_DIR OUT.json
"""
import csv
import json
import sys
from pathlib import Path


def main():
    times_f, fdir, out = sys.argv[1:4]
    times = [json.loads(l) for l in open(times_f) if l.startswith("{")]
    # rocprofv3 counter rows: per dispatch, in launch order; group by kernel name
    disp = {}
    for f in Path(fdir).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            key = (r["Kernel_Name"], int(r["Dispatch_Id"]))
            disp[key] = disp.get(key, 0.0) + float(r["Counter_Value"])
    sizes = sorted({t["table_bytes"] for t in times})
    rows = []
    for t in times:
        name = t["kernel"]
        ids = sorted(d for (k, d) in disp if name in k.replace(" ", ""))
        per = len(ids) // len(sizes)            # dispatches per table size (1 warm + reps)
        grp = ids[sizes.index(t["table_bytes"]) * per:(sizes.index(t["table_bytes"]) + 1) * per]
        sel = grp[1:] if len(grp) > 1 else grp   # skip the warm launch (the table's first fill)
        keyed = {d: v for (k, d), v in disp.items() if name in k.replace(" ", "")}
        fb = sum(keyed[d] for d in sel) / max(len(sel), 1) * 1024.0
        per_line = fb / t["lines"]
        rows.append({**t, "fetch_bytes_per_launch": fb, "fetch_bytes_per_line": per_line,
                     "factor_to_128B_lines": 128.0 / per_line if per_line else None,
                     "gbs_at_128B_lines": t["lines"] * 128 / (t["ms"] * 1e-3) / 1e9,
                     "dispatches": len(sel)})
    doc = {"source": "tools/mb/gather_fetch.hip + tools/gather_cal.sh (rocprofv3 --pmc FETCH_SIZE, "
                     "its own pass)",
           "rows": rows,
           "note": "every line of the table is touched exactly once per launch; FETCH_SIZE per "
                   "line reported by the counter; factor_to_128B_lines = 128 / that"}
    Path(out).write_text(json.dumps(doc, indent=2) + "\n")
    for r in rows:
        print(f"{r['kernel']:14s} T={r['table_bytes'] >> 20:5d} MiB  {r['ms']:.4f} ms  "
              f"fetch/line {r['fetch_bytes_per_line']:.1f} B  factor {r['factor_to_128B_lines']}")


if __name__ == "__main__":
    main()
