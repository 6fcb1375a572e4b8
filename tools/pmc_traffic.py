"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

Per the MI355X guide (HBM/rocprofv3 section): the two counters are collected in separate
passes; FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of
wide coalesced streaming reads (doubled below, flagged as such: the fan kernel's gathers are
an uncalibrated access width, so both the raw and the corrected read bytes are recorded).

    python tools/pmc_traffic.py KEY KERNEL_SUBSTR FETCH_DIR WRITE_DIR [per_dispatch|steps=N] [OUT]

OUT (default profiles/pmc_traffic.json): the JSON file the entry is merged into (round 3 writes
profiles/r03_pmc_traffic.json, which bench.py reads first).

per_dispatch (default): average over the matching dispatches (one kernel per launch);
steps=N: sum of every matching dispatch / N (a multi-kernel pipeline run N times).
"""
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def per_dispatch(d: Path, counter: str, substr: str):
    vals = {}
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or substr not in r["Kernel_Name"]:
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    key, substr, fdir, wdir = sys.argv[1:5]
    mode = sys.argv[5] if len(sys.argv) > 5 else "per_dispatch"
    out_name = sys.argv[6] if len(sys.argv) > 6 else "pmc_traffic.json"
    fetch = per_dispatch(Path(fdir), "FETCH_SIZE", substr)
    write = per_dispatch(Path(wdir), "WRITE_SIZE", substr)
    if not fetch or not write:
        raise SystemExit(f"no samples for {substr!r}: fetch {len(fetch)} write {len(write)}")
    if mode.startswith("steps="):
        n = int(mode.split("=")[1])
        fk, wk = sum(fetch) / n, sum(write) / n
    else:
        fk, wk = sum(fetch) / len(fetch), sum(write) / len(write)
    out_f = ROOT / "profiles" / out_name
    data = json.loads(out_f.read_text()) if out_f.exists() else {}
    data[key] = {
        "kernel": substr,
        "fetch_kib_per_launch": fk,
        "write_kib_per_launch": wk,
        "bytes_per_launch_raw": (fk + wk) * 1024.0,
        "bytes_per_launch": (2.0 * fk + wk) * 1024.0,
        "dispatches_sampled": [len(fetch), len(write)],
        "note": "HBM-side bytes from TCC EA requests (Infinity-Cache hits included); "
                "FETCH_SIZE doubled per the gfx950 correction for wide reads (uncalibrated for "
                "gathers: bytes_per_launch_raw is the uncorrected figure)",
    }
    out_f.write_text(json.dumps(data, indent=2) + "\n")
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
