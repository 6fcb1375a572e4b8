"""Join tools/mb/gather_ceiling's JSON lines into profiles/r05_gather_ceiling.json: per lane width
(2, 4, 12 bytes: the fan's probes, walk starts, point records) the highest chip-wide rate of
divergent lane-loads measured over the table sizes and chains per lane -- the ceiling bench.py's
fan roofline divides by -- with the clock the chip held and every run kept beside it.
usage: python tools/gather_ceiling.py RUNS.jsonl OUT.json [PMC_DIR]
PMC_DIR: rocprofv3 --pmc pass of `gather_ceiling 2` (3 dispatches per run, the same run order):
each run gets its TA / TD busy fractions, L1 tags per load instruction and L1 miss fraction."""
import csv
import hashlib
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "tools" / "mb" / "gather_ceiling.hip"

runs = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
if len(sys.argv) > 3:
    disp = defaultdict(dict)
    for f in Path(sys.argv[3]).rglob("*counter_collection.csv"):
        for row in csv.DictReader(open(f)):
            if "k_gather_chain" in row["Kernel_Name"]:
                disp[int(row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
    ids = sorted(disp)
    if len(ids) == 3 * len(runs):
        for i, r in enumerate(runs):
            d = [disp[j] for j in ids[3 * i + 1:3 * i + 3]]   # the two timed dispatches
            m = {k: sum(x[k] for x in d) / len(d) for k in d[0]}
            cyc = m["GRBM_GUI_ACTIVE"] / 8   # per XCD
            n_cu = r["cus"]
            vm = r["waves"] * r["chains_per_lane"] * 256   # load instructions per dispatch
            r["pmc"] = {"ta_busy_frac": m["TA_TA_BUSY_sum"] / n_cu / cyc,
                        "td_busy_frac": m["TD_TD_BUSY_sum"] / n_cu / cyc,
                        "l1_tags_per_load_instruction": m["TCP_TOTAL_CACHE_ACCESSES_sum"] / vm,
                        "l1_miss_frac": m["TCP_TCC_READ_REQ_sum"] /
                        max(m["TCP_TOTAL_CACHE_ACCESSES_sum"], 1.0)}
    else:
        print(f"pmc: {len(ids)} dispatches for {len(runs)} runs: not joined", file=sys.stderr)
best = {}
for r in runs:
    w = str(r["lane_bytes"])
    if w not in best or r["lane_loads_per_s"] > best[w]["lane_loads_per_s"]:
        best[w] = r
out = {
    "what": "chip-wide divergent lane-loads per second on gfx950 for the fan kernel's load "
            "shape: one wave per workgroup, 8 waves per SIMD, each lane's load at the start of "
            "a pseudo-random 128-B line, the next address depending on the loaded value "
            "(dependent chains, 1 or 4 per lane), 64 or 24 active lanes, tables of 8 / 16 KiB "
            "(L1-resident, ~1.6 / ~1.3 lanes per line as in the fan), 2 MiB (L2), 16 / 96 MiB "
            "(Infinity Cache); the ceiling of a width = its best run",
    "source": "tools/mb/gather_ceiling.hip (tools/gather_ceiling.sh)",
    "source_sha16": hashlib.sha256(SRC.read_bytes()).hexdigest()[:16],
    "ceiling_lane_loads_per_s": {w: b["lane_loads_per_s"] for w, b in sorted(best.items())},
    "ceiling_run": best,
    "clock_mhz_median_over_runs": sorted(r["clock_mhz"] for r in runs)[len(runs) // 2],
    "model": "bench.py _fan_roofline: peak = the fan's lane-loads per launch / sum over widths "
             "of (its lane-loads of that width / the width's ceiling); frac = lane-loads / "
             "kernel time / peak",
    "runs": runs,
}
Path(sys.argv[2]).write_text(json.dumps(out, indent=1) + "\n")
for r in runs:
    p = r.get("pmc", {})
    print(f"W={r['lane_bytes']:>2} C={r['chains_per_lane']} A={r['active_lanes']:>2} "
          f"T={r['table_bytes'] >> 10:>6} KiB: {r['lane_loads_per_s']:.3e}/s "
          f"{r['per_cu_per_cycle']:.3f}/CU/cyc @{r['clock_mhz']:.0f} MHz "
          f"TA {p.get('ta_busy_frac', float('nan')):.2f} TD {p.get('td_busy_frac', float('nan')):.2f} "
          f"tags/instr {p.get('l1_tags_per_load_instruction', float('nan')):.1f} "
          f"L1 miss {p.get('l1_miss_frac', float('nan')):.2f}")
for w, b in sorted(best.items()):
    print(f"ceiling W={w:>2}: {b['lane_loads_per_s']:.4e} lane-loads/s ({b['per_cu_per_cycle']:.3f} "
          f"per CU and cycle at {b['clock_mhz']:.0f} MHz; table {b['table_bytes'] >> 10} KiB, "
          f"{b['chains_per_lane']} chains/lane, {b['active_lanes']} active lanes)")
