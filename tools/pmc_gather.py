"""The fan kernel's texture-path counters at THIS tree, stamped with its sources: TA / TD busy
fractions and L1 tag lookups per launch from tools/pmc_fan.sh's rocprofv3 --pmc passes ->
profiles/r05_fan_gather_path.json.  bench.py prints them as roofline.gather_path and marks them
stale (gather_path_stale) when the tree's fan sources differ from the stamp.
usage: python tools/pmc_gather.py OUT.json [fan|cells] gpurun_out/pmcf_*
(cells: reference mode's k_score_cells from tools/pmc_cells.sh's passes, stamped "cells")"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from pointcloud_processor_amd._stamps import workload_stamp  # noqa: E402

KERNELS = {"fan": "k_raycast_fan_xcd<0,",   # the production launch (MODE 0), not the stats one
           "cells": "k_score_cells<"}          # not k_score_cells_stats / _wide
args = sys.argv[2:]
WL = "fan"
if args and args[0] in KERNELS:
    WL, args = args[0], args[1:]
KERNEL = KERNELS[WL]
vals = defaultdict(list)
kname = None
for d in args:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if KERNEL in row.get("Kernel_Name", ""):
                kname = row["Kernel_Name"]
                vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
mean = {k: sum(v) / len(v) for k, v in vals.items()}
n_cu, n_xcd = 256, 8
cyc = mean["GRBM_GUI_ACTIVE"] / n_xcd   # GRBM_GUI_ACTIVE sums the XCDs' busy cycles
out = {
    "kernel": kname,
    "source_stamp": workload_stamp(WL),
    "td_busy_frac": mean["TD_TD_BUSY_sum"] / n_cu / cyc,
    "ta_busy_frac": mean["TA_TA_BUSY_sum"] / n_cu / cyc,
    "ta_addr_stalled_by_tc_frac": mean.get("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 0.0) / n_cu / cyc,
    "td_tc_stall_frac": mean.get("TD_TC_STALL_sum", 0.0) / n_cu / cyc,
    "l1_tag_lookups": mean.get("TCP_TOTAL_CACHE_ACCESSES_sum"),
    "tcp_tcc_read_req": mean.get("TCP_TCC_READ_REQ_sum"),
    "vmem_read_instructions": mean.get("SQ_INSTS_VMEM_RD"),
    "busy_cycles_per_xcd": cyc,
    "counters_mean_per_dispatch": mean,
    "dispatches_per_counter": {k: len(v) for k, v in vals.items()},
    "note": f"per launch; rocprofv3 --pmc passes of `bench.py --mode {WL}` (tools/pmc_{WL}.sh), busy "
            "fractions = *_BUSY_sum / 256 CUs / (GRBM_GUI_ACTIVE / 8 XCDs)",
}
if mean.get("SQ_WAVE_CYCLES"):
    out["wave_wait_any_frac"] = mean.get("SQ_WAIT_ANY", 0.0) / mean["SQ_WAVE_CYCLES"]
    out["wave_valu_active_frac"] = mean.get("SQ_ACTIVE_INST_VALU", 0.0) / mean["SQ_WAVE_CYCLES"]
if out["vmem_read_instructions"] and out["l1_tag_lookups"]:
    out["tags_per_vmem_instruction"] = out["l1_tag_lookups"] / out["vmem_read_instructions"]
Path(sys.argv[1]).write_text(json.dumps(out, indent=1) + "\n")
print(json.dumps({k: v for k, v in out.items() if k != "counters_mean_per_dispatch"}, indent=1))
