#!/bin/bash
# parse tools/r06_evidence.sh output (gpurun_out/) into profiles/ (round 6)
set -eu
cd "$(dirname "$0")/.."
python3 tools/pmc_gather.py profiles/r06_fan_gather_path.json fan gpurun_out/pmcfr06_[1-5] > /dev/null
python3 tools/pmc_gather.py profiles/r06_cells_gather_path.json cells gpurun_out/pmccr06_[1-5] > /dev/null
rm -f profiles/r06_pmc_traffic.json
python3 tools/pmc_traffic.py fan "k_raycast_fan_xcd<0," gpurun_out/pmctr06_fetch gpurun_out/pmctr06_write per_dispatch r06_pmc_traffic.json profiles/r04_fetch_calibration.json > /dev/null
python3 tools/pmc_traffic.py filter "pcp::" gpurun_out/pmcfltr06_fetch gpurun_out/pmcfltr06_write steps=10 r06_pmc_traffic.json > /dev/null
python3 tools/pmc_traffic.py cells "k_score_cells<" gpurun_out/pmccr06_fetch gpurun_out/pmccr06_write per_dispatch r06_pmc_traffic.json > /dev/null
st=$(python3 -c "import json; print(json.load(open('profiles/r06_pmc_traffic.json'))['filter']['source_stamp'])")
{ echo "# C3 frame (2 x 5 M points) per kernel, the r06 PMC passes of profiles/r06_pmc_traffic.json (stamp $st): python3 tools/pmc_by_kernel.py gpurun_out/pmcfltr06_fetch gpurun_out/pmcfltr06_write"
  python3 tools/pmc_by_kernel.py gpurun_out/pmcfltr06_fetch gpurun_out/pmcfltr06_write; } > profiles/r06_c3_traffic_by_kernel.txt
cp gpurun_out/prof_c3/run_kernel_stats.csv profiles/r06_c3_kernel_stats.csv
python3 tools/c5_timeline.py gpurun_out/c5tl 32 > profiles/r06_c5_timeline.txt
python3 -c "
import json
d=json.load(open('profiles/r06_pmc_traffic.json'))
print({k: (round(v['bytes_per_launch']/1e6,1), v['source_stamp']) for k,v in d.items()})
for f in ('fan','cells'):
    g=json.load(open(f'profiles/r06_{f}_gather_path.json')); print(f, g['source_stamp'], round(g['td_busy_frac'],3), round(g['wave_wait_any_frac'],3))
"
head -3 profiles/r06_c5_timeline.txt
