#!/bin/bash
# After tools/r04_evidence.sh B (gpurun_out/ merged back): the round-4 PMC traffic entries with
# their source stamps and the gather-calibrated fan factor -> profiles/r04_pmc_traffic.json,
# profiles/r04_fetch_calibration.json (the calibration is parsed on the box by gather_cal.sh
# into gpurun_out's copy of profiles/; copy it over first).
set -eu
cd "$(dirname "$0")/.."
[ -f gpurun_out/gcal_times.jsonl ] && python3 tools/gather_cal.py gpurun_out/gcal_times.jsonl gpurun_out/gcal_fetch profiles/r04_fetch_calibration.json
python3 tools/pmc_traffic.py fan "k_raycast_fan_xcd" gpurun_out/pmctr04_fetch gpurun_out/pmctr04_write per_dispatch r04_pmc_traffic.json profiles/r04_fetch_calibration.json
# bench.py --mode filter --steps 3 --warmup 1 --no-pcie: 4 timed + 3 profiled + 3 eager frames
python3 tools/pmc_traffic.py filter "pcp::" gpurun_out/pmcfltr04_fetch gpurun_out/pmcfltr04_write steps=10 r04_pmc_traffic.json
