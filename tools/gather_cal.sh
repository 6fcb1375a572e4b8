#!/bin/bash
# FETCH_SIZE calibration of divergent gathers (tools/mb/gather_fetch.hip): one plain run (launch
# times), one rocprofv3 --pmc FETCH_SIZE pass, then tools/gather_cal.py -> profiles/r04_fetch_calibration.json
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 tools/mb/gather_fetch 10 > gpurun_out/gcal_times.jsonl 2> gpurun_out/gcal_times.err || { echo "plain rc=$?"; cat gpurun_out/gcal_times.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gcal_fetch -o pmc --output-format csv -- tools/mb/gather_fetch 3 > gpurun_out/gcal_fetch.log 2>&1 || { echo "pmc rc=$?"; tail -20 gpurun_out/gcal_fetch.log; exit 1; }
python3 tools/gather_cal.py gpurun_out/gcal_times.jsonl gpurun_out/gcal_fetch profiles/r04_fetch_calibration.json
