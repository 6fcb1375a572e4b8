#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_nodes_cli.py -x -v --timeout 200 --timeout-method thread \
    -k "allreduce or own_communicator or score_stats or parity_bar or score_poses_matches or drift" > gpurun_out/r6_g2_tests.log 2>&1 || { tail -60 gpurun_out/r6_g2_tests.log; exit 1; }
tail -8 gpurun_out/r6_g2_tests.log
grep -h "parity bar\|frame" gpurun_out/r6_g2_tests.log | head -20
timeout -k 10 60 tools/mb/chain > gpurun_out/r6_chain.log 2>&1 || { cat gpurun_out/r6_chain.log; exit 1; }
cat gpurun_out/r6_chain.log
timeout -k 10 300 python bench.py --mode cells --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6_cells.json 2> gpurun_out/r6_cells.err || { tail -20 gpurun_out/r6_cells.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6_cells.json')); print(json.dumps(d['detail']['roofline'], indent=1)[:3000]); print(d['value'], d['ms_per_step'])"
