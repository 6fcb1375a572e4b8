#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_nodes_cli.py -v --timeout 200 --timeout-method thread \
    -k "parity_bar or drift or score_stats or score_allreduce or exclusive_scan or knobs or without_tf" -s > gpurun_out/r6_g3_tests.log 2>&1
grep -h "census\|parity bar\|frame [0-9]\|PASS\|FAIL\|Error\|assert" gpurun_out/r6_g3_tests.log | head -80
timeout -k 10 60 tools/mb/chain > gpurun_out/r6_chain.log 2>&1 || { cat gpurun_out/r6_chain.log; exit 1; }
cat gpurun_out/r6_chain.log
timeout -k 10 300 python bench.py --mode cells --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6_cells.json 2> gpurun_out/r6_cells.err || { tail -20 gpurun_out/r6_cells.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r6_cells.json')); print(json.dumps(d['detail']['roofline'], indent=1)[:3000]); print(d['value'], d['ms_per_step'])"
