set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "filter_merge or crop or voxel" --timeout 300 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { tail -30 gpurun_out/c3_tests.log; exit 1; }
tail -3 gpurun_out/c3_tests.log
for f in 1 0; do PCP_FM_FAST=$f timeout -k 10 300 python bench.py --mode filter --steps 50 --warmup 10 --no-pcie --no-cpu-baseline > gpurun_out/c3_fast$f.json 2>gpurun_out/c3_fast$f.err || exit 1; done
for f in 1 0; do PCP_FM_FAST=$f timeout -k 10 300 python bench.py --mode filter --steps 50 --warmup 10 --no-pcie --no-cpu-baseline > gpurun_out/c3b_fast$f.json 2>gpurun_out/c3b_fast$f.err || exit 1; done
cd /tmp && cd - >/dev/null
PCP_NO_GRAPHS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c3prof -o c3 --output-format csv -- python3 bench.py --mode filter --steps 20 --warmup 5 --no-pcie --no-cpu-baseline > gpurun_out/c3prof.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("c3_fast1","c3_fast0","c3b_fast1","c3b_fast0"):
    d=json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["ms_per_step"], d["roofline"]["avg_kernel_ms"], d["config"]["n_out"])
PY
