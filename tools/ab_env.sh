#!/bin/bash
# A/B of the whole fan step (bench.py --mode fan, one process per variant, alternating rounds):
#   bash tools/ab_env.sh ROUNDS "name:ENV=V,ENV=V" ...
# prints ms_per_step and the kernel time of every run (MODE=filter|cells for the other loops)
set -u
cd "$(dirname "$0")/.."
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    name=${v%%:*}; env=${v#*:}
    out=$(env ${env//,/ } timeout -k 10 200 python bench.py --mode ${MODE:-fan} --steps 50 --warmup 5 \
          --no-cpu-baseline 2>/dev/null | grep '^{') || { echo "r$r $name FAILED"; exit 1; }
    echo "r$r $name $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("step %.4f ms  kernel %.4f ms  value %.4g" % (d["ms_per_step"], d.get("roofline", {}).get("avg_kernel_ms", float("nan")), d["value"]))')"
  done
done
