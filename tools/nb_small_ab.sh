#!/bin/bash
# k_nb_lists with 16-bit LDS key indices (4 blocks per CU, default) vs 32-bit (PCP_NB_SMALL=0):
# kernel stats under bench --mode c1 and the C1 frame time, alternating
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/nbs
for r in 1 2; do
  for v in 1 0; do
    o=gpurun_out/nbs/s${v}_r$r
    rm -rf $o
    PCP_NB_SMALL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o -o run --output-format csv -- \
      python3 bench.py --mode c1 --steps 30 --warmup 3 --no-cpu-baseline > $o.log 2>&1 || { echo "r$r $v rc=$?"; exit 1; }
    python3 - $o $v $r <<'PY'
import csv, glob, json, sys
o, v, r = sys.argv[1:]
f = glob.glob(o + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {row["Name"].split("(")[0].replace("void ", ""): float(row["AverageNs"]) / 1e3 for row in csv.DictReader(open(f))}
d = [json.loads(l) for l in open(o + ".log") if l.startswith("{")][-1]
c = d.get("c1", d)
print(f"r{r} PCP_NB_SMALL={v} c1 p50 {c['value']:.4f} ms |", " | ".join(f"{k} {t:.1f}" for k, t in ks.items() if "nb_lists" in k or "nb_sums" in k))
PY
  done
done
