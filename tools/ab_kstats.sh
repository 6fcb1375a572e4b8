#!/bin/bash
# kernel-time A/B over library builds, alternating rounds, under bench.py --mode ${MODE:-c1}:
#   KERNELS='k_nb_sums|k_nb_lists' bash tools/ab_kstats.sh ROUNDS DIR...
# (DIR under pointcloud_processor_amd/_lib; "." = the working tree's build).  Prints each matching
# kernel's average duration (us) per variant and round, from rocprofv3 --kernel-trace --stats
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/abk
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for d in "$@"; do
    o=gpurun_out/abk/${d//\//_}_r$r
    rm -rf "$o"
    PCP_LIB=pointcloud_processor_amd/_lib/$d/libpcp.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      -d "$o" -o run --output-format csv -- python3 bench.py --mode ${MODE:-c1} --steps ${STEPS:-20} --warmup 3 \
      --no-cpu-baseline > "$o.log" 2>&1 || { echo "r$r $d rc=$?"; exit 1; }
    python3 - "$o" "$d" "$r" <<'PY'
import csv, glob, os, re, sys
o, d, r = sys.argv[1:]
f = glob.glob(os.path.join(o, "**", "*kernel_stats.csv"), recursive=True)[0]
pat = re.compile(os.environ.get("KERNELS", "."))
out = []
for row in csv.DictReader(open(f)):
    n = row["Name"]
    if pat.search(n):
        out.append("%s %.1f" % (n.split("(")[0].replace("void ", "")[:32], float(row["AverageNs"]) / 1e3))
print("r%s %-10s" % (r, d), " | ".join(out))
PY
  done
done
