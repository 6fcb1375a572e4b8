# C3 frame A/B over environments, alternating processes (ROUNDS):
#   bash tools/c3_env_ab.sh "name:ENV=V,ENV=V" ...
set -u
cd "$(dirname "$0")/.."
ROUNDS=${ROUNDS:-3}
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env ${envs//,/ } timeout -k 10 200 python3 bench.py --mode filter --steps 30 --warmup 5 --no-pcie --no-cpu-baseline > gpurun_out/c3ab_$name.json 2>gpurun_out/c3ab_$name.err || exit 1
    python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/c3ab_$name.json') if l.startswith('{')][-1]; c=d.get('c3', d)
print('r$r $name ms %.4f dev %.4f' % (c['ms_per_step'], c['roofline']['avg_kernel_ms']))"
  done
done
