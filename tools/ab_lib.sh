# A/B two library builds on one box: alternating processes
set -u
for r in 1 2; do
  for lib in pointcloud_processor_amd/_lib/alt_head/libpcp.so pointcloud_processor_amd/_lib/libpcp.so; do
    echo "== $lib round $r"
    PCP_LIB=$lib timeout -k 10 200 python tools/fan_ab.py fine:PCP_FAN_BATCH=0 xcd:PCP_FAN_BATCH=4 2>&1 | grep -v amdgpu.ids | head -3 || exit 1
  done
done
