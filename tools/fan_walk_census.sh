set -e
cd /root/repo
PCP_LIB=pointcloud_processor_amd/_lib/census/libpcp.so timeout -k 10 300 python3 -u tools/fan_walk_census.py > gpurun_out/fan_walk_census.json
cat gpurun_out/fan_walk_census.json
