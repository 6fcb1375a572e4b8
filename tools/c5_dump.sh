set -e
bash tools/replay.sh > /dev/null 2>&1 || true
read TN CN BB < gpurun_out/replay/args
mkdir -p gpurun_out/c5dump
timeout -k 10 100 pointcloud_processor_amd/_lib/pcp_nodes_cli replay gpurun_out/replay/t.f32 $TN gpurun_out/replay/c.f64 gpurun_out/replay/n.f32 $CN $BB 5 60032 1 gpurun_out/c5dump > gpurun_out/c5dump/out.json
