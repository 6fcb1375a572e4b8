#!/bin/bash
# On a one-GPU box: the C5 replicas line at N = 1 and N = 2 (both replicas on the one GPU, gloo for
# the final reduction) and the default line at N = 2 (gloo rehearsal of the pose-sharded step).
set -u
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode c5 --steps 100 > gpurun_out/c5_n1.json 2> gpurun_out/c5_n1.err || { tail gpurun_out/c5_n1.err; exit 1; }
cat gpurun_out/c5_n1.json
timeout -k 10 300 python bench.py --gpus 2 --mode c5 --steps 100 > gpurun_out/c5_n2.json 2> gpurun_out/c5_n2.err || { tail gpurun_out/c5_n2.err; exit 1; }
cat gpurun_out/c5_n2.json
timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { tail gpurun_out/bench_n2.err; exit 1; }
head -c 600 gpurun_out/bench_n2.json
