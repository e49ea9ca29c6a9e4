#!/bin/bash
# Round-2 bench sweep: default N=1 line (with the sigma=256 / printable legs and the CPU baseline),
# the N=1 sharded path with replicas + locate, and the configs[4] strong-scaling N=1 point (4 GiB).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps 20 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python3 bench.py --sharded --steps 5 --warmup 1 > gpurun_out/sharded1.json 2> gpurun_out/sharded1.err || { echo "sharded rc=$?"; tail -20 gpurun_out/sharded1.err; exit 1; }
cat gpurun_out/sharded1.json
timeout -k 10 400 python3 bench.py --strong --steps 2 --warmup 1 --patterns 0 > gpurun_out/strong1.json 2> gpurun_out/strong1.err || { echo "strong rc=$?"; tail -20 gpurun_out/strong1.err; exit 1; }
cat gpurun_out/strong1.json
