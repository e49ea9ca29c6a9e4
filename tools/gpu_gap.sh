#!/bin/bash
# One-step kernel trace of the 1 GiB build (rocprofv3 --kernel-trace), printed with the idle gap before
# every dispatch (tools/gap_trace.py); output gpurun_out/gap/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --patterns 0 --no-legs --no-pcie --no-eps --no-harness \
    > gpurun_out/gap.json 2> gpurun_out/gap.err || { echo "trace rc=$?"; tail -5 gpurun_out/gap.err; exit 1; }
db=gpurun_out/gap/run_kernel_trace.csv
python3 tools/gap_trace.py "$db" > gpurun_out/gap.txt && tail -60 gpurun_out/gap.txt
exit 0
