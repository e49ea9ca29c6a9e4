#!/bin/bash
# Round-4 evidence on the final library (the GPU suite ran on it in gpu_r4p.sh): smoke, the default bench
# line with every leg, rocprofv3 kernel stats / PMC traffic / SQ counters, strong 4 GiB N = 1, emulated
# N = 2 / 8 ranks (tools/gpu_r4_profile.sh), one-step kernel gap trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4q_smoke.log 2>&1 || exit $?
cat gpurun_out/r4q_smoke.log
TAG=r4q bash tools/gpu_r4_profile.sh || exit $?
bash tools/gpu_gap.sh > gpurun_out/r4q_gap.log 2>&1 || exit $?
tail -2 gpurun_out/r4q_gap.log
