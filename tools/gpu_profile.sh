#!/bin/bash
# Round profile: the default N=1 bench line, rocprofv3 kernel stats of the same command, PMC HBM
# traffic of the roofline kernels (separate FETCH_SIZE / WRITE_SIZE passes), and the emulated
# per-rank work of the N=8 sharded build.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit $?
echo "bench ok"; cat gpurun_out/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err || exit $?
echo "stats ok"
bash tools/gpu_pmc.sh || exit $?
timeout -k 10 400 python3 tools/shard_emulate.py --nranks 8 --ranks 0 3 7 --pos64 > gpurun_out/emul8.jsonl 2> gpurun_out/emul8.err || exit $?
cat gpurun_out/emul8.jsonl
