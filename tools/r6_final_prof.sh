#!/bin/bash
# round-6 evidence on the final tree: the default bench command under rocprofv3 --kernel-trace --stats (its
# JSON line and the per-kernel summary), then a steady-state tools/kprof.py of the 1 GiB step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r6f}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_rocprof -o run -- \
  python3 bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_under_rocprof.json 2> gpurun_out/${T}_bench_under_rocprof.err
rc=$?; echo "rocprof bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cut -c1-200 gpurun_out/${T}_bench_under_rocprof.json
if [ -n "$KPROF" ]; then
  timeout -k 10 1000 python3 tools/kprof.py --tag ${T}k --limit 150 -- python3 bench.py --steps 5 --warmup 1 --no-legs \
    --no-cpu-baseline --no-pcie --no-harness --no-eps --patterns 1000000 --query-reps 2 --wt-reps 1 > gpurun_out/${T}k_kprof.log 2>&1
  rc=$?; echo "kprof rc=$rc"; head -4 gpurun_out/${T}k_kprof.log | cut -c1-300
fi
exit $rc
