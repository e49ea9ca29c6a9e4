#!/bin/bash
# Round-3 profile set: one-step gap trace, rocprofv3 kernel stats of a short default bench, SQ counters
# of the bucket sort and the partition passes.  Each GPU step has its own time limit.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r3d
bash tools/gpu_gap.sh > gpurun_out/r3d/gap_tail.txt || { cat gpurun_out/r3d/gap_tail.txt; exit 1; }
tail -3 gpurun_out/r3d/gap_tail.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3d/stats -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/r3d/stats_bench.json 2> gpurun_out/r3d/stats_bench.err
rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/r3d/stats_bench.err; exit $rc; }
KRE="bucket_sort_fast|cpart" bash tools/gpu_sqpmc.sh > gpurun_out/r3d/sq.txt 2>&1
rc=$?; echo "sq rc=$rc"; tail -40 gpurun_out/r3d/sq.txt
exit $rc
