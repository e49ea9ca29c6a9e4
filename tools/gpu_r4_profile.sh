#!/bin/bash
# Round-4 evidence on the final tree: the default bench line (all legs), rocprofv3 kernel stats of a
# bench run, PMC HBM traffic of the roofline kernels (FETCH_SIZE / WRITE_SIZE in separate passes), SQ
# counters of the build kernels, the strong 4 GiB N = 1 line, emulated N = 2 / 8 ranks.
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${TAG:-r4k}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
echo "bench ok"; tail -8 gpurun_out/${TAG}_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-pcie --no-harness \
    > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.err || exit $?
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_pmc_$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --no-pcie --no-harness --no-eps --patterns 0 \
      > gpurun_out/${TAG}_pmc_$c.json 2> gpurun_out/${TAG}_pmc_$c.err || exit $?
  echo "$c ok"
done
KRE="bucket_sort_fast|cpart|slice_hist|slice_cpart" SQCMD="python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --no-pcie --no-harness --no-eps --patterns 0" \
  bash tools/gpu_sqpmc.sh > gpurun_out/${TAG}_sq.txt 2>&1 || { tail -5 gpurun_out/${TAG}_sq.txt; exit 1; }
echo "sq ok"
timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 > gpurun_out/${TAG}_strong.json 2> gpurun_out/${TAG}_strong.err || exit $?
echo "strong ok"
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 2 --ranks 0 > gpurun_out/${TAG}_emul2.jsonl 2> gpurun_out/${TAG}_emul2.err || exit $?
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 7 --pos64 > gpurun_out/${TAG}_emul8.jsonl 2> gpurun_out/${TAG}_emul8.err || exit $?
echo "emul ok"
