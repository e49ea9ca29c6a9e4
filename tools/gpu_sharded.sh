cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --sharded > gpurun_out/sh1.json 2> gpurun_out/sh1.err && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --sharded --pos64 > gpurun_out/sh2.json 2> gpurun_out/sh2.err; rc=$?; cat gpurun_out/sh1.json gpurun_out/sh2.json; tail -3 gpurun_out/sh2.err; exit $rc
