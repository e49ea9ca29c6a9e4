#!/bin/bash
# GPU tests, radix diagnostics, the 1 GiB bench, optional rocprofv3 kernel trace.
# Stops after any crash/timeout (only pytest's "tests failed" rc=1 lets later steps proceed).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "${DIAG:-1}" = "1" ]; then
  timeout -k 10 300 python tools/radix_diag.py $((1<<30)) > gpurun_out/diag.log 2>&1
  rc=$?; echo "diag rc=$rc"; cat gpurun_out/diag.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${SHARD:-0}" = "1" ]; then
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 1 --sharded --steps 3 --warmup 1 > gpurun_out/shard.json 2> gpurun_out/shard.err
  rc=$?; echo "shard rc=$rc"; tail -3 gpurun_out/shard.err; cat gpurun_out/shard.json
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port 29512 bench.py --gpus 1 --sharded --pos64 --steps 3 --warmup 1 > gpurun_out/shard64.json 2> gpurun_out/shard64.err
  rc=$?; echo "shard64 rc=$rc"; tail -3 gpurun_out/shard64.err; cat gpurun_out/shard64.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
  rc=$?
  echo "rocprof rc=$rc"
fi
exit $rc
