#!/bin/bash
# Bucket-sort iteration: the bucket-build parity tests, then one traced 1 GiB step (phase cycles).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_gpu_bucket.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/qt.log 2>&1
rc=$?; tail -3 gpurun_out/qt.log; [ $rc -eq 0 ] || exit $rc
HKCSA_BS_TRACE=1 timeout -k 10 200 python bench.py --steps 1 --warmup 0 --patterns 0 --no-cpu-baseline > gpurun_out/trace.json 2> gpurun_out/trace.err
rc=$?; grep -E "trace|ms/step" gpurun_out/trace.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --patterns 0 --no-cpu-baseline > gpurun_out/qbench.json 2> gpurun_out/qbench.err
rc=$?; grep -E "ms/step" gpurun_out/qbench.err; exit $rc
