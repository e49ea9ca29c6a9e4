#!/bin/bash
# Quick GPU iteration: selected tests (T=pytest -k expr / file list), then the 1 GiB bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TT:-400} python -u -m pytest ${TESTS:-tests/test_gpu_bucket.py} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/quick_tests.log | tail -40
if [ $rc -ne 0 ]; then tail -60 gpurun_out/quick_tests.log; exit $rc; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BARGS} > gpurun_out/qbench.json 2> gpurun_out/qbench.err
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/qbench.err; cat gpurun_out/qbench.json
fi
exit $rc
