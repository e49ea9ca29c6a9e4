#!/bin/bash
# Round 4: A/B of the pre-pass variant (selection-free register scan, 2-D bucket reduce, per-digit pass B
# cursors), then its parity on the bucket / slice / parity suites.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
LIBS="main pre" REPS="1 2 3" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4h_ab.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
HKCSA_LIB=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_pre.so timeout -k 10 900 \
  python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bucket.py tests/test_gpu_slices.py \
  tests/test_gpu_parity.py > gpurun_out/r4h_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4h_tests.log; exit $rc
