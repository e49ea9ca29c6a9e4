#!/bin/bash
# Round 4: the 4 GiB single-handle tests alone (progress on stdout), then the rest of the suite.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py 2>&1 | tee gpurun_out/r4d_scale.log
rc=${PIPESTATUS[0]}
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bucket.py tests/test_gpu_slices.py tests/test_gpu_english.py tests/test_gpu_dist.py 2>&1 | tee gpurun_out/r4d_rest.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
LIBS="base rec3 main" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4d_ab.log
exit ${PIPESTATUS[0]}
