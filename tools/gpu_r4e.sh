#!/bin/bash
# Round 4: quick parity of the packed path (bucket tests), the 3-way library A/B, then the long tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bucket.py tests/test_gpu_slices.py 2>&1 | tee gpurun_out/r4e_quick.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
LIBS="base rec3 main" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4e_ab.log
rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_scale.py tests/test_gpu_english.py 2>&1 | tee gpurun_out/r4e_scale.log
exit ${PIPESTATUS[0]}
