#!/bin/bash
# Round 4: slot-ordered tie lists (wave 0 ranks the ties; no extra workgroup
# barriers): A/B of the 1 GiB build against the previous library, then the bucket / refinement tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS="1 2 3" LIBS="base main" bash tools/gpu_ab_lib.sh || exit $?
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_bucket.py tests/test_gpu_english.py > gpurun_out/r4y_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4y_tests.log; exit $rc
