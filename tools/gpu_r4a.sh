#!/bin/bash
# Round 4, first GPU call: the new natural-language-like parity tests and the host-boundary locate.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dropin.py::test_locate_batch_host_boundary tests/test_gpu_english.py \
  > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r4a_tests.log
exit $rc
