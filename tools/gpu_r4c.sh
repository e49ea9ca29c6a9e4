#!/bin/bash
# Round 4: the full GPU suite on the switch-free library, then the default bench line (all legs).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests \
  > gpurun_out/r4c_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4c_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r4c_bench.json 2> gpurun_out/r4c_bench.err
rc=$?
tail -12 gpurun_out/r4c_bench.err
exit $rc
