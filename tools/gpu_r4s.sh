#!/bin/bash
# Round 4, final library (refinement hands a list still holding > 1/4 of the suffixes to prefix doubling
# after its first chunk round): the whole GPU suite, smoke, the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4s_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4s_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4s_smoke.log 2>&1 || exit $?
cat gpurun_out/r4s_smoke.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/r4s_bench.json 2> gpurun_out/r4s_bench.err || exit $?
tail -8 gpurun_out/r4s_bench.err
