#!/bin/bash
# Round-4 evidence on the final tree: the whole GPU suite, smoke(), then tools/gpu_r4_profile.sh (default
# bench line with every leg, rocprofv3 kernel stats, FETCH/WRITE_SIZE, SQ counters, strong 4 GiB N = 1,
# emulated N = 2 / 8 ranks) and a one-step kernel gap trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4m_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4m_smoke.log 2>&1 || exit $?
cat gpurun_out/r4m_smoke.log
TAG=r4m bash tools/gpu_r4_profile.sh || exit $?
bash tools/gpu_gap.sh > gpurun_out/r4m_gap.log 2>&1 || exit $?
tail -3 gpurun_out/r4m_gap.log
