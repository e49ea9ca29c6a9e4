#!/bin/bash
# Round 4: new parity tests (english-like text, host-boundary locate, single-GPU slices) then the
# strong 4 GiB N = 1 line through the library build.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_dropin.py::test_locate_batch_host_boundary tests/test_gpu_slices.py tests/test_gpu_english.py \
  > gpurun_out/r4b_tests.log 2>&1
rc=$?
tail -30 gpurun_out/r4b_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --strong --steps 3 --warmup 1 > gpurun_out/r4b_strong.json 2> gpurun_out/r4b_strong.err
rc=$?
tail -5 gpurun_out/r4b_strong.err; cut -c1-600 gpurun_out/r4b_strong.json
exit $rc
