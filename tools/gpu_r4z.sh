#!/bin/bash
# Round 4, library with slot-ordered tie lists: the whole GPU suite, smoke, the default bench line, the
# one-step kernel trace with host gaps, emulated N = 8 rank 0.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4z_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4z_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z_smoke.log 2>&1 || exit $?
cat gpurun_out/r4z_smoke.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.err || exit $?
tail -8 gpurun_out/r4z_bench.err
bash tools/gpu_gap.sh > gpurun_out/r4z_gap.log 2>&1 || exit $?
tail -2 gpurun_out/r4z_gap.log
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 > gpurun_out/r4z_emul8.jsonl 2> gpurun_out/r4z_emul8.err || exit $?
cut -c1-200 gpurun_out/r4z_emul8.jsonl
