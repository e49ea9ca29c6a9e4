#!/bin/bash
# Round 4, final library (+ half-staged slice pass A for N >= 6): the whole GPU suite, smoke, the default
# bench line, emulated N = 2 / 8 ranks.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4v_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4v_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4v_smoke.log 2>&1 || exit $?
cat gpurun_out/r4v_smoke.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/r4v_bench.json 2> gpurun_out/r4v_bench.err || exit $?
tail -8 gpurun_out/r4v_bench.err
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 2 --ranks 0 > gpurun_out/r4v_emul2.jsonl 2> gpurun_out/r4v_emul2.err || exit $?
timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 7 --pos64 > gpurun_out/r4v_emul8.jsonl 2> gpurun_out/r4v_emul8.err || exit $?
cat gpurun_out/r4v_emul2.jsonl gpurun_out/r4v_emul8.jsonl | cut -c1-200
