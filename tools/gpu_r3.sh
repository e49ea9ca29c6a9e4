#!/bin/bash
# Round-3 GPU iteration: selected tests (TESTS / KEXPR), then emulated sharded ranks (EMUL_ARGS lines,
# ';'-separated) and optional bench lines (BENCH_ARGS lines, ';'-separated).  Every GPU step has its own
# time limit and the steps stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
# heartbeat: long host-side checks inside one test print nothing until the test ends
( while sleep 60; do date >> gpurun_out/r3_heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ -n "${TESTS}" ]; then
  timeout -k 10 ${TT:-600} python -u -m pytest ${TESTS} -m gpu -x -v --timeout ${PT:-150} --timeout-method thread \
    ${KEXPR:+-k "$KEXPR"} > gpurun_out/r3_tests.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/r3_tests.log | tail -60
  if [ $rc -ne 0 ]; then tail -80 gpurun_out/r3_tests.log; exit $rc; fi
fi
if [ -n "${EMUL_ARGS}" ]; then
  IFS=';' read -ra RUNS <<< "${EMUL_ARGS}"
  i=0
  for a in "${RUNS[@]}"; do
    HKCSA_SHARD_DEBUG=1 timeout -k 10 300 python3 tools/shard_emulate.py $a > gpurun_out/r3_emul_$i.jsonl 2> gpurun_out/r3_emul_$i.err
    rc=$?; echo "== emul $a rc=$rc"; grep -E "^\[(shard|slice)" gpurun_out/r3_emul_$i.err | head -8; cat gpurun_out/r3_emul_$i.jsonl
    [ $rc -eq 0 ] || { tail -20 gpurun_out/r3_emul_$i.err; exit $rc; }
    i=$((i+1))
  done
fi
if [ -n "${BENCH_ARGS}" ]; then
  IFS=';' read -ra RUNS <<< "${BENCH_ARGS}"
  i=0
  for a in "${RUNS[@]}"; do
    timeout -k 10 400 python3 bench.py $a > gpurun_out/r3_bench_$i.json 2> gpurun_out/r3_bench_$i.err
    rc=$?; echo "== bench $a rc=$rc"; tail -4 gpurun_out/r3_bench_$i.err; cat gpurun_out/r3_bench_$i.json
    [ $rc -eq 0 ] || { tail -30 gpurun_out/r3_bench_$i.err; exit $rc; }
    i=$((i+1))
  done
fi
exit 0
