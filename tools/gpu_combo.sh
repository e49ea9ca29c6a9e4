#!/bin/bash
# Selected GPU tests (TESTS, -k KEXPR), then emulated per-rank sharded builds (EMUL_ARGS) if given.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TT:-500} python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} ${KEXPR:+-k "$KEXPR"} -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/combo_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -cE "PASSED" gpurun_out/combo_tests.log; grep -E "FAILED|Error" gpurun_out/combo_tests.log | head -20
if [ $rc -ne 0 ]; then tail -50 gpurun_out/combo_tests.log; exit $rc; fi
if [ -n "$EMUL_ARGS" ]; then bash tools/gpu_emul.sh || exit $?; fi
