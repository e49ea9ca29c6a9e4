#!/bin/bash
# Slice pass A iteration: the sharded parity tests, then a traced emulated N = 8 rank and the emulated
# ranks of N = 2 / 4 / 8 (per-stage times).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${K:-shard or strong or weak}" > gpurun_out/sl_tests.log 2>&1 || { tail -30 gpurun_out/sl_tests.log; exit 1; }
tail -2 gpurun_out/sl_tests.log
HKCSA_SL_TRACE=1 timeout -k 10 200 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --reps 1 --pos64 > gpurun_out/tr8.json 2> gpurun_out/tr8.err || { tail gpurun_out/tr8.err; exit 1; }
grep "trace\]" gpurun_out/tr8.err | tail -1
EMUL_ARGS="${EMUL:---nranks 2 --ranks 0;--nranks 8 --ranks 0 --pos64}" bash tools/gpu_emul.sh
