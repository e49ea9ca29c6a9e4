#!/bin/bash
# Round 4: packed u8 pre-pass partials (k_bucket_reduce8) vs the previous library: A/B of the 1 GiB
# build, the whole GPU suite on the new library, emulated N = 8 rank 0 on both.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS="1 2 3" LIBS="base main" bash tools/gpu_ab_lib.sh || exit $?
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4w_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4w_tests.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for v in base main; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 --pos64 \
    > gpurun_out/r4w_emul8_$v.jsonl 2> gpurun_out/r4w_emul8_$v.err || exit $?
  echo $v; cut -c1-300 gpurun_out/r4w_emul8_$v.jsonl
done
