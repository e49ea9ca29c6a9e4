#!/bin/bash
# Round 4: tie lists written in slot order by the bucket sorts (no radix sort of the list before the
# refinement): the whole GPU suite on the new library, then A/B of the 1 GiB build and of the bench
# legs (English-like 200 MiB) against the previous library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4x_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4x_tests.log; [ $rc -eq 0 ] || exit $rc
REPS="1 2" LIBS="base main" bash tools/gpu_ab_lib.sh || exit $?
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for v in base main; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-eps --no-pcie \
    --no-harness > gpurun_out/r4x_legs_$v.json 2> gpurun_out/r4x_legs_$v.err || exit $?
  echo $v; grep 'english\|sigma=4\|sigma256\|printable' gpurun_out/r4x_legs_$v.err | cut -c1-200
done
