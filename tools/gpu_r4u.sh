#!/bin/bash
# Round 4: slice pass A with half staging for slices of <= 1/6 of T' (three workgroups per CU,
# libhkcsa_h3.so): sharded parity through it, emulated N = 8 rank main vs h3, its phase stamps.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
HKCSA_LIB=$L/libhkcsa_h3.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "shard" > gpurun_out/r4u_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4u_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in main h3; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 > gpurun_out/r4u_e8_$v.jsonl 2> gpurun_out/r4u_e8_$v.err || exit $?
  python3 -c "
import json
for l in open('gpurun_out/r4u_e8_$v.jsonl'):
    r = json.loads(l); print('$v', r['nranks'], r['rank'], r['build_ms'], {k: v['ms_per_build'] for k, v in r['stages'].items() if v['ms_per_build'] > 0.3})"
done
done
HKCSA_LIB=$L/libhkcsa_h3.so HKCSA_SL_TRACE=1 timeout -k 10 300 python3 tools/shard_emulate.py --nranks 8 --ranks 0 > gpurun_out/r4u_tr.jsonl 2> gpurun_out/r4u_tr.err || exit $?
grep "trace\]" gpurun_out/r4u_tr.err | head -2
