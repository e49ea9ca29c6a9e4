#!/bin/bash
# Round 4: heavily tied lists (> 1/4 of the suffixes after the first sort) go straight to prefix doubling
# (libhkcsa_sd.so): parity suites that drive refinement / doubling through it, the English-like leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
HKCSA_LIB=$L/libhkcsa_sd.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_english.py tests/test_gpu_dist.py \
  tests/test_gpu_dropin.py > gpurun_out/r4r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4r_tests.log; [ $rc -eq 0 ] || exit $rc
for v in main sd; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('$v english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
" > gpurun_out/r4r_eng_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/r4r_eng_$v.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
done
