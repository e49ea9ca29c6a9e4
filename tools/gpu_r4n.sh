#!/bin/bash
# Round 4: large tied groups sorted alone (seg_sort_groups + sort_big_groups: only their members pass the
# radix sort) in refinement and doubling rounds — libhkcsa_hy.so (full build, new Index layout):
# parity suites through it, the English-like leg (main vs hy), 1 GiB A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
HKCSA_LIB=$L/libhkcsa_hy.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_english.py tests/test_gpu_dist.py \
  tests/test_gpu_dropin.py tests/test_gpu_bucket.py > gpurun_out/r4n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4n_tests.log; [ $rc -eq 0 ] || exit $rc
for v in main hy; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('$v english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
print('$v launches', {k: v['launches'] for k, v in r['stages_ms_total'].items()})
" > gpurun_out/r4n_eng_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/r4n_eng_$v.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="main hy" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4n_ab.log
exit ${PIPESTATUS[0]}
