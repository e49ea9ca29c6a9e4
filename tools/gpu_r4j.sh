#!/bin/bash
# Round 4: adaptive refinement (early hand-over to prefix doubling, direct radix sort for large groups,
# settled-only SA / BWT writes in doubling rounds) + pass A keys without boundary tests on whole tiles:
# parity of every GPU suite but the 4 GiB ones, the English-like leg (main vs c1), 1 GiB A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_english.py tests/test_gpu_dist.py \
  tests/test_gpu_dropin.py tests/test_gpu_bucket.py > gpurun_out/r4j_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j_tests.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib
for v in c1 main; do
  lib=$L/libhkcsa_$v.so; [ "$v" = main ] && lib=$L/libhkcsa.so
  HKCSA_LIB=$lib timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('$v english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
print('$v tied', r['tied_after_round'])
" > gpurun_out/r4j_eng_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/r4j_eng_$v.log; [ $rc -eq 0 ] || exit $rc
done
LIBS="c1 main" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4j_ab.log
exit ${PIPESTATUS[0]}
