#!/bin/bash
# Round 4: doubling rounds skip the ISA entries they leave unchanged, sort in place when groups are small
# (sticky fall-back to the list sort), chunk rounds leave a tied suffix's BWT to its final round:
# parity suites, the English-like leg.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_slices.py tests/test_gpu_english.py tests/test_gpu_dist.py \
  tests/test_gpu_dropin.py tests/test_gpu_bucket.py > gpurun_out/r4k_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
print('tied', r['tied_after_round'])
print('launches', {k: v['launches'] for k, v in r['stages_ms_total'].items()})
" > gpurun_out/r4k_eng.log 2>&1
rc=$?; tail -3 gpurun_out/r4k_eng.log; exit $rc
