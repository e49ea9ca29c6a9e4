#!/bin/bash
# Round 4: row-major grouping kernels of the refinement / doubling rounds (coalesced loads and compacted
# stores, one block scan per row): the whole GPU suite, the English-like leg, A/B c1 / main / bh (u32
# per-lane byte histogram).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4l_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
print('tied', r['tied_after_round'])
print('launches', {k: v['launches'] for k, v in r['stages_ms_total'].items()})
" > gpurun_out/r4l_eng.log 2>&1
rc=$?; tail -3 gpurun_out/r4l_eng.log; [ $rc -eq 0 ] || exit $rc
LIBS="c1 main bh" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4l_ab.log
exit ${PIPESTATUS[0]}
