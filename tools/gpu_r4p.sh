#!/bin/bash
# Round 4: fused-slice buffers kept across builds (per-build 34 GB allocate / free stalled some strong
# builds by 3-4 s), pairs / quads of the segmented sort without the 16-network: parity suites, the
# strong probe + line, the English-like leg, 1 GiB A/B against c1.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q -s --timeout 600 --timeout-method thread -m gpu tests \
  > gpurun_out/r4p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4p_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/strong_probe.py > gpurun_out/r4p_probe.log 2>&1 || exit $?
grep build gpurun_out/r4p_probe.log
timeout -k 10 300 python3 -u bench.py --strong --steps 5 --warmup 1 > gpurun_out/r4p_strong.json 2> gpurun_out/r4p_strong.err || exit $?
python3 -c "
import json;d=json.loads(open('gpurun_out/r4p_strong.json').read());print('strong', d['ms_per_step'])"
timeout -k 10 300 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(seed=2, leg_steps=3, wt_reps=1, patterns=100000, query_reps=1)
r = bench.english_leg(a)
print('english', r['ms_per_step'], 'refine', r['refinement_ms_per_step'], 'dbl', r['doubling_ms_per_step'],
      'rounds', r['chunk_rounds'], r['doubling_rounds'], {k: round(v['ms'] / 3, 2) for k, v in r['stages_ms_total'].items()})
" > gpurun_out/r4p_eng.log 2>&1
rc=$?; tail -2 gpurun_out/r4p_eng.log; [ $rc -eq 0 ] || exit $rc
LIBS="c1 main" REPS="1 2" bash tools/gpu_ab_lib.sh 2>&1 | tee gpurun_out/r4p_ab.log
exit ${PIPESTATUS[0]}
