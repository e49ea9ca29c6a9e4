#!/bin/bash
# round-6 scratch: A/B of library variants on the English-like / protein-like legs
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/r6l_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/r6l_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
  for v in ${VARS:-c2 main}; do
    so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa_$v.so; [ $v = main ] && so=high-order-entropy-compressed-suffix-array_amd/hkcsa/_lib/libhkcsa.so
    for leg in ${LEGS:-english}; do
      HKCSA_LIB=$PWD/$so timeout -k 10 150 python bench.py --only-leg $leg --leg-steps ${LSTEPS:-3} --patterns 1000 --wt-reps 1 --query-reps 1 > gpurun_out/r6l.json 2> gpurun_out/r6l.err || { tail -5 gpurun_out/r6l.err; exit 1; }
      python3 -c "
import json;d=json.loads(open('gpurun_out/r6l.json').read());st=d['stages_ms_total'];s=d['steps']
print('$v $leg rep $rep', d['ms_per_step'], {k: round(x['ms']/s,2) for k,x in st.items() if x['ms']/s > 0.3})"
    done
  done
done
