#!/bin/bash
# A/B of an env toggle on the 1 GiB bench: optional parity tests (TESTS), then bench runs alternating
# AB_VAR=1 / 0 (AB_VALS to override), each printing ms/step and the per-launch ms of every stage.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 160 --timeout-method thread ${K:+-k "$K"} > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
i=0
for v in ${AB_VALS:-1 0 1 0}; do
  env $AB_VAR=$v timeout -k 10 300 python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-legs --no-cpu-baseline --no-pcie --no-eps ${BARGS} > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -5 gpurun_out/ab_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$i.json')); st=d['detail']['stages_ms_total']; print('$AB_VAR=$v', d['ms_per_step'], {k: round(v['ms']/v['launches'],3) for k, v in st.items()})"
  i=$((i+1))
done
