#!/bin/bash
# Full GPU suite, then the 1 GiB bench with an env toggle on / off twice (AB_VAR=NAME).
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -30 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
for v in 1 0 1 0; do
  env $AB_VAR=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-pcie > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); st=d['detail']['stages_ms_total']; print('$AB_VAR=$v', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k, v in st.items()})"
done
