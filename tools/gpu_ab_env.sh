#!/bin/bash
# A/B of a diagnostic environment switch: bench (no locate) with and without AB_ENV set.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 0 1; do
  if [ $v = 1 ]; then export $AB_ENV=1; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --patterns 0 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/ab_$v.json')); s=d['detail']['stages_ms_total']
print('$AB_ENV=$v', d['ms_per_step'], {k: round(v['ms']/v['launches'],3) for k,v in s.items() if v['launches']<=10})"
done
