#!/bin/bash
# A/B of pass modes on one box: HKCSA_PASS_MODE 0 (tables), 3 (lookback both), 2 (table A, lookback B)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in ${MODES:-0 3 2 0 3}; do
  HKCSA_PASS_MODE=$m timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --patterns 0 > gpurun_out/ab_$m.json 2> gpurun_out/ab_$m.err || exit $?
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab_$m.json').read());st=d['detail']['stages_ms_total']
print('mode $m', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k,v in st.items() if v['ms']/d['steps'] > 0.5})"
done
