#!/bin/bash
# A/B of bench.py (1 GiB sigma=4, SA+BWT steps) under environment variants: each argument is one
# variant ("VAR=1 VAR2=x" or "-" for none).  TESTS=1 runs the GPU suite first; TRACE=1 adds the
# bucket-sort phase stamps of each variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || { tail -40 gpurun_out/gputest.log; exit 1; }
  tail -2 gpurun_out/gputest.log
fi
i=0
for v in "$@"; do
  i=$((i+1))
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline ${BARGS} --no-pcie > gpurun_out/abv_$i.json 2> gpurun_out/abv_$i.err || { echo "variant $i failed"; tail gpurun_out/abv_$i.err; exit 1; }
  python3 - "$v" gpurun_out/abv_$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); r = d['roofline']
st = {k: v['ms'] / v['launches'] for k, v in d['detail']['stages_ms_total'].items()}
print(f"[{sys.argv[1] or 'default'}] {d['ms_per_step']} ms/step", {k: round(v, 3) for k, v in st.items() if v > 0.2},
      "wt", d['detail']['wt_build_ms'], "loc/s", d['locate_patterns_per_s'])
PY
  if [ -n "$TRACE" ]; then
    env $v HKCSA_BS_TRACE=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-legs --no-cpu-baseline --patterns 0 ${BARGS} 2>&1 >/dev/null | grep trace
  fi
done
