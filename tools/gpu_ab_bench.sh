#!/bin/bash
# 1 GiB bench only, env toggle on / off twice (AB_VAR=NAME): step and the three big passes.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
for v in 1 0 1 0; do
  env $AB_VAR=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-pcie > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); st=d['detail']['stages_ms_total']; print('$AB_VAR=$v', d['ms_per_step'], {k: round(st[k]['ms']/d['steps'],3) for k in ('sa_bucket_hist','radix_part_text','radix_part','sa_bucket_sort')})"
done
