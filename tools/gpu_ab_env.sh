#!/bin/bash
# Parity (everything but the sharded cases unless K is set), then the 1 GiB bench with an env toggle
# on / off twice: AB_VAR=NAME.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_bucket.py tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 160 --timeout-method thread -k "${K:-not shard}" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for v in 1 0 1 0; do
  env $AB_VAR=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-legs --no-cpu-baseline --no-pcie > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); st=d['detail']['stages_ms_total']; print('$AB_VAR=$v', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k, v in st.items() if not k.startswith('radix_part') and k not in ('sa_bucket_sort','byte_hist')})"
done
