#!/bin/bash
# Sharded parity tests, then the strong 4 GiB line with an env toggle (AB_VAR) on / off.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
( while sleep 60; do date >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_gpu_dropin.py -m gpu -x -q --timeout ${PT:-200} --timeout-method thread -k "${K:-shard or strong or weak or replic}" > gpurun_out/sl_tests.log 2>&1 || { tail -30 gpurun_out/sl_tests.log; exit 1; }
tail -2 gpurun_out/sl_tests.log
for v in ${AB_VALS:-1 0}; do
  env $AB_VAR=$v timeout -k 10 400 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-legs --no-eps --no-pcie > gpurun_out/strong_$v.json 2> gpurun_out/strong_$v.err || { tail -5 gpurun_out/strong_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/strong_$v.json').read().strip().splitlines()[-1]); st=d['detail']['stages_ms_total']; print('$AB_VAR=$v', d['ms_per_step'], {k: round(v['ms']/d['steps'],3) for k, v in st.items()})"
done
